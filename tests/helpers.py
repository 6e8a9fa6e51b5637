"""Shared loaders for the golden fixtures and oracle replays (test infrastructure)."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def stream(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def bluenoise():
    return np.load(os.path.join(GOLD, "bluenoise_rgba8.npy"))


def mesh(meta_or_key):
    key = meta_or_key if isinstance(meta_or_key, str) else meta_or_key["mesh"][len("mesh_"):-len(".npz")]
    m = np.load(os.path.join(GOLD, "mesh_%s.npz" % key))
    return {"bvh": m["bvh"], "tri": m["tri"]}


def texture_payloads(meta, m):
    """The two 2048x2048 RGBA32F arrays exactly as the setup script uploads them (zero tail)."""
    out = {}
    for kind in ("bvh", "tri"):
        full = np.zeros(2048 * 2048 * 4, np.float32)
        flat = m[kind].reshape(-1)
        full[:flat.size] = flat
        out[kind] = full
    return out


def path_call(frame):
    return next(c for c in frame if c["shader"] == "pathTracingFragmentShader")


def output_call(frame):
    return next(c for c in frame if c["shader"] == "screenOutputFragmentShader")


def oracle_scene(meta, width=None, height=None, mesh_arrays=None):
    import ptoracle as po
    w, h = width or meta["width"], height or meta["height"]
    if meta["scene"] == "gltf":
        m = mesh_arrays if mesh_arrays is not None else mesh(meta)
        return po.Scene("gltf", w, h, bluenoise(), m["bvh"], m["tri"])
    return po.Scene(meta["scene"], w, h, bluenoise())


def with_resolution(uniforms, w, h):
    """The uniforms a setup script pushes after resizing to w x h (handleWindowResize +
    onApply, js/GLTF_Model_Path_Tracing.js:521-537, 815-816): uResolution and uULen = uVLen*w/h."""
    u = dict(uniforms)
    if [float(w), float(h)] != [float(v) for v in u["uResolution"][1]]:
        u["uResolution"] = ["f", [float(w), float(h)]]
        u["uULen"] = ["f", [u["uVLen"][1][0] * (w / h)]]
    return u


def oracle_replay(meta, frames=None, width=None, height=None, nthreads=0, with_output=False, mesh=None):
    """Run the oracle over the recorded stream: returns accumulation after each frame (+ canvas)."""
    import ptoracle as po
    w, h = width or meta["width"], height or meta["height"]
    sc = oracle_scene(meta, w, h, mesh)
    acc = np.zeros((h, w, 4), np.float32)
    accs, canvases, counters = [], [], []
    for f in meta["frames"][:frames]:
        u = with_resolution(path_call(f)["uniforms"], w, h)
        acc, cnt = sc.path_trace(u, acc, nthreads=nthreads)
        accs.append(acc.copy())
        counters.append(cnt)
        if with_output:
            ou = output_call(f)["uniforms"]
            exp = ou.get("uToneMappingExposure", ["f", [0.0]])[1][0]
            canvases.append(po.screen_output(acc, ou["uOneOverSampleCounter"][1][0], exp))
    return accs, canvases, counters
