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
    """The RGBA32F arrays exactly as the setup script uploads them: the two 2048x2048 mesh textures
    (zero tail) and, for the HDRI scene, the environment (synthetic_hdr)."""
    out = {}
    for kind in ("bvh", "tri"):
        full = np.zeros(2048 * 2048 * 4, np.float32)
        flat = m[kind].reshape(-1)
        full[:flat.size] = flat
        out[kind] = full
    if meta["scene"] == "hdri":
        out["hdr"] = synthetic_hdr()
    return out


def path_call(frame):
    return next(c for c in frame if c["shader"] == "pathTracingFragmentShader")


def output_call(frame):
    return next(c for c in frame if c["shader"] == "screenOutputFragmentShader")


def oracle_scene(meta, width=None, height=None, mesh_arrays=None):
    import ptoracle as po
    w, h = width or meta["width"], height or meta["height"]
    if meta["scene"] in ("gltf", "hdri"):
        m = mesh_arrays if mesh_arrays is not None else mesh(meta)
        hdr = synthetic_hdr() if meta["scene"] == "hdri" else None
        return po.Scene(meta["scene"], w, h, bluenoise(), m["bvh"], m["tri"], hdr)
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


HDR_W, HDR_H, SUN_X, SUN_Y = 2048, 1024, 1536, 300


def synthetic_hdr():
    """The synthetic equirect environment the fixture generator hands to the HDRI setup script in
    place of its missing .hdr files (tests/golden/gen/browser_env.js syntheticHDR): (1024, 2048, 4)
    float32 in the order the script passes it to RawTexture.CreateRGBATexture (invertY = true).
    Every value is a short dyadic rational, so both generators produce the same bits."""
    i = np.arange(HDR_W * HDR_H, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x85EBCA77)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    n = (h & np.uint64(255)).astype(np.float64).reshape(HDR_H, HDR_W) / 4096.0
    y = np.arange(HDR_H, dtype=np.float64)[:, None]
    t = (HDR_H / 2 - y) / 2048.0
    sky = y < HDR_H / 2
    out = np.ones((HDR_H, HDR_W, 4), np.float64)
    out[..., 0] = np.where(sky, 0.25 + t + n, 0.125 + n)
    out[..., 1] = np.where(sky, 0.375 + t + n, 0.1875 + n)
    out[..., 2] = np.where(sky, 0.75 + 2 * t + n, 0.0625 + n)
    out[SUN_Y - 2:SUN_Y + 3, SUN_X - 2:SUN_X + 3, :3] = 512.0
    out[SUN_Y, SUN_X, :3] = 4096.0
    return out.astype(np.float32)
