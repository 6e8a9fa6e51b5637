#!/usr/bin/env python3
"""oracle/xcheck/run_xcheck.py — TEST INFRASTRUCTURE (build container only: needs /root/reference).

Builds the mechanical transcriptions of the reference's fragment shaders (transcribe.py ->
oracle/_ref/xcheck_<scene>.cpp -> oracle/_ref/libxcheck_<scene>.so), replays the committed
uniform streams through them, compares every frame with the C oracle (oracle/ptoracle.c) fed the
same previousBuffer, and writes
  tests/golden/xcheck/<stream>_<W>x<H>.npz   the transcription's accumulation after each frame
                                             (data: the fixtures tests/test_xcheck.py pins the
                                             oracle to, on hosts without /root/reference)
  tests/golden/xcheck/report.json            per stream: pixels compared, pixels whose RGBA32F
                                             bits differ, max |difference|, RMSE

usage: run_xcheck.py [stream ...]   (default: every recorded stream of a reference shader)
       run_xcheck.py --build          (only transcribe and compile every scene into oracle/_ref/)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_OUT = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden", "xcheck")
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))   # pt_assets (JPEG maps)
import helpers as H  # noqa: E402

# stream -> (width, height, frames, PBR maps): small sizes the scalar transcription runs in seconds
STREAMS = {
    "cornell_256": (64, 64, 3, None),
    "sky_256": (64, 64, 3, None),
    "quadric_256": (64, 64, 3, None),
    "gltf_teapot_320x180": (96, 54, 3, None),
    "gltf_duck_320x180": (96, 54, 3, None),
    "gltf_helmet_320x180": (96, 54, 3, "helmet"),
    "gltf_bunny_1080p": (96, 54, 3, None),
    "hdri_teapot_320x180": (96, 54, 3, None),
    "hdri_helmet_320x180": (96, 54, 3, "helmet"),
}
SAMPLER_KEYS = {"bvh": "tAABBTexture", "tri": "tTriangleTexture"}
MAP_SAMPLERS = {"albedo": "tAlbedoTexture", "bump": "tBumpTexture", "metallic": "tMetallicTexture",
                "emissive": "tEmissiveTexture"}
CXXFLAGS = ["-std=c++20", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-pthread"]


def build(scene):
    os.makedirs(REF_OUT, exist_ok=True)
    cpp = os.path.join(REF_OUT, "xcheck_%s.cpp" % scene)
    so = os.path.join(REF_OUT, "libxcheck_%s.so" % scene)
    rep = subprocess.run([sys.executable, os.path.join(HERE, "transcribe.py"), scene, cpp], check=True,
                         capture_output=True, text=True).stdout
    subprocess.run(["g++"] + CXXFLAGS + ["-I" + HERE, "-o", so, cpp], check=True)
    lib = ctypes.CDLL(so)
    lib.xc_set_uniform.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int]
    lib.xc_set_sampler.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.xc_render.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    return lib, [l for l in rep.splitlines() if l.startswith("ORDER-CHECK")]


class XScene:
    """The transcription with one stream's textures bound (kept alive here)."""

    def __init__(self, lib, meta, w, h, maps):
        self.lib, self.w, self.h = lib, w, h
        self.keep = []
        self.sampler("blueNoiseTexture", H.bluenoise(), 0)
        if meta["scene"] in ("gltf", "hdri"):
            pay = H.texture_payloads(meta, H.mesh(meta))
            for k, name in SAMPLER_KEYS.items():
                self.sampler(name, pay[k].reshape(2048, 2048, 4), 1)
            if meta["scene"] == "hdri":   # uploaded with invertY: GL rows are the payload's reversed
                self.sampler("tHDRTexture", pay["hdr"][::-1], 1)
        for k, m in (maps or {}).items():
            self.sampler(MAP_SAMPLERS[k], m, 0)

    def sampler(self, name, arr, f32):
        a = np.ascontiguousarray(arr, dtype=np.float32 if f32 else np.uint8)
        self.keep.append(a)
        rc = self.lib.xc_set_sampler(name.encode(), a.ctypes.data, a.shape[1], a.shape[0], f32)
        if rc < 0:
            raise RuntimeError(name)

    def frame(self, uniforms, prev):
        for name, (kind, vals) in uniforms.items():
            v = np.asarray(vals, dtype=np.float32)
            if self.lib.xc_set_uniform(name.encode(), v.ctypes.data, v.size) < 0:
                raise RuntimeError("uniform %s" % name)
        prev = np.ascontiguousarray(prev, dtype=np.float32)
        self.sampler("previousBuffer", prev, 1)
        out = np.zeros((self.h, self.w, 4), np.float32)
        self.lib.xc_render(self.w, self.h, out.ctypes.data, max(1, (os.cpu_count() or 4) // 4))
        return out


def compare(ref, got):
    ra, ga = ref.view(np.uint32), got.view(np.uint32)
    diff = (ra != ga).any(-1)
    d = np.abs(ref.astype(np.float64) - got.astype(np.float64))
    return {"pixels": int(diff.size), "pixels_differing": int(diff.sum()),
            "max_abs": float(np.nanmax(d)) if d.size else 0.0,
            "rmse": float(np.sqrt(np.nanmean(d[..., :3] ** 2)))}


def quantize(c):
    """the canvas store of a [0,1] colour: u8 = floor(255 c + 0.5) in binary32"""
    c = np.asarray(c, np.float32)
    return np.floor(c * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


# screenOutput at the sample counts either side of its two bypass thresholds
# (js/PathTracingCommon.js:293: 1/N < 0.005 for sharp pixels, 1/N < 0.0002 for all)
OUTPUT_STREAMS = ["cornell_256", "gltf_bunny_1080p", "hdri_helmet_320x180"]
OUTPUT_N = [1, 2, 200, 201, 4999, 5001]


def run_output():
    """screenCopy and screenOutput transcribed, on the oracle's accumulation of each stream."""
    out_lib, _ = build("screen_output")
    copy_lib, _ = build("screen_copy")
    rpath = os.path.join(GOLD, "report.json")
    report = json.load(open(rpath))
    for name in OUTPUT_STREAMS:
        w, h, frames, maps_kind = STREAMS[name]
        meta = H.stream(name)
        maps = H.helmet_maps() if maps_kind == "helmet" else None
        accs, _, _ = H.oracle_replay(meta, frames, width=w, height=h, maps=maps)
        acc = np.ascontiguousarray(accs[-1])
        exposure = H.output_call(meta["frames"][frames - 1])["uniforms"].get("uToneMappingExposure", ["f", [1.0]])[1][0]
        res, outs = {}, {"acc": acc}
        for n in OUTPUT_N:
            inv = np.float32(1.0 / n)
            for lib, uni in ((out_lib, {"uOneOverSampleCounter": inv, "uToneMappingExposure": np.float32(exposure)}),):
                for k, v in uni.items():
                    vv = np.asarray([v], np.float32)
                    lib.xc_set_uniform(k.encode(), vv.ctypes.data, 1)
                lib.xc_set_sampler(b"accumulationBuffer", acc.ctypes.data, w, h, 1)
                got = np.zeros((h, w, 4), np.float32)
                lib.xc_render(w, h, got.ctypes.data, max(1, (os.cpu_count() or 4) // 4))
            outs["out_%d" % n] = got
            want = H.po_screen_output(acc, float(inv), exposure)
            res[str(n)] = int((quantize(got) != want).any(-1).sum())
        copy_lib.xc_set_sampler(b"pathTracedImageBuffer", acc.ctypes.data, w, h, 1)
        cp = np.zeros((h, w, 4), np.float32)
        copy_lib.xc_render(w, h, cp.ctypes.data, 1)
        res["copy"] = int((cp.view(np.uint32) != acc.view(np.uint32)).any(-1).sum())
        np.savez_compressed(os.path.join(GOLD, "screen_output_%s_%dx%d.npz" % (name, w, h)), **outs)
        report.setdefault("_screen_output", {})[name] = {"width": w, "height": h, "exposure": exposure,
                                                        "pixels": w * h, "pixels_differing_by_N": res}
        print("screenOutput", name, res, flush=True)
    with open(rpath, "w") as f:
        json.dump(report, f, indent=1, sort_keys=True)


def run(names):
    os.makedirs(GOLD, exist_ok=True)
    rpath = os.path.join(GOLD, "report.json")
    report = json.load(open(rpath)) if os.path.exists(rpath) else {}
    libs = {}
    for name in names:
        w, h, frames, maps_kind = STREAMS[name]
        meta = H.stream(name)
        scene = meta["scene"]
        if scene not in libs:
            libs[scene] = build(scene)
        lib, order = libs[scene]
        maps = H.helmet_maps() if maps_kind == "helmet" else None
        ref_accs, _, _ = H.oracle_replay(meta, frames, width=w, height=h, maps=maps)
        xs = XScene(lib, meta, w, h, maps)
        prev = np.zeros((h, w, 4), np.float32)
        outs, per_frame = {}, []
        for k, f in enumerate(meta["frames"][:frames]):
            u = H.with_resolution(H.path_call(f)["uniforms"], w, h)
            got = xs.frame(u, prev)
            outs["acc%d" % k] = got
            per_frame.append(compare(ref_accs[k], got))
            prev = ref_accs[k]   # both sides see the oracle's history: each frame is checked alone
        np.savez_compressed(os.path.join(GOLD, "%s_%dx%d.npz" % (name, w, h)), **outs)
        report[name] = {"width": w, "height": h, "frames": frames, "maps": maps_kind, "scene": scene,
                        "order_checks": order, "per_frame": per_frame}
        print(name, json.dumps(per_frame), flush=True)
    with open(rpath, "w") as f:
        json.dump(report, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["--build"]:
        for sc in sorted({H.stream(n)["scene"] for n in STREAMS}) + ["screen_copy", "screen_output"]:
            build(sc)
            print("built oracle/_ref/libxcheck_%s.so" % sc)
    elif sys.argv[1:] == ["--output"]:
        run_output()
    else:
        run(sys.argv[1:] or list(STREAMS))
        if not sys.argv[1:]:
            run_output()
