#!/usr/bin/env python3
"""The fp32 tolerance study (TEST INFRASTRUCTURE, CPU only): how far a render moves when
only the GLSL built-ins' rounding changes, within what GLSL ES 3.00 allows a GL driver.

The parity bar of this repo is bit-exactness against the pinned restatement (oracle/libptoracle.so:
one IEEE op per GLSL op, pinned transcendental sequences). A browser's GL driver is free to use other
built-ins. The same oracle, compiled under other legal built-in sets (oracle/Makefile):
  fma   FMA contraction allowed (GLSL lets the compiler fuse a*b+c);
  libm  + the C library's transcendentals (glibc exp2f / log2f / expf / logf / powf / sinf / cosf /
        atanf / atan2f / acosf) in place of the pinned sequences;
  gpu   + normalize as v * rsq(dot(v, v)) with the reciprocal square root within 1 ulp (rounded toward
        zero), as a GPU driver compiles it.
For each recorded stream (the nine the transcription check covers) and the dragon stand-in, frames
1..N (fresh uRandomVec2 per frame, camera still, history cleared at frame 1) are rendered by every
build in lockstep. Per build against the pinned one: the share of pixels whose per-frame sample
differs in any bit, the share whose path was re-routed (a channel differs by more than 1e-3 relative:
a flipped `rand() < P` or a different hit, SURVEY §7 hard part 1), and the RMSE of the progressive
estimate accumulation / k at k = 1, 64, 1024, next to the pinned build's own Monte Carlo standard
error at k (the per-pixel sample standard deviation / sqrt(k), RMS over pixels).

usage: tolerance.py [--frames 1024] [--out tests/golden/tolerance.json] [names...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "tests", os.path.join("babylon.js-pathtracing-renderer_amd", "python")):
    sys.path.insert(0, os.path.join(ROOT, p))

import helpers as H      # noqa: E402
import ptoracle as po    # noqa: E402
import babylon_pt as bp  # noqa: E402  (uniform synthesis only: no device call)

# name -> (recorded stream, mesh kind, helmet maps?, size)
CASES = {
    "cornell_256": ("cornell_256", None, False, (64, 64)),
    "sky_256": ("sky_256", None, False, (64, 64)),
    "quadric_256": ("quadric_256", None, False, (64, 64)),
    "gltf_teapot": ("gltf_teapot_320x180", "own", False, (96, 54)),
    "gltf_duck": ("gltf_duck_320x180", "own", False, (96, 54)),
    "gltf_helmet": ("gltf_helmet_320x180", "own", True, (96, 54)),
    "gltf_bunny": ("gltf_bunny_1080p", "own", False, (96, 54)),
    "hdri_teapot": ("hdri_teapot_320x180", "own", False, (96, 54)),
    "hdri_helmet": ("hdri_helmet_320x180", "own", True, (96, 54)),
    "dragon_standin": ("gltf_bunny_1080p", "dragon", False, (96, 54)),
}
CHECKPOINTS = (1, 64, 1024)
REROUTE_REL = 1e-3


def toolchain():
    """What the fma / libm / gpu builds' bits depend on besides the source: the C compiler (how
    -ffp-contract=fast fuses), the C library (its expf / sinf / atan2f / powf ...) and the ISA (-mfma)."""
    import platform
    import subprocess
    try:
        gcc = subprocess.run(["gcc", "-dumpfullversion"], capture_output=True, text=True, timeout=30).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        gcc = None
    try:
        libc = os.confstr("CS_GNU_LIBC_VERSION")
    except (ValueError, OSError):
        libc = None
    return {"gcc": gcc, "libc": libc, "machine": platform.machine()}


def frame_uniforms(meta, k, W, Hh, seed=12345):
    """Frame k (1-based) of a still-camera progressive run from a cleared history: the last recorded
    frame's uniforms with uFrameCounter = uSampleCounter = k and a fresh uRandomVec2."""
    u = dict(H.with_resolution(H.path_call(meta["frames"][-1])["uniforms"], W, Hh))
    u["uFrameCounter"] = ["f", [float(k)]]
    u["uSampleCounter"] = ["f", [float(k)]]
    u["uCameraIsMoving"] = ["i", [0]]
    u["uRandomVec2"] = ["f", bp.splitmix64_uniforms(seed * 1000003 + k, 2)]
    return u


def run_case(name, frames, variants):
    key, mesh_kind, maps_on, (W, Hh) = CASES[name]
    meta = H.stream(key)
    m = H.synthetic_dragon() if mesh_kind == "dragon" else H.mesh(meta) if mesh_kind else None
    maps = H.helmet_maps() if maps_on else None
    builds = [""] + list(variants)
    scenes = {}
    for v in builds:
        if m is not None:
            hdr = H.synthetic_hdr() if meta["scene"] == "hdri" else None
            scenes[v] = po.Scene(meta["scene"], W, Hh, H.bluenoise(), m["bvh"], m["tri"], hdr, maps, variant=v)
        else:
            scenes[v] = po.Scene(meta["scene"], W, Hh, H.bluenoise(), variant=v)
    zeros = np.zeros((Hh, W, 4), np.float32)
    acc = {v: np.zeros((Hh, W, 3), np.float32) for v in builds}
    s1 = np.zeros((Hh, W, 3), np.float64)   # pinned samples: running sums for the Monte Carlo error
    s2 = np.zeros((Hh, W, 3), np.float64)
    stats = {v: {"bit": [], "rerouted": []} for v in variants}
    out = {v: {} for v in variants}
    mc = {}
    t0 = time.perf_counter()
    for k in range(1, frames + 1):
        u = frame_uniforms(meta, k, W, Hh)
        samp = {}
        for v in builds:
            o, _ = scenes[v].path_trace(u, zeros)
            samp[v] = o[..., :3]
            # the shader's accumulation (camera still): prev + sample, in binary32; frame 1 clears
            acc[v] = samp[v].copy() if k == 1 else (acc[v] + samp[v]).astype(np.float32)
        ref = samp[""]
        s1 += ref
        s2 += ref.astype(np.float64) ** 2
        for v in variants:
            d = samp[v] != ref
            stats[v]["bit"].append(float(d.any(-1).mean()))
            rel = np.abs(samp[v].astype(np.float64) - ref) > REROUTE_REL * np.maximum(1.0, np.abs(ref.astype(np.float64)))
            stats[v]["rerouted"].append(float(rel.any(-1).mean()))
        if k in CHECKPOINTS:
            est_ref = acc[""].astype(np.float64) / k
            mean = float(est_ref.mean())
            var = np.maximum(s2 / k - (s1 / k) ** 2, 0.0) * (k / max(1, k - 1))
            mc[str(k)] = float(np.sqrt((var / k).mean())) if k > 1 else None
            for v in variants:
                e = acc[v].astype(np.float64) / k - est_ref
                rmse = float(np.sqrt((e ** 2).mean()))
                out[v][str(k)] = {"rmse": rmse, "rel_rmse": rmse / mean if mean else None,
                                  "max_abs": float(np.abs(e).max()), "mean_radiance": mean}
    res = {"stream": key, "scene": meta["scene"], "width": W, "height": Hh, "frames": frames,
           "mesh": mesh_kind, "maps": maps_on, "seconds": round(time.perf_counter() - t0, 1),
           "mc_standard_error_rms": mc, "variants": {}}
    for v in variants:
        b, r = np.array(stats[v]["bit"]), np.array(stats[v]["rerouted"])
        res["variants"][v] = {"bit_divergent_frac_mean": float(b.mean()), "bit_divergent_frac_frame1": float(b[0]),
                              "rerouted_frac_mean": float(r.mean()), "rerouted_frac_max": float(r.max()),
                              "estimate": out[v]}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--variants", default="fma,libm,gpu")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "tolerance.json"))
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    names = a.names or list(CASES)
    report = {"frames": a.frames, "checkpoints": [k for k in CHECKPOINTS if k <= a.frames],
              "reroute_rel": REROUTE_REL, "variants": a.variants.split(","), "toolchain": toolchain(), "cases": {}}
    if os.path.exists(a.out) and a.names:
        with open(a.out) as f:
            report["cases"] = json.load(f).get("cases", {})
    for n in names:
        report["cases"][n] = run_case(n, a.frames, a.variants.split(","))
        print(json.dumps({n: report["cases"][n]["variants"], "seconds": report["cases"][n]["seconds"]}), flush=True)
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
