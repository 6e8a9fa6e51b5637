#!/usr/bin/env python3
"""Render K progressive frames of a bench workload through the C ABI and save the displayed canvas
(screenOutput: 5x5 denoise, 1/N, Reinhard, gamma) as a PNG - a visual check of the converged image
(BASELINE configs[4]-style: many samples + the output filter). Prints Mpaths/s over the run.

usage: render_png.py [--workload dragon|bunny|helmet] [--size WxH] [--frames K] --out PATH"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", choices=("dragon", "bunny", "helmet"), default="dragon")
ap.add_argument("--size", default="1920x1080")
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--out", required=True)
a = ap.parse_args()
W, Hh = (int(v) for v in a.size.lower().split("x"))
meta = H.stream("hdri_helmet_320x180" if a.workload == "helmet" else "gltf_bunny_1080p")
mesh = H.synthetic_dragon() if a.workload == "dragon" else H.mesh(meta)
e = bp.Engine(0)
p = bp.StreamPlayer(e, meta, H.bluenoise(), H.texture_payloads(meta, mesh), W, Hh)
if a.workload == "helmet":
    maps = H.synthetic_pbr_maps(2048)
    for kind, sampler in H.PBR_SAMPLERS.items():
        p.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
e.resize_canvas(W, Hh)
for call in p.meta["frames"][0]:
    p.play_call(call)
e.sync()
t0 = time.perf_counter()
for k in range(a.frames):
    for call in p.synth_frame(k):
        p.play_call(call)
e.sync()
dt = time.perf_counter() - t0
img = e.read_canvas(W, Hh)[::-1, :, :3]          # GL rows bottom-up -> image rows top-down
from PIL import Image                             # noqa: E402
Image.fromarray(np.ascontiguousarray(img)).save(a.out)
print("%s %dx%d %d frames: %.1f Mpaths/s, mean %.1f, saved %s" % (a.workload, W, Hh, a.frames,
      W * Hh * a.frames / dt / 1e6, img.mean(), a.out))
