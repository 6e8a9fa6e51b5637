#!/usr/bin/env python3
"""Minimal profiling driver: K frames of a recorded stream (default: the bench workload, StanfordBunny
1920x1080) through libpt, no counting kernels, no CPU work — for rocprofv3 --pmc / --kernel-trace."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--stream", default="gltf_bunny_1080p")
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--dragon", action="store_true", help="the StanfordDragon stand-in mesh instead of the stream's")
a = ap.parse_args()
meta = H.stream(a.stream)
e = bp.Engine(0)
mesh = H.texture_payloads(meta, H.synthetic_dragon() if a.dragon else H.mesh(meta)) if meta["scene"] in ("gltf", "hdri") else None
p = bp.StreamPlayer(e, meta, H.bluenoise(), mesh, a.width or None, a.height or None)
for k in range(a.frames):
    for call in p.synth_frame(k):
        p.play_call(call)
e.sync()
print("ok", a.stream, a.frames)
if os.environ.get("PT_QSTATS"):
    print("queue stats:", e.queue_stats())
