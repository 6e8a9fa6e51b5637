#!/usr/bin/env python3
"""Minimal profiling driver: K frames of a bench workload (or of a recorded stream) through libpt,
no counting kernels, no CPU work — the program under rocprofv3 --pmc / --kernel-trace (tools/gpu_pmc.sh,
and bench.py's live HBM-traffic passes). Never imports torch."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default=None, choices=sorted(H.WORKLOADS), help="a bench.py workload")
ap.add_argument("--stream", default="gltf_bunny_1080p")
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--dragon", action="store_true", help="the StanfordDragon stand-in mesh instead of the stream's")
ap.add_argument("--parts", type=int, default=1, help="draw only rank --part's bands of a --parts-way row partition")
ap.add_argument("--part", type=int, default=0)
a = ap.parse_args()
maps = None
if a.workload:
    meta, mesh_arrays, maps, (W, Hh) = H.workload(a.workload)
    a.width, a.height = a.width or W, a.height or Hh
else:
    meta = H.stream(a.stream)
    mesh_arrays = H.synthetic_dragon() if a.dragon else (H.mesh(meta) if meta["scene"] in ("gltf", "hdri") else None)
e = bp.Engine(0)
mesh = H.texture_payloads(meta, mesh_arrays) if mesh_arrays is not None else None
p = bp.StreamPlayer(e, meta, H.bluenoise(), mesh, a.width or None, a.height or None)
if maps:
    for kind, sampler in H.PBR_SAMPLERS.items():
        p.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
e.resize_canvas(p.width, p.height)
if a.parts > 1:   # one rank's share of an N-GPU frame, as bench.py's rank_share_4k draws it
    e.set_row_partition(a.parts, a.part)
    e.set_output_partition(True)
for k in range(a.frames):
    for call in p.synth_frame(k):
        p.play_call(call)
e.sync()
print("ok", a.workload or a.stream, a.frames)
if os.environ.get("PT_QSTATS"):
    print("queue stats:", e.queue_stats())
