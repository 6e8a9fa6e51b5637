#!/usr/bin/env python3
"""BVH stack traffic of the megakernel (experiment build: tools/build_variant.sh secprof "-DPT_SECPROF -DPT_SECPROF_LOADS",
run with PT_LIBPT=build_variants/secprof/libpt.so): per workload and launch, the stack pops and
pushes of every walk and how many of them fall beyond the LDS levels into the global slab (each
such access is a vector-memory instruction of its wave), next to the reference-priced node fetches
and leaf tests. The counting pass carries the counts; never bit-checked."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

NAMES = ["wave_record_loads", "uniform_wave_record_loads", "lanes_at_record_loads", "pops_slab", "node_fetches", "leaf_tests", "paths"]
for wl in (sys.argv[1:] or ["helmet", "bunny", "dragon", "sky_dragon"]):
    meta, mesh_arrays, maps, (W, Hh) = H.workload(wl)
    e = bp.Engine(0)
    e.set_bvh_layout(os.environ.get("PT_BVH", "pairs"))   # trail: pops_slab counts the walk's restarts
    mesh = H.texture_payloads(meta, mesh_arrays) if mesh_arrays is not None else None
    p = bp.StreamPlayer(e, meta, H.bluenoise(), mesh, W, Hh)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            p.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
    e.resize_canvas(p.width, p.height)
    for k in range(3):
        for call in p.synth_frame(k):
            p.play_call(call)
    e.set_counting(True)
    e.reset_counters()
    for call in p.synth_frame(3):
        p.play_call(call)
    vals = [int(v) for v in e.counters().values()]
    e.dispose()
    d = dict(zip(NAMES, vals))
    d["workload"] = wl
    d["lanes_per_wave_load"] = round(vals[2] / max(1, vals[0]), 2)
    d["uniform_share"] = round(vals[1] / max(1, vals[0]), 4)
    print(json.dumps(d), flush=True)
