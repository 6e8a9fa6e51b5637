#!/usr/bin/env python3
"""Section profile of the megakernel (experiment build: tools/build_variant.sh secprof -DPT_SECPROF,
run with PT_LIBPT=build_variants/secprof/libpt.so): per workload, the share of wave clock spent in
camera ray / analytic intersection / BVH walk / hit attributes / shading / epilogue, charged once
per wave (divergent code counts once). The counting pass carries the marks; never bit-checked."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

NAMES = ["camera", "analytic", "walk", "attributes", "shade+epilogue", "max_wave", "waves", "total"]
for wl in (sys.argv[1:] or ["helmet", "bunny", "dragon", "sky_dragon"]):
    meta, mesh_arrays, maps, (W, Hh) = H.workload(wl)
    e = bp.Engine(0)
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
    e.sync()
    e.timing_begin()
    for k in range(1):
        for call in p.synth_frame(3 + k):
            p.play_call(call)
    ms, _ = e.timing_end(meta["scene"])
    c = e.counters()
    e.dispose()
    vals = [int(v) for v in (c.values() if isinstance(c, dict) else c)]
    tot = max(1, vals[7])
    print(json.dumps({"workload": wl, "waves": vals[6], "cycles_per_wave": vals[7] / max(1, vals[6]),
                      "max_wave_cycles": vals[5], "kernel_ms": ms,
                      "share": {NAMES[i]: round(vals[i] / tot, 4) for i in (0, 1, 2, 3, 4)}}), flush=True)
    e2 = None
