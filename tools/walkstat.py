#!/usr/bin/env python3
"""Load coherence of the child-pair walk, per bounce (experiment build: tools/build_variant.sh secprof
-DPT_SECPROF, run with PT_LIBPT=build_variants/secprof/libpt.so): for one 1 spp frame of each workload,
the walk loop's wave iterations, the iterations that issue the four record loads, how many of those
load one record for every loading lane (a wave-uniform fetch), the loading lanes per such load, and
the share of loading lanes that load the first loading lane's record. Counted by WalkStat
(pt_device.h); the instrumentation slows the kernel, so only the counts are meaningful."""
import ctypes
import json
import os
import sys

import numpy as np

os.environ.setdefault("PT_WALKSTAT", "1")   # the SECPROF build's walk statistics are opt-in (pt_capi.cpp)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

fn = bp.lib().pt_debug_walk_stats
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
for wl in (sys.argv[1:] or ["dragon", "bunny", "helmet", "sky_dragon"]):
    meta, mesh_arrays, maps, (W, Hh) = H.workload(wl)
    e = bp.Engine(0)
    mesh = H.texture_payloads(meta, mesh_arrays) if mesh_arrays is not None else None
    p = bp.StreamPlayer(e, meta, H.bluenoise(), mesh, W, Hh)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            p.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
    e.resize_canvas(p.width, p.height)
    buf = np.zeros(40, np.uint64)
    for k in range(4):
        for call in p.synth_frame(k):
            p.play_call(call)
        e.sync()
        fn(buf.ctypes.data)          # read and reset: the last frame's counts remain
    st = buf.reshape(8, 5).astype(np.int64)
    rows = []
    for b in range(8):
        it, ld, un, ln, fi = (int(v) for v in st[b])
        if it == 0:
            continue
        rows.append({"bounce": b, "wave_iters": it, "wave_loads": ld, "uniform_loads": un,
                     "uniform_share": round(un / max(1, ld), 4), "lanes_per_load": round(ln / max(1, ld), 2),
                     "first_record_share": round(fi / max(1, ln), 4), "loading_lanes": ln})
    tot = st.sum(0)
    print(json.dumps({"workload": wl, "size": [p.width, p.height], "wave_iters": int(tot[0]), "wave_loads": int(tot[1]),
                      "uniform_share": round(int(tot[2]) / max(1, int(tot[1])), 4),
                      "lanes_per_load": round(int(tot[3]) / max(1, int(tot[1])), 2),
                      "first_record_share": round(int(tot[4]) / max(1, int(tot[3])), 4), "per_bounce": rows}), flush=True)
    e.dispose()
