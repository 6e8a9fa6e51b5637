#!/usr/bin/env python3
"""Wave timeline of the production megakernel (experiment build: tools/build_variant.sh secprof
-DPT_SECPROF, run with PT_LIBPT=build_variants/secprof/libpt.so): every workgroup (one wave)
stores its (start, end) wall clock (100 MHz) and its section cycle sums (PT_SEC marks: 0 camera ray,
1 analytic objects, 2 BVH walk, 3 hit attributes, 4 shading) and the CU it ran on (__smid). Per workload:
the launch span, the longest wave and when it started, wave-duration percentiles, how much of the span
the last 1 % of waves cover, and the CU occupancy over the span: the share of the launch during which
fewer than half (and fewer than 90 %) of the CUs hold a wave - the tail that overlapping the next
frame's path tracing can fill.
A longest wave close to the span means the launch is bound by its slowest wave, not by throughput."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

SEC = ["camera", "analytic", "walk", "hit_attr", "shade"]
fn = bp.lib().pt_debug_wave_log
fn.restype = ctypes.c_size_t
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
out_dir = sys.argv[1]
for wl in (sys.argv[2:] or ["helmet", "bunny", "dragon", "sky_dragon"]):
    meta, mesh_arrays, maps, (W, Hh) = H.workload(wl)
    e = bp.Engine(0)
    mesh = H.texture_payloads(meta, mesh_arrays) if mesh_arrays is not None else None
    p = bp.StreamPlayer(e, meta, H.bluenoise(), mesh, W, Hh)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            p.textures[sampler] = bp.Texture(e, maps[kind], name=kind)
    e.resize_canvas(p.width, p.height)
    for k in range(10):
        for call in p.synth_frame(k):
            p.play_call(call)
    e.sync()
    e.timing_begin()
    for call in p.synth_frame(10):
        p.play_call(call)
    ms, _ = e.timing_end(meta["scene"])
    buf = np.zeros((1 << 20, 13), np.uint64)
    n = fn(buf.ctypes.data, buf.shape[0])
    log = buf[:n].astype(np.int64)
    log = log[log[:, 1] > 0]   # rows of the grid's padding workgroups (split tiles) stay zero
    n = len(log)
    t0 = log[:, 0].min()
    s, en = (log[:, 0] - t0) / 100.0, (log[:, 1] - t0) / 100.0
    d = en - s
    span = en.max()
    order = np.argsort(en)
    i_long = int(np.argmax(d))
    sec = log[:, 4:9].astype(np.float64)
    slow = np.argsort(-d)[:max(1, n // 100)]
    np.save(os.path.join(out_dir, "wavelog_%s.npy" % wl), log)
    # CU occupancy in 1-us bins: a CU is busy in a bin when any of its waves covers part of it
    cu_ids, cu = np.unique(log[:, 12], return_inverse=True)
    nb = int(np.ceil(span)) + 1
    busy = np.zeros((len(cu_ids), nb), bool)
    for k in range(n):
        busy[cu[k], int(s[k]):int(np.ceil(en[k])) + 1] = True
    ncu = busy.sum(axis=0)
    occ = {"cus_seen": int(len(cu_ids)),
           "share_lt_half_cus": round(float((ncu < 0.5 * len(cu_ids)).mean()), 4),
           "share_lt_90pct_cus": round(float((ncu < 0.9 * len(cu_ids)).mean()), 4),
           "cu_time_idle_share": round(float(1.0 - busy.mean()), 4),
           "first_bin_lt_half_us": int(np.argmax(ncu < 0.5 * len(cu_ids))) if (ncu < 0.5 * len(cu_ids)).any() else None}
    print(json.dumps({"workload": wl, "kernel_ms": round(ms, 4), "span_us": round(span, 1), "waves": int(n),
                      "longest_us": round(d.max(), 1), "longest_starts_us": round(s[i_long], 1),
                      "longest_slot": i_long,
                      "dur_pct_us": {q: round(float(np.percentile(d, q)), 1) for q in (50, 90, 99, 99.9)},
                      "last_start_us": round(s.max(), 1),
                      "t_99pct_waves_done_us": round(float(en[order[int(0.99 * n)]]), 1),
                      "mean_us": round(float(d.mean()), 1),
                      "longest_wave_walk_iters": int(log[i_long, 2]), "longest_wave_max_lane_steps": int(log[i_long, 3]),
                      "section_share": {nm: round(float(sec[:, k].sum() / max(1, sec.sum())), 4) for k, nm in enumerate(SEC)},
                      "section_share_slowest_1pct": {nm: round(float(sec[slow, k].sum() / max(1, sec[slow].sum())), 4) for k, nm in enumerate(SEC)},
                      "clock_ghz": round(float(sec.sum(axis=1).sum() / max(1e-9, (d * 1e3).sum())), 3),
                      "cu_occupancy": occ,
                      "top10_iters_vs_lane": [[int(log[i, 2]), int(log[i, 3]), round(float(d[i]), 1)] for i in np.argsort(-d)[:10]]}), flush=True)
    e.dispose()
