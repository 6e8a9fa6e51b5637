#!/usr/bin/env python3
"""bench.py — Mpaths/s of the reference's per-pixel path-tracing frame on MI355X.

Workload (BASELINE.json configs[1]): the StanfordBunny glTF scene (BVH + triangle textures exactly
as the reference's BVH_Fast_Builder / Prepare_Model_For_PathTracing produce them, tests/golden),
1920x1080, 1 sample per pixel per frame, driven through the Babylon-effect-shaped C ABI with the
uniform stream the reference setup script pushes (recorded, then continued with fresh
uRandomVec2 per frame). One step = one displayed frame = pathTracing + screenCopy +
screenOutput, as in the reference's render loop (js/GLTF_Model_Path_Tracing.js:1228-1235).

Multi-GPU (one process per GPU, launched by torch.distributed.run): weak scaling over the
framebuffer. N GPUs render a frame of N x 2.07 MP (1920x1080, 3840x1080, 3840x2160, 7680x2160 for
N = 1, 2, 4, 8), split into 16-row bands dealt round-robin (pt_set_row_partition). Each frame every
rank exchanges the 2 accumulation rows above and below its bands with its band neighbours (RCCL
P2P), runs screenOutput on its own bands (pt_set_output_partition) into a canvas over a torch
tensor, and the RGBA8 bands are gathered to rank 0 (RCCL) - 4 B per pixel cross the fabric, not 16.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

FRAME_SIZES = {1: (1920, 1080), 2: (3840, 1080), 4: (3840, 2160), 8: (7680, 2160)}
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# algorithmic bytes per counted event
BYTES = {"node_fetches": 32, "leaf_tests": 48, "hit_lookups": 128, "rgba8_taps": 4, "hdr_taps": 16}
PIXEL_IO = 32                  # previousBuffer texel read + accumulation texel write (+4 B blue noise = an rgba8 tap)


def frame_size(n):
    if n in FRAME_SIZES:
        return FRAME_SIZES[n]
    return 1920, 1080 * n


def algorithmic_bytes(cnt):
    return sum(cnt[k] * b for k, b in BYTES.items()) + PIXEL_IO * cnt["paths"]


def cpu_baseline(meta, width, height, budget_s, mesh=None, maps=None):
    """The CPU oracle (C restatement of the reference GLSL, OpenMP over rows) on this host,
    timing whole 1920x1080 frames of the same stream until ~budget_s of wall time is spent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import helpers as H
    cores = min(16, os.cpu_count() or 1)
    sc = H.oracle_scene(meta, width, height, mesh, maps)
    acc = np.zeros((height, width, 4), np.float32)
    frames, t0 = 0, time.perf_counter()
    while True:
        f = meta["frames"][frames % len(meta["frames"])]
        u = H.with_resolution(H.path_call(f)["uniforms"], width, height)
        acc, _ = sc.path_trace(u, acc, nthreads=cores)
        frames += 1
        dt = time.perf_counter() - t0
        if dt > budget_s or frames >= 200:
            break
    return {"value": round(frames * width * height / dt / 1e6, 3), "unit": "Mpaths/s", "cores": cores,
            "kind": "port",
            "sample": "%d full %dx%d frames of the bench stream, CPU oracle (C restatement, OpenMP %d threads), %.1f s"
                      % (frames, width, height, cores, dt)}


def load_pmc(workload):
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def baseline_metric():
    """BASELINE.json's metric, verbatim (the value is Mpaths/s of whole frames; the HBM GB/s part is
    the roofline object)."""
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "Mpaths/s + achieved HBM GB/s, StanfordDragon 1080p 1spp, 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-oracle baseline (0 = skip)")
    ap.add_argument("--no-output", action="store_true", help="time pathTracing+copy only (no screenOutput/gather)")
    ap.add_argument("--workload", choices=("dragon", "bunny", "helmet"), default="dragon",
                    help="dragon (default): the model BASELINE.json's metric names, as the 524,288-triangle "
                         "StanfordDragon stand-in (helpers.synthetic_dragon; the .glb is missing from the reference); "
                         "bunny: BASELINE configs[1] (the reference's StanfordBunny through its own builder); "
                         "helmet: BASELINE configs[2] (DamagedHelmet in the HDRI scene, all four PBR samplers bound "
                         "to seeded 2048x2048 stand-ins, seeded 2048x1024 equirect in place of the missing .hdr)")
    ap.add_argument("--size", default=None,
                    help="WxH frame size (e.g. 3840x2160 for the 4K configs); at N > 1 the same frame is split over "
                         "the GPUs (strong scaling, BASELINE configs[3]: --gpus 8 --size 3840x2160)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist

    import babylon_pt as bp
    import helpers as H

    meta = H.stream("hdri_helmet_320x180" if args.workload == "helmet" else "gltf_bunny_1080p")
    W, Hh = frame_size(world)
    if args.size:
        W, Hh = (int(v) for v in args.size.lower().split("x"))
    engine = bp.Engine(local)
    mesh_arrays = H.synthetic_dragon() if args.workload == "dragon" else H.mesh(meta)
    mesh = H.texture_payloads(meta, mesh_arrays)
    program = meta["scene"]

    rt_ptrs, acc_t = None, None
    pad_bands = bp.padded_bands(Hh, world)
    if dist is not None:
        import torch
        # the accumulation target is the first H rows of a band-padded torch buffer, so a rank's
        # bands are a strided view of it (no repacking of the whole frame)
        acc_t = torch.zeros((pad_bands * 16, W, 4), dtype=torch.float32, device="cuda")
        copy_t = torch.zeros((Hh, W, 4), dtype=torch.float32, device="cuda")
        rt_ptrs = {"pathTracingRenderTarget": acc_t.data_ptr(), "screenCopyRenderTarget": copy_t.data_ptr()}
        torch.cuda.synchronize()
    if dist is not None:
        # draws, the band gather (RCCL) and rank 0's screenOutput are ordered on one stream
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), mesh, W, Hh, rt_ptrs)
    if args.workload == "helmet":
        maps = H.synthetic_pbr_maps(2048)
        for kind, sampler in H.PBR_SAMPLERS.items():
            player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    engine.resize_canvas(W, Hh)
    engine.set_row_partition(world, rank)

    if dist is not None:
        import torch
        # the canvas is the first H rows of a band-padded uint8 tensor: screenOutput writes this
        # rank's bands there, and they are gathered to rank 0's full canvas - asynchronously, two
        # canvases alternating, so frame k's gather overlaps frame k+1's path tracing
        engine.set_output_partition(True)
        halo = bp.halo_buffers(acc_t, world)
        gather = bp.PipelinedBandGather(dist, world, rank, pad_bands * 16, W, "cuda")

    def step(k):
        frame = player.synth_frame(k)
        pt_call, cp_call, out_call = frame
        player.play_call(pt_call)
        player.play_call(cp_call)
        if args.no_output:
            return
        if dist is None:
            player.play_call(out_call)
            return
        # halo rows from the band neighbours (RCCL P2P), screenOutput of this rank's bands, async
        # RCCL gather of the RGBA8 bands to rank 0 (no host sync in a frame)
        bp.exchange_halos(dist, acc_t, world, rank, halo)
        engine.canvas_wrap(W, Hh, gather.target().data_ptr())
        player.play_call(out_call)
        gather.submit()

    def barrier_sync():
        if dist is not None:
            gather.drain()   # every frame's gather is part of the timed work
        engine.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for k in range(args.warmup):
        step(k)
    barrier_sync()
    engine.timing_begin()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    pt_ms, pt_n = engine.timing_end(program)
    cp_ms, _ = engine.timing_end("screenCopy")
    out_ms, _ = engine.timing_end("screenOutput")

    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # algorithmic bytes of the measured launches: a counted (untimed) replay of the same frames
    engine.set_counting(True)
    engine.reset_counters()
    nc = min(args.steps, 5)
    for k in range(args.warmup, args.warmup + nc):
        player.play_call(player.synth_frame(k)[0])
    cnt = engine.counters()
    engine.set_counting(False)
    layout = engine.bvh_layout_used()
    bytes_per_launch = algorithmic_bytes(cnt) / nc
    if dist is not None:
        import torch
        t = torch.tensor([bytes_per_launch, cnt["paths"] / nc], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        bytes_total_launch = float(t[0].item())
    else:
        bytes_total_launch = bytes_per_launch

    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return

    paths = W * Hh * args.steps
    value = paths / elapsed / 1e6
    avg_launch_ms = pt_ms / max(1, pt_n)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    workload = "%s_%s_%dx%d" % (program, {"bunny": "bunny", "helmet": "helmet_pbr", "dragon": "dragon_standin"}[args.workload],
                                W, Hh)
    pmc = load_pmc(workload)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    line = {
        "metric": baseline_metric() if args.workload == "dragon" else {
            "bunny": "Mpaths/s + achieved HBM GB/s, StanfordBunny 1080p 1spp (BASELINE configs[1])",
            "helmet": "Mpaths/s + achieved HBM GB/s, DamagedHelmet PBR + HDRI env 1080p (BASELINE configs[2])"}[args.workload],
        "value": round(value, 2),
        "unit": "Mpaths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        # weak: N GPUs render N x 2.07 MP (frame_size); --size fixes the frame, split over the N GPUs
        "scaling": "strong" if args.size and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic: the reference setup script's recorded %s uniform stream, continued with fresh "
                 % ("DamagedHelmet/HDRI" if args.workload == "helmet" else "StanfordBunny") +
                 "uRandomVec2 per frame; mesh textures = " +
                 {"bunny": "the reference BVH_Fast_Builder output",
                  "helmet": "the reference BVH_Fast_Builder output for DamagedHelmet (HDRI setup script's stream); "
                            "PBR maps and environment = seeded stand-ins (helpers.synthetic_pbr_maps / synthetic_hdr)",
                  "dragon": "a 524,288-triangle procedural stand-in for the missing StanfordDragon.glb, built by the "
                            "native builder"}[args.workload]),
        "config": {"workload": workload, "width": W, "height": Hh, "spp_per_frame": 1, "max_bounces": 6,
                   "triangles": int(mesh_arrays["tri"].shape[0]), "parallelism": "row-bands x%d" % world,
                   "gather": ("per frame: 2-row halo exchange with band neighbours (RCCL P2P), screenOutput "
                              "of own bands, async RCCL gather of RGBA8 bands to rank 0 overlapping the next "
                              "frame") if world > 1 else None},
        "pathtrace_mpaths_per_s": round(W * Hh / world / (avg_launch_ms * 1e-3) / 1e6 * world, 2),
        "kernel_ms": {"pathtrace": round(avg_launch_ms, 4), "screen_copy": round(cp_ms / max(1, pt_n), 4),
                      "screen_output": round(out_ms / max(1, pt_n), 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": "pt_trace<%s%s%s>" % ("PAIRS+" if layout == "pairs" else "", program.upper(),
                                                     "+TEX" if args.workload == "helmet" else ""),
                     "algorithmic_bytes_per_launch": int(bytes_per_launch),
                     "counts_per_launch": {k: v / nc for k, v in cnt.items()}},
    }
    if args.cpu_budget > 0:
        line["cpu_baseline"] = (cpu_baseline(meta, 1920, 1080, args.cpu_budget, mesh_arrays,
                                             maps if args.workload == "helmet" else None) if world == 1 else None)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
