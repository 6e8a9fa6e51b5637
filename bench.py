#!/usr/bin/env python3
"""bench.py — Mpaths/s of the reference's per-pixel path-tracing frame on MI355X.

Workloads (--workload; tests/helpers.py WORKLOADS), each driven through the Babylon-effect-shaped C
ABI with the uniform stream the reference setup script pushes (recorded, then continued with fresh
uRandomVec2 per frame, camera still). One step = one displayed frame = pathTracing + screenCopy +
screenOutput, as in the reference's render loop (js/GLTF_Model_Path_Tracing.js:1228-1235):
  dragon      (default, BASELINE.json's metric) the 524,288-triangle StanfordDragon stand-in in the
              glTF scene, 1920x1080, 1 spp per frame;
  bunny       BASELINE configs[1]: the reference's StanfordBunny through its own BVH_Fast_Builder;
  helmet      BASELINE configs[2]: DamagedHelmet in the HDRI scene with its four real PBR maps
              (the reference's JPEGs, tests/golden/helmet_maps), seeded equirect for the missing .hdr;
  sky_dragon  BASELINE configs[4]: physical sky + the dragon stand-in (PT_PROG_SKY_MESH) at 3840x2160.

Multi-GPU (one process per GPU): `--gpus N` with no WORLD_SIZE in the environment launches the N
ranks itself (torch.distributed.run, 127.0.0.1) before anything touches a GPU; under a launcher,
WORLD_SIZE must equal --gpus. dragon / bunny / helmet scale weakly (N GPUs render N x 2.07 MP:
1920x1080, 3840x1080, 3840x2160, 7680x2160 for N = 1, 2, 4, 8); --size or sky_dragon fix the frame
and split it (strong scaling, BASELINE configs[3]/[4]). The frame is cut into 16-row bands dealt
round-robin (pt_set_row_partition); per frame every rank exchanges the 2 accumulation rows above and
below its bands with its band neighbours (RCCL P2P), runs screenOutput on its own bands into a
canvas over a torch tensor, and the RGBA8 bands are gathered to rank 0 (RCCL, asynchronous, under
the next frame). Every libpt draw and every torch/RCCL op of a rank is ordered on one dedicated
torch stream (not the legacy default stream).

At N = 1 the line also carries the roofline of the path-tracing kernel: algorithmic bytes per launch
(counted exactly by a counting replay of the same frames) over the average launch
time (HIP events in the timed region) against 8 TB/s, and the L2-to-fabric traffic of the same
kernel measured live by two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over 5 frames of the
same workload, and the CPU baseline (the oracle on the host's cores available to this job, pinned
with taskset, in a child process). Prints ONE JSON line (rank 0).
"""
import argparse
import csv
import glob
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

FRAME_SIZES = {1: (1920, 1080), 2: (3840, 1080), 4: (3840, 2160), 8: (7680, 2160)}
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# algorithmic bytes per counted event
BYTES = {"node_fetches": 32, "leaf_tests": 48, "hit_lookups": 128, "rgba8_taps": 4, "hdr_taps": 16}
PIXEL_IO = 32                  # previousBuffer texel read + accumulation texel write (+4 B blue noise = an rgba8 tap)
CONVERGED_SPP = 1024           # BASELINE configs[4]

METRICS = {
    "bunny": "Mpaths/s + achieved HBM GB/s, StanfordBunny 1080p 1spp (BASELINE configs[1])",
    "helmet": "Mpaths/s + achieved HBM GB/s, DamagedHelmet full PBR maps + HDRI env 1080p (BASELINE configs[2])",
    "sky_dragon": "Mpaths/s + achieved HBM GB/s, Physical_Sky_Model + StanfordDragon 3840x2160 progressive "
                  "(BASELINE configs[4])",
}
DATA = {
    "dragon": "a 524,288-triangle procedural stand-in for the missing StanfordDragon.glb (native builder), "
              "under the reference glTF page's recorded StanfordBunny stream",
    "bunny": "the reference BVH_Fast_Builder output for StanfordBunny, the glTF page's recorded stream",
    "helmet": "the reference BVH_Fast_Builder output for DamagedHelmet under the HDRI page's recorded stream; "
              "its four PBR maps are the reference's JPEGs decoded by Pillow; environment = seeded equirect "
              "(the .hdr files are missing from the reference)",
    "sky_dragon": "the physical-sky page's recorded stream + the glTF model uniforms (helpers.sky_mesh_stream), "
                  "the 524,288-triangle dragon stand-in",
}


def frame_size(n):
    if n in FRAME_SIZES:
        return FRAME_SIZES[n]
    return 1920, 1080 * n


def algorithmic_bytes(cnt):
    return sum(cnt[k] * b for k, b in BYTES.items()) + PIXEL_IO * cnt["paths"]


def baseline_metric():
    """BASELINE.json's metric, verbatim (the value is Mpaths/s of whole frames; the HBM GB/s part is
    the roofline object)."""
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "Mpaths/s + achieved HBM GB/s, StanfordDragon 1080p 1spp, 1/2/4/8 MI355X"


# ------------------------------------------------------------------------------ CPU baseline
def job_cpus():
    """CPUs this job may use: the affinity mask, capped by the cgroup CPU quota (on the GPU box a
    job gets a share of the host, while nproc / os.cpu_count() report the whole machine)."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    n = len(aff) if quota is None else max(1, min(len(aff), int(math.floor(quota))))
    return aff[:n], quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(workload, budget):
    """The CPU oracle (C restatement of the reference GLSL, OpenMP over rows) on every CPU of this
    job, pinned with taskset, in a child process: whole frames of the same workload stream."""
    cpus, quota = job_cpus()
    n = len(cpus)
    env = dict(os.environ, OMP_NUM_THREADS=str(n), OMP_PROC_BIND="close", OMP_PLACES="cores")
    cmd = ["taskset", "-c", ",".join(map(str, cpus)), sys.executable, os.path.join(ROOT, "tools", "cpu_baseline.py"),
           "--workload", workload, "--budget", str(budget), "--threads", str(n)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=budget * 4 + 120)
    if r.returncode != 0:
        return {"value": None, "error": r.stderr[-400:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": round(res["mpaths_per_s"], 3), "unit": "Mpaths/s", "cores": n, "kind": "port",
            "sample": "%d full %dx%d frames of the same stream, CPU oracle (C restatement of the reference GLSL, "
                      "OpenMP %d threads pinned with taskset to CPUs %s), %.1f s"
                      % (res["frames"], res["width"], res["height"], n,
                         "%d-%d" % (cpus[0], cpus[-1]) if cpus == list(range(cpus[0], cpus[-1] + 1)) else cpus,
                         res["seconds"]),
            "nproc": os.cpu_count(), "job_cpus": n, "cgroup_cpu_quota": quota, "cpu_model": cpu_model()}


# ------------------------------------------------------------------------------ live PMC traffic
def live_traffic(workload, W, Hh, frames=5):
    """L2-to-fabric bytes per launch of the path-tracing kernel, measured now: two rocprofv3 --pmc
    passes (FETCH_SIZE and WRITE_SIZE need 3 + 2 of the 4 TCC slots, so one pass each) over
    tools/prof_frames.py rendering `frames` frames of this workload. gfx950 correction
    (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 128-B read requests at 64 B -> doubled; KiB -> B."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    vals = {}
    tmp = tempfile.mkdtemp(prefix="pt_pmc_", dir="/tmp")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", "90", exe, "--kernel-trace", "--pmc", ctr, "--output-format", "csv",
                   "-d", out, "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "prof_frames.py"),
                   "--workload", workload, "--frames", str(frames), "--width", str(W), "--height", str(Hh)]
            r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True)
            if r.returncode != 0:
                return None, "rocprofv3 --pmc %s exited %d" % (ctr, r.returncode)
            per = []
            for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as f:
                    for row in csv.DictReader(f):
                        if "pt_trace<" in row["Kernel_Name"] and row["Counter_Name"] == ctr:
                            per.append(float(row["Counter_Value"]))
            if not per:
                return None, "no %s samples for pt_trace" % ctr
            vals[ctr] = sum(per) / len(per)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return int((2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024), None


# ------------------------------------------------------------------------------ launch
def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N ranks (one process per GPU) and exit with their code."""
    port = str(29500 + os.getpid() % 1000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def launch_check(args, world, rank):
    """--check-launch: bring the process group up exactly as the bench does (nccl on GPUs, gloo
    without) and report the rank count the backend sees - no rendering (CPU-testable)."""
    import torch
    import torch.distributed as tdist
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1:
        tdist.init_process_group(backend)
        seen = tdist.get_world_size()
        tdist.barrier()
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"check": "launch", "n_gpus": world, "ranks_seen": seen, "backend": backend if world > 1 else None,
                          "gpus_requested": args.gpus}), flush=True)
    if world > 1:
        tdist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-oracle baseline (0 = skip)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    ap.add_argument("--no-output", action="store_true", help="time pathTracing+copy only (no screenOutput/gather)")
    ap.add_argument("--check-launch", action="store_true", help="start the ranks, report the world size, render nothing")
    ap.add_argument("--workload", choices=("dragon", "bunny", "helmet", "sky_dragon"), default="dragon",
                    help="dragon (default): BASELINE.json's metric on the StanfordDragon stand-in; bunny: configs[1]; "
                         "helmet: configs[2] (real PBR maps); sky_dragon: configs[4] (physical sky + dragon, 4K)")
    ap.add_argument("--event-every", type=int, default=10, metavar="K",
                    help="time the kernels with HIP events around every K-th frame of the timed region")
    ap.add_argument("--dump-canvas", default=None, metavar="PATH",
                    help="rank 0 saves the last timed frame's RGBA8 canvas (.npy) - e.g. to compare an N-rank "
                         "frame with a one-rank render of the same size")
    ap.add_argument("--size", default=None,
                    help="WxH frame size (e.g. 3840x2160 for the 4K configs); at N > 1 the same frame is split over "
                         "the GPUs (strong scaling, BASELINE configs[3]: --gpus 8 --size 3840x2160)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    if args.check_launch:
        return launch_check(args, world, rank)

    dist, torch, stream = None, None, None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
        # one dedicated stream per rank for libpt draws and torch/RCCL work alike (the legacy default
        # stream would not order them: libpt's own stream is non-blocking)
        stream = torch.cuda.Stream(device=local)
        torch.cuda.set_stream(stream)

    import babylon_pt as bp
    import helpers as H

    meta, mesh_arrays, maps, (W, Hh) = H.workload(args.workload)
    fixed = args.size is not None or args.workload == "sky_dragon"
    if args.workload != "sky_dragon":
        W, Hh = frame_size(world)
    if args.size:
        W, Hh = (int(v) for v in args.size.lower().split("x"))
    engine = bp.Engine(local)
    mesh = H.texture_payloads(meta, mesh_arrays)
    program = meta["scene"]

    rt_ptrs, acc_t = None, None
    pad_bands = bp.padded_bands(Hh, world)
    if dist is not None:
        # the accumulation target is the first H rows of a band-padded torch buffer, so a rank's
        # bands are a strided view of it (no repacking of the whole frame)
        acc_t = torch.zeros((pad_bands * 16, W, 4), dtype=torch.float32, device="cuda")
        copy_t = torch.zeros((Hh, W, 4), dtype=torch.float32, device="cuda")
        rt_ptrs = {"pathTracingRenderTarget": acc_t.data_ptr(), "screenCopyRenderTarget": copy_t.data_ptr()}
        stream.synchronize()
        engine.set_stream(stream.cuda_stream)
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), mesh, W, Hh, rt_ptrs)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    engine.resize_canvas(W, Hh)
    engine.set_row_partition(world, rank)

    if dist is not None:
        # the canvas is the first H rows of a band-padded uint8 tensor: screenOutput writes this
        # rank's bands there, and they are gathered to rank 0's full canvas - asynchronously, two
        # canvases alternating, so frame k's gather overlaps frame k+1's path tracing
        engine.set_output_partition(True)
        halo = bp.halo_buffers(acc_t, world)
        gather = bp.PipelinedBandGather(dist, world, rank, pad_bands * 16, W, "cuda")

    def step(k):
        pt_call, cp_call, out_call = player.synth_frame(k)
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
            torch.cuda.synchronize()
            dist.barrier()

    for k in range(args.warmup):
        step(k)
    barrier_sync()
    # kernel durations from HIP event pairs around every --event-every-th frame's draws (an event
    # record costs ~5 us of stream time between kernels: bracketing every draw slowed the dragon
    # stand-in's frame by 1.7 %, the bunny's by 3.8 %)
    os.environ["PT_TIMING_EVERY"] = str(args.event_every)
    engine.timing_begin()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if args.dump_canvas:
        import numpy as np
        if dist is None:
            np.save(args.dump_canvas, engine.read_canvas(W, Hh))
        elif rank == 0:
            np.save(args.dump_canvas, gather.last_frame()[:Hh].cpu().numpy())
    pt_ms, pt_n = engine.timing_end(program)
    cp_ms, _ = engine.timing_end("screenCopy")
    out_ms, _ = engine.timing_end("screenOutput")

    ranks_seen = world
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ranks_seen = dist.get_world_size()

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

    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return 0

    paths = W * Hh * args.steps
    value = paths / elapsed / 1e6
    avg_launch_ms = max(pt_ms / max(1, pt_n), 1e-9)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    wname = {"bunny": "bunny", "helmet": "helmet_pbr", "dragon": "dragon_standin", "sky_dragon": "dragon_standin"}
    workload = "%s_%s_%dx%d" % (program, wname[args.workload], W, Hh)
    kernel = "pt_trace<%s%s%s>" % ("PAIRS+" if layout == "pairs" else "", program.upper(),
                                   "+TEX" if args.workload == "helmet" else "")
    traffic, pmc_note = None, "N > 1: not collected"
    if world == 1:
        if args.no_pmc:
            pmc_note = "skipped (--no-pmc)"
        elif any(k.startswith("ROCPROF") for k in os.environ):
            pmc_note = "skipped (running under rocprofv3)"
        else:
            traffic, pmc_note = live_traffic(args.workload, W, Hh)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                "achieved_counter_gbs": round(traffic / (avg_launch_ms * 1e-3) / 1e9, 1) if traffic else None,
                "traffic_source": ("live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over 5 frames of this workload, "
                                   "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per launch (gfx950 correction)")
                if traffic else pmc_note,
                "kernel": kernel, "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "counts_per_launch": {k: v / nc for k, v in cnt.items()}}
    line = {
        "metric": baseline_metric() if args.workload == "dragon" else METRICS[args.workload],
        "value": round(value, 2),
        "unit": "Mpaths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if fixed and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: " + DATA[args.workload] + "; continued with fresh uRandomVec2 per frame",
        "config": {"workload": workload, "width": W, "height": Hh, "spp_per_frame": 1, "max_bounces": 6,
                   "triangles": int(mesh_arrays["tri"].shape[0]), "parallelism": "row-bands x%d" % world,
                   "ranks_seen": ranks_seen,
                   "gather": ("per frame: 2-row halo exchange with band neighbours (RCCL P2P), screenOutput "
                              "of own bands, async RCCL gather of RGBA8 bands to rank 0 overlapping the next "
                              "frame") if world > 1 else None},
        "pathtrace_mpaths_per_s": round(W * Hh / (avg_launch_ms * 1e-3) / 1e6 * world, 2),
        "kernel_timing": "HIP events around the draws of every %d-th timed frame (%d launches)" % (args.event_every, pt_n),
        "kernel_ms": {"pathtrace": round(avg_launch_ms, 4), "screen_copy": round(cp_ms / max(1, pt_n), 4),
                      "screen_output": round(out_ms / max(1, pt_n), 4)},
        "roofline": roofline,
    }
    if args.workload == "sky_dragon":
        line["converge_%dspp_s" % CONVERGED_SPP] = round(CONVERGED_SPP * elapsed / args.steps, 3)
        line["converge_note"] = ("%d frames timed; seconds for %d progressive frames = %s"
                                 % (args.steps, CONVERGED_SPP, "measured" if args.steps == CONVERGED_SPP
                                    else "ms_per_step x %d" % CONVERGED_SPP))
    if args.cpu_budget > 0:
        line["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_budget) if world == 1 else None
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
