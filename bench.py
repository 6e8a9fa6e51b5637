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
WORLD_SIZE must equal --gpus. At N > 1 the frame is BASELINE configs[3]'s 3840x2160 split over the
GPUs (strong scaling; the N = 1 line carries the same frame on one GPU as `dragon_4k_1gpu`), or with
--scaling weak N x 2.07 MP (1920x1080, 3840x1080, 3840x2160, 7680x2160). The frame is cut into 16-row bands dealt
round-robin (pt_set_row_partition); per frame every rank exchanges the 2 accumulation rows above and
below its bands with its band neighbours (RCCL P2P), runs screenOutput on its own bands into a
canvas over a torch tensor, and the RGBA8 bands are gathered to rank 0 (RCCL, asynchronous, under
the next frame). Every libpt draw and every torch/RCCL op of a rank is ordered on one dedicated
torch stream (not the legacy default stream). Rank 0 then measures the same frame over the same GPUs
through one multi-part context (`--engine multipart`: libpt's own fan-out, peer copies, no RCCL) in a
child process and adds it to the line as `multipart`.

At N = 1 the line also carries the roofline of the path tracing: algorithmic bytes per frame (SURVEY.md
§8d, counted exactly by a counting replay of the same frames) over ms_per_step against 8 TB/s, the
L2-to-fabric traffic and VALU instructions of pt_trace + pt_cont measured live by rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU) over 5 frames of the same workload, the bound those fractions
name, and the frame latency (a frame's path tracing ready -> its canvas complete); the CPU baseline (the
oracle on the host's cores available to this job, pinned with taskset, in a child process); and, for the
default dragon workload, fields measured in the same run: the 4K frame on one GPU (`dragon_4k_1gpu`), the
scan-like stand-in (`bunny16_1080p`), one rank's share of the 4K frame at N = 2/4/8 (`rank_share_4k`) and
configs[4]'s 1024-frame converging run timed whole (`converge_1024spp`), the 4K ones with the same roofline
object. Prints ONE JSON line (rank 0).
"""
import argparse
import csv
import datetime
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
# the walk's memory-pipe cost per lane-step at full waves (tools/ubench/td_width.hip,
# profiles/r03_ubench_td_width.txt, 48 MiB table, 64 active lanes): a child-pair inner step (3 x dwordx4 +
# dwordx2) 243.8 CU cycles per wave-step, a leaf step (3 x dwordx4) 189.2, at 2.4 GHz
PIPE_CYC_PER_LANE_STEP = {"inner": 243.8 / 64, "leaf": 189.2 / 64}
CUS, CLOCK_GHZ = 256, 2.4
CONVERGED_SPP = 1024           # BASELINE configs[4]
PG_TIMEOUT_S = 240             # N > 1: process-group / store timeout, well inside the driver's per-run budget
PARITY_FRAMES = 2              # N > 1: recorded frames replayed after the timed region and compared with one GPU

METRICS = {
    "bunny": "Mpaths/s + achieved HBM GB/s, StanfordBunny 1080p 1spp (BASELINE configs[1])",
    "helmet": "Mpaths/s + achieved HBM GB/s, DamagedHelmet full PBR maps + HDRI env 1080p (BASELINE configs[2])",
    "sky_dragon": "Mpaths/s + achieved HBM GB/s, Physical_Sky_Model + StanfordDragon 3840x2160 progressive "
                  "(BASELINE configs[4])",
    "bunny16": "Mpaths/s + achieved HBM GB/s, StanfordBunny split x16 (485,408 triangles) 1080p 1spp",
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
    "bunny16": "the reference's StanfordBunny with every triangle split x16 at edge midpoints (same surface, "
               "485,408 triangles, native builder), the glTF page's recorded stream",
}


def frame_size(n):
    if n in FRAME_SIZES:
        return FRAME_SIZES[n]
    return 1920, 1080 * n


def algorithmic_bytes(cnt):
    return sum(cnt[k] * b for k, b in BYTES.items()) + PIXEL_IO * cnt["paths"]


SIMDS, VALU_CYC = 1024, 2   # 4 SIMDs per CU; a wave64 VALU instruction issues over 2 cycles (MI355X_MICROARCH.md)


def roofline_fracs(bytes_per_launch, counts, kernel_ms, frame_ms, traffic, valu=None):
    """The bounds the path tracing can be held against, as fractions of one displayed
    frame's time (ms_per_step: with frames in flight that is the time the job spends per frame):
    frac          SURVEY §8d: reference-priced algorithmic bytes per frame / ms_per_step / 8 TB/s;
    frac_span     the same bytes over the average HIP-event span of a frame's path tracing on its side
                  stream (pt_trace, and pt_cont when the draw compacts; with frames overlapping a span
                  includes time shared with the neighbouring frames' kernels, so it is no kernel time);
    counter_frac  the measured L2-to-fabric bytes of pt_trace + pt_cont (2 x FETCH_SIZE + WRITE_SIZE) per
                  frame / ms_per_step / 8 TB/s (null without the PMC passes);
    pipe_frac     the walk's lane-steps (node fetches / 2 inner steps + leaf tests) x the memory pipe's cost per
                  lane-step at full waves (PIPE_CYC_PER_LANE_STEP) / (256 CUs x ms_per_step x 2.4 GHz): how busy
                  the vector-memory path would be if every load instruction ran 64 lanes;
    valu_frac     the VALU wave-instructions of pt_trace + pt_cont per frame (PMC SQ_INSTS_VALU) x 2 issue cycles /
                  (1024 SIMDs x ms_per_step x 2.4 GHz): how busy the SIMDs' vector issue is (null without PMC).
    bound         the resource with the largest of these fractions: "hbm" (frac or counter_frac), "vmem"
                  (pipe_frac) or "valu" (valu_frac)."""
    peak = PEAK_HBM_GBS * 1e9
    inner, leaf = counts["node_fetches"] / 2.0, counts["leaf_tests"]
    pipe_cycles = inner * PIPE_CYC_PER_LANE_STEP["inner"] + leaf * PIPE_CYC_PER_LANE_STEP["leaf"]
    f = {"frac": round(bytes_per_launch / (frame_ms * 1e-3) / peak, 4),
         "frac_span": round(bytes_per_launch / (kernel_ms * 1e-3) / peak, 4) if kernel_ms else None,
         "counter_frac": round(traffic / (frame_ms * 1e-3) / peak, 4) if traffic else None,
         "pipe_frac": round(pipe_cycles / (CUS * frame_ms * 1e-3 * CLOCK_GHZ * 1e9), 4),
         "valu_frac": round(valu * VALU_CYC / (SIMDS * frame_ms * 1e-3 * CLOCK_GHZ * 1e9), 4) if valu else None,
         "pipe_model": {"lane_steps_per_launch": int(inner + leaf),
                        "cycles_per_lane_step": {k: round(v, 3) for k, v in PIPE_CYC_PER_LANE_STEP.items()},
                        "source": "tools/ubench/td_width.hip (profiles/r03_ubench_td_width.txt), 64 active lanes",
                        "cus": CUS, "clock_ghz": CLOCK_GHZ}}
    cand = {"frac": "hbm", "counter_frac": "hbm", "pipe_frac": "vmem", "valu_frac": "valu"}
    key = max((k for k in cand if f[k] is not None), key=lambda k: f[k])
    f["bound"], f["bound_by"] = cand[key], key
    return f


def roofline_object(bytes_per_frame, counts, span_ms, frame_ms, traffic, valu, kernels, note):
    """The line's roofline object for one workload: every rate over ms_per_step (roofline_fracs), the
    kernels its traffic and VALU count cover named."""
    fr = roofline_fracs(bytes_per_frame, counts, span_ms, frame_ms, traffic, valu)
    return {"bound": fr["bound"], "bound_by": fr["bound_by"],
            "achieved": round(bytes_per_frame / (frame_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": fr["frac"], "traffic": traffic,
            "frac_span": fr["frac_span"], "counter_frac": fr["counter_frac"], "pipe_frac": fr["pipe_frac"],
            "valu_frac": fr["valu_frac"], "valu_insts_per_launch": int(valu) if valu else None,
            "pipe_model": fr["pipe_model"],
            "achieved_counter_gbs": round(traffic / (frame_ms * 1e-3) / 1e9, 1) if traffic else None,
            "traffic_source": ("live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes over 5 frames of this "
                               "workload, (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per frame (gfx950 correction)")
            if traffic else note,
            "kernels": kernels, "algorithmic_bytes_per_launch": int(bytes_per_frame),
            "counts_per_launch": counts,
            "rates_over": "ms_per_step (one displayed frame; frames overlap, DESIGN.md §4)",
            "pricing": ("the reference's work (counting variant: full closest-hit walks and hit lookups); the "
                        "timed kernel ends shadow rays and eligible last segments at their first occluder "
                        "(same image bits, DESIGN.md §6), so 'achieved' is reference work per second")}


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
def live_traffic(workload, W, Hh, frames=5, parts=1, part=0):
    """L2-to-fabric bytes and vector-ALU instructions per frame of the path tracing (pt_trace, and
    pt_cont when late-bounce compaction runs), measured now: three rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE need 3 + 2 of the 4 TCC slots, so one
    pass each; SQ_INSTS_VALU) over tools/prof_frames.py rendering `frames` frames of this workload.
    gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 128-B read requests at 64 B ->
    doubled; KiB -> B. Returns (bytes, VALU wave-instructions, note)."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, None, "rocprofv3 not found"
    vals = {}
    tmp = tempfile.mkdtemp(prefix="pt_pmc_", dir="/tmp")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"):
            out = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", "90", exe, "--kernel-trace", "--pmc", ctr, "--output-format", "csv",
                   "-d", out, "-o", "run", "--", sys.executable, os.path.join(ROOT, "tools", "prof_frames.py"),
                   "--workload", workload, "--frames", str(frames), "--width", str(W), "--height", str(Hh),
                   "--parts", str(parts), "--part", str(part)]
            r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True)
            if r.returncode != 0:
                return None, None, "rocprofv3 --pmc %s exited %d" % (ctr, r.returncode)
            # per frame: pt_trace's launches, and late-bounce compaction's pt_cont with them when it runs
            # (the path tracing of one frame; a counter is summed over a dispatch's rows)
            tot, launches = 0.0, set()
            for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as f:
                    for row in csv.DictReader(f):
                        kn = row["Kernel_Name"]
                        if ("pt_trace<" in kn or "pt_cont<" in kn) and row["Counter_Name"] == ctr:
                            tot += float(row["Counter_Value"])
                            if "pt_trace<" in kn:
                                launches.add(row.get("Dispatch_Id", len(launches)))
            if not launches:
                return None, None, "no %s samples for pt_trace" % ctr
            vals[ctr] = tot / len(launches)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return int((2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024), vals["SQ_INSTS_VALU"], None


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
                          "gpus_requested": args.gpus, "workload": args.workload, **plan(args, world)}), flush=True)
    if world > 1:
        tdist.destroy_process_group()
    return 0


def make_player(engine, workload, W, Hh, rt_ptrs=None):
    """The workload's recorded stream, mesh and maps bound to `engine` at W x H (tests/helpers.py)."""
    import babylon_pt as bp
    import helpers as H
    meta, mesh_arrays, maps, _ = H.workload(workload)
    player = bp.StreamPlayer(engine, meta, H.bluenoise(), H.texture_payloads(meta, mesh_arrays), W, Hh, rt_ptrs)
    if maps:
        for kind, sampler in H.PBR_SAMPLERS.items():
            player.textures[sampler] = bp.Texture(engine, maps[kind], name=kind)
    return player, meta["scene"], int(mesh_arrays["tri"].shape[0])


def frame_size_for(args, world):
    """--size, else the workload's own size at N = 1 (1080p; sky_dragon 4K); at N > 1 BASELINE
    configs[3]'s 3840x2160 split over the GPUs (strong, the default), or N x 2.07 MP (weak)."""
    if args.size:
        return tuple(int(v) for v in args.size.lower().split("x"))
    if args.workload == "sky_dragon" or (world > 1 and args.scaling == "strong"):
        return 3840, 2160
    return frame_size(world)


def plan(args, world):
    """What a run measures, from its arguments (CPU-testable): the frame, the scaling mode (none at
    one GPU), the kernel-timing sample rate, and at N > 1 the recorded frames replayed after the timed
    region through the N-GPU route and compared bit for bit with a one-GPU render (n_gpu_bitexact)."""
    W, Hh = frame_size_for(args, world)
    fixed = world > 1 and (args.scaling == "strong" or args.size is not None or args.workload == "sky_dragon")
    return {"width": W, "height": Hh, "scaling": None if world == 1 else "strong" if fixed else "weak",
            "event_every": args.event_every or max(1, args.steps // 10),
            # --no-output renders no canvas and gathers nothing: there is no N-GPU frame to compare
            "parity_frames": (PARITY_FRAMES if world > 1 and not getattr(args, "no_check", False)
                              and not getattr(args, "no_output", False) else 0)}


# ------------------------------------------------------------------------------ N-GPU parity check
def one_gpu_reference(workload, W, Hh, device, frames):
    """The recorded frames `frames` (indices) of the workload rendered whole on one GPU by a fresh
    context: (RGBA8 canvas, RGBA32F accumulation) as numpy arrays, rows in GL order."""
    import babylon_pt as bp
    engine = bp.Engine(device)
    try:
        player, _, _ = make_player(engine, workload, W, Hh)
        engine.resize_canvas(W, Hh)
        for i in frames:
            player.play_frame(i)
        engine.sync()
        return engine.read_canvas(W, Hh), player.textures["pathTracingRenderTarget"].read()
    finally:
        engine.dispose()


def compare_frames(canvas, acc, ref_canvas, ref_acc):
    """Bitwise comparison of an N-GPU frame (canvas RGBA8, accumulation RGBA32F) with the one-GPU
    render of the same frames: the line's n_gpu_bitexact and the differing pixel counts."""
    import numpy as np
    canvas, ref_canvas = np.asarray(canvas), np.asarray(ref_canvas)
    acc, ref_acc = np.ascontiguousarray(acc, np.float32), np.ascontiguousarray(ref_acc, np.float32)
    if canvas.shape != ref_canvas.shape or acc.shape != ref_acc.shape:
        return {"n_gpu_bitexact": False, "error": "shape %s / %s vs %s / %s" % (canvas.shape, acc.shape,
                                                                            ref_canvas.shape, ref_acc.shape)}
    dc = int((canvas != ref_canvas).any(-1).sum())
    da = int((acc.view(np.uint32) != ref_acc.view(np.uint32)).any(-1).sum())
    return {"n_gpu_bitexact": dc == 0 and da == 0, "canvas_pixels_differing": dc, "accumulation_pixels_differing": da,
            "pixels": int(canvas.shape[0] * canvas.shape[1])}


def latency_summary(lat, ms_per_step):
    """frame_latency_ms of a line: p50 / max over the bracketed frames (pt_timing_latency) of the device
    time from a frame's path tracing becoming ready on its stream to its canvas being complete."""
    if not lat:
        return None
    v = sorted(lat)
    p50 = v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
    return {"p50": round(p50, 4), "max": round(v[-1], 4), "frames": len(v),
            "p50_per_step": round(p50 / ms_per_step, 3) if ms_per_step else None,
            "definition": "device time from a frame's path-tracing draw being ready to start (event on its side "
                          "stream after the waits that order it) to the end of its screenOutput (canvas "
                          "complete, main stream); every event_every-th frame of the timed region"}


def timing_fields(kernel_ms, launches, lat, ms_per_step, event_every):
    """The line's kernel-timing fields: the sampled HIP-event spans per draw kind, the frame latency and the
    spans' sum against the step (event windows add their own stream time around the bracketed draws: a sum
    above the step time flags sampled spans inflated by them - or, with frames overlapping, spans that share
    the GPU)."""
    ksum = sum(kernel_ms.values())
    return {"kernel_timing": ("HIP events around the draws of every %d-th timed frame (%d launches); pathtrace = the "
                              "span of a frame's path tracing on its side stream (pt_trace, then pt_cont when the "
                              "draw compacts), which overlaps the neighbouring frames' spans" % (event_every, launches)),
            "kernel_ms": kernel_ms,
            "frame_latency_ms": latency_summary(lat, ms_per_step),
            "kernel_sum_ms": round(ksum, 4),
            "kernel_sum_exceeds_step": bool(ksum > ms_per_step)}


def timed_region(engine, step, first, count, event_every, barrier_sync, program):
    """`count` steps from frame index `first`, bracketed by barrier_sync, with HIP-event windows around
    every event_every-th draw of each kind. Returns (elapsed s, kernel_ms dict, bracketed launches,
    per-frame latencies in ms)."""
    os.environ["PT_TIMING_EVERY"] = str(event_every)
    engine.timing_begin()
    t0 = time.perf_counter()
    for k in range(first, first + count):
        step(k)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    pt_ms, pt_n = engine.timing_end(program)
    cp_ms, _ = engine.timing_end("screenCopy")
    out_ms, _ = engine.timing_end("screenOutput")
    lat = engine.timing_latency(program)
    n = max(1, pt_n)
    return elapsed, {"pathtrace": round(pt_ms / n, 4), "screen_copy": round(cp_ms / n, 4),
                     "screen_output": round(out_ms / n, 4)}, pt_n, lat


def kernel_name(layout, program, workload):
    return "pt_trace<%s%s%s>" % ({"pairs": "PAIRS+", "trail": "TRAIL+"}.get(layout, ""), program.upper(),
                                 "+TEX" if workload == "helmet" else "")


def single_gpu_run(engine, workload, W, Hh, warmup, steps, event_every, from_frame_one=False):
    """One workload at W x H on `engine`, pathTracing + screenCopy + screenOutput per step. With
    from_frame_one the run starts at the stream's frame 1 (history cleared, the recorded frames
    first), so the last timed frame is frame warmup + steps of a progressive run from scratch
    (configs[4]); else it continues after the recording. Returns (player, program, triangles,
    elapsed s, kernel_ms, bracketed launches, per-frame latencies)."""
    player, program, tris = make_player(engine, workload, W, Hh)
    engine.resize_canvas(W, Hh)
    nrec = len(player.meta["frames"])

    def step(k):
        if from_frame_one and k < nrec:
            player.play_frame(k)
            return
        for call in player.synth_frame(k - nrec if from_frame_one else k):
            player.play_call(call)

    for k in range(warmup):
        step(k)
    engine.sync()
    elapsed, km, n, lat = timed_region(engine, step, warmup, steps, event_every, engine.sync, program)
    return player, program, tris, elapsed, km, n, lat


def rank_share_run(engine, workload, W, Hh, world, rank, warmup, steps):
    """One rank's share of an N-GPU frame on this GPU: the rank's 16-row bands of the N-way partition,
    pathTracing + screenCopy of them and screenOutput of them, as the ranks draw them, without the RCCL
    halo exchange and gather (the per-rank half of a strong-scaling point; tools/rank_proxy.py).
    Returns (Mpaths/s of the rank's own pixels, ms per frame, rows, player, frame latencies). The
    partition stays set (the caller's counting replay prices the same bands); end_partition resets it."""
    import babylon_pt as bp
    player, program, _ = make_player(engine, workload, W, Hh)
    engine.resize_canvas(W, Hh)
    engine.set_row_partition(world, rank)
    engine.set_output_partition(True)

    def step(k):
        for call in player.synth_frame(k):
            player.play_call(call)

    for k in range(warmup):
        step(k)
    engine.sync()
    dt, km, _, lat = timed_region(engine, step, warmup, steps, max(1, steps // 10), engine.sync, program)
    rows = len(bp.owned_rows(Hh, world, rank))
    return rows * W * steps / dt / 1e6, 1e3 * dt / steps, rows, player, km, lat


def end_partition(engine):
    engine.set_output_partition(False)
    engine.set_row_partition(1, 0)


def compaction(engine):
    """What the draws' late-bounce compaction auto mode decided (pt_queue_stats; synchronises)."""
    q = engine.queue_stats()
    return {"mode": q["late_bounce_compaction"], "trial_ms_on_per_off": q["compaction_trial_ratio"],
            "frames_in_flight": q["frames_in_flight"]}


def counted_frame(engine, player, first, n=5):
    """Algorithmic-byte counts per frame of the frames just measured: a counting (untimed) replay of the
    path-tracing draws of synthetic frames first.. first + n - 1 on the same engine, target and partition
    (counting draws neither overlap nor compact: the counts are the reference's work). Returns
    (bytes per frame, counts per frame)."""
    engine.set_counting(True)
    engine.reset_counters()
    for k in range(first, first + n):
        player.play_call(player.synth_frame(k)[0])
    cnt = engine.counters()
    engine.set_counting(False)
    return algorithmic_bytes(cnt) / n, {k: v / n for k, v in cnt.items()}


def pmc_note(args):
    if args.no_pmc:
        return "skipped (--no-pmc)"
    if any(k.startswith("ROCPROF") for k in os.environ):
        return "skipped (running under rocprofv3)"
    return None


def measure_roofline(engine, player, args, workload, W, Hh, first, frame_ms, span_ms, parts=1, part=0):
    """The roofline object of a workload just timed at W x H (rank `part` of `parts` when partitioned):
    counts from the counting replay, PMC bytes and VALU instructions from live rocprofv3 passes at the same
    size and partition, all over ms_per_step (roofline_object)."""
    bpf, counts = counted_frame(engine, player, first)
    note = pmc_note(args)
    traffic = valu = None
    if note is None:
        traffic, valu, note = live_traffic(workload, W, Hh, parts=parts, part=part)
    kernels = "pt_trace (+ pt_cont when the draws compact) of one frame" + (", rank %d of %d" % (part, parts)
                                                                              if parts > 1 else "")
    return roofline_object(bpf, counts, span_ms, frame_ms, traffic, valu, kernels, note)


def moving_camera_run(engine, args):
    """The headline frame while the camera moves: the dragon stand-in at 1920x1080 with uCameraIsMoving
    set on every path-tracing draw (the reference's 0.5 blend, js/PathTracingCommon.js:1331-1337). Such
    draws run one frame in flight (PT_MOVING_SERIAL): throughput and frame latency."""
    player, program, _ = make_player(engine, "dragon", 1920, 1080)
    engine.resize_canvas(1920, 1080)
    moving = {"uCameraIsMoving": ["i", [1]]}

    def step(k):
        for call in player.synth_frame(k):
            player.play_call(call, uniform_override=moving)

    for k in range(20):
        step(k)
    engine.sync()
    el, km, _, lat = timed_region(engine, step, 20, args.steps, max(1, args.steps // 10), engine.sync, program)
    ms = el / args.steps * 1e3
    return {"value": round(1920 * 1080 * args.steps / el / 1e6, 2), "unit": "Mpaths/s", "ms_per_step": round(ms, 4),
            "steps": args.steps, "kernel_ms": km, "frame_latency_ms": latency_summary(lat, ms),
            "one_frame_in_flight": os.environ.get("PT_MOVING_SERIAL", "1") != "0"}


def run_anchors(engine, args):
    """Fields beside the N = 1 headline, measured in the same run on the same engine:
    dragon_4k_1gpu - the dragon stand-in at 3840x2160 (BASELINE configs[3] on one GPU: the anchor of
                     the driver's 1 -> N strong-scaling curve, which renders that frame);
    bunny16_1080p  - the StanfordBunny split x16 (485,408 triangles: scanned geometry at the dragon's
                     size) at the metric's config, beside the procedural torus;
    rank_share_4k  - rank 0's share of that 4K frame split over N = 2, 4, 8 GPUs, rendered on this GPU
                     (its bands' draws as the ranks make them, no RCCL): per-rank Mpaths/s against
                     dragon_4k_1gpu's, the strong-scaling curve's per-rank half;
    converge_1024spp - BASELINE configs[4] as a run: sky + dragon stand-in at 3840x2160, frames 1..1024
                     from a cleared history, pathTracing + screenCopy + 5x5 screenOutput each, timed
                     whole (no extrapolation); --dump-canvas PATH also saves frame 1024's canvas.
    The 4K fields (north_star's target frame) carry the same roofline object as the headline, and
    every field its frame latency."""
    out = {}
    steps4k = max(20, args.steps // 5)
    # (100 warmup draws: the late-bounce compaction trial ends at the 93rd)
    player, _, tris, el, km, n, lat = single_gpu_run(engine, "dragon", 3840, 2160, 100, steps4k, max(1, steps4k // 10))
    ms = el / steps4k * 1e3
    out["dragon_4k_1gpu"] = {"value": round(3840 * 2160 * steps4k / el / 1e6, 2), "unit": "Mpaths/s",
                             "ms_per_step": round(ms, 4), "steps": steps4k, "kernel_ms": km,
                             "width": 3840, "height": 2160, "triangles": tris,
                             "late_bounce_compaction": compaction(engine),
                             "frame_latency_ms": latency_summary(lat, ms)}
    out["dragon_4k_1gpu"]["roofline"] = measure_roofline(engine, player, args, "dragon", 3840, 2160, 100 + steps4k,
                                                         ms, km["pathtrace"])
    player, _, tris, el, km, n, lat = single_gpu_run(engine, "bunny16", 1920, 1080, 100, args.steps,
                                                     max(1, args.steps // 10))
    ms = el / args.steps * 1e3
    out["bunny16_1080p"] = {"value": round(1920 * 1080 * args.steps / el / 1e6, 2), "unit": "Mpaths/s",
                            "ms_per_step": round(ms, 4), "steps": args.steps, "kernel_ms": km,
                            "triangles": tris, "bvh_walk": engine.bvh_layout_used(),
                            "late_bounce_compaction": compaction(engine), "frame_latency_ms": latency_summary(lat, ms)}
    out["moving_camera_1080p"] = moving_camera_run(engine, args)
    shares = {}
    for world in (2, 4, 8):
        v, ms, rows, player, km, lat = rank_share_run(engine, "dragon", 3840, 2160, world, 0, 100, 100)
        try:
            shares["n%d" % world] = {"value": round(v, 2), "ms_per_step": round(ms, 4), "rows": rows,
                                     "per_rank_efficiency": round(v / out["dragon_4k_1gpu"]["value"], 3),
                                     "kernel_ms": km, "late_bounce_compaction": compaction(engine),
                                     "frame_latency_ms": latency_summary(lat, ms)}
            if world == 8:
                shares["n8"]["roofline"] = measure_roofline(engine, player, args, "dragon", 3840, 2160, 200, ms,
                                                            km["pathtrace"], parts=8, part=0)
        finally:
            end_partition(engine)
    out["rank_share_4k"] = dict(shares, unit="Mpaths/s", note="rank 0's bands of the 3840x2160 dragon stand-in "
                                "frame split N ways, on this GPU, 100 frames after 100; no halo exchange or gather")
    player, _, tris, el, km, n, lat = single_gpu_run(engine, "sky_dragon", 3840, 2160, 0, CONVERGED_SPP,
                                                     CONVERGED_SPP // 10, from_frame_one=True)
    ms = el / CONVERGED_SPP * 1e3
    conv = {"seconds": round(el, 4), "frames": CONVERGED_SPP, "ms_per_frame": round(ms, 4),
            "mpaths_per_s": round(3840 * 2160 * CONVERGED_SPP / el / 1e6, 2), "kernel_ms": km, "measured": True,
            "late_bounce_compaction": compaction(engine), "frame_latency_ms": latency_summary(lat, ms),
            "note": "frames 1..%d of the sky + dragon stand-in stream from a cleared history, 3840x2160, each "
                    "pathTracing + screenCopy + screenOutput; wall clock of the whole run" % CONVERGED_SPP}
    if args.dump_canvas:
        import numpy as np
        path = os.path.splitext(args.dump_canvas)[0] + "_sky_dragon_%dspp.npy" % CONVERGED_SPP
        np.save(path, engine.read_canvas(3840, 2160))
        conv["canvas"] = os.path.basename(path)
    conv["roofline"] = measure_roofline(engine, player, args, "sky_dragon", 3840, 2160, CONVERGED_SPP, ms,
                                        km["pathtrace"])
    out["converge_%dspp" % CONVERGED_SPP] = conv
    return out


def multipart_devices(args):
    if args.devices:
        return [int(d) for d in args.devices.split(",")]
    n = args.gpus
    try:
        import torch
        visible = torch.cuda.device_count()   # counts without initialising the GPU on this image
    except Exception:
        visible = 1
    return list(range(n)) if visible >= n else [0] * n


def multipart_main(args, event_every):
    """--engine multipart: one process, one pt_ctx_create_devices context of --gpus parts (the route
    the Node host takes with PT_DEVICES, js/babylon_pt.js): every draw fans out inside pt_render, halo
    rows and the canvas gather move by peer copies, no RCCL. Prints one JSON line."""
    import babylon_pt as bp
    devs = multipart_devices(args)
    W, Hh = frame_size_for(args, len(devs))
    engine = bp.Engine(devices=devs)
    player, program, tris = make_player(engine, args.workload, W, Hh)
    engine.resize_canvas(W, Hh)

    def step(k):
        for call in player.synth_frame(k):
            player.play_call(call)

    for k in range(args.warmup):
        step(k)
    engine.sync()
    elapsed, km, n, lat = timed_region(engine, step, args.warmup, args.steps, event_every, engine.sync, program)
    if args.dump_canvas:
        import numpy as np
        np.save(args.dump_canvas, engine.read_canvas(W, Hh))
    check = None
    if len(devs) > 1 and not args.no_check:
        # the recorded frames again (the first clears the history) through the parts, against one GPU
        idx = list(range(PARITY_FRAMES))
        for i in idx:
            player.play_frame(i)
        engine.sync()
        got = engine.read_canvas(W, Hh), player.textures["pathTracingRenderTarget"].read()
        check = compare_frames(*got, *one_gpu_reference(args.workload, W, Hh, devs[0], idx))
        check["frames"] = PARITY_FRAMES
    line = {"metric": baseline_metric() if args.workload == "dragon" else METRICS[args.workload],
            "value": round(W * Hh * args.steps / elapsed / 1e6, 2), "unit": "Mpaths/s",
            "n_gpus": len(set(devs)), "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if len(devs) > 1 else None, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: " + DATA[args.workload], "engine": "multipart", "parts_seen": engine.parts,
            "devices": devs,
            "config": {"workload": "%s_%s_%dx%d" % (program, args.workload, W, Hh), "width": W, "height": Hh,
                       "triangles": tris, "parallelism": "row-bands x%d (one context, %d parts)" % (len(devs), engine.parts),
                       "gather": "per frame: 2-row halo pulls from band neighbours and the RGBA8 gather to part 0 "
                                 "as peer copies inside pt_render (hipMemcpy2DAsync, event-ordered)"},
            "kernel_timing": "HIP events around every %d-th timed frame's draws, slowest part (%d launches)" % (event_every, n),
            "kernel_ms": km, "frame_latency_ms": latency_summary(lat, elapsed / args.steps * 1e3)}
    if check is not None:
        line["n_gpu_bitexact"] = check["n_gpu_bitexact"]
        line["n_gpu_check"] = check
    print(json.dumps(line), flush=True)
    engine.dispose()
    return 0


def multipart_child(args, world, W, Hh):
    """Rank 0 of an N-rank run: the multipart curve of the same frame over the same GPUs, in a child
    process (the ranks keep their contexts but wait on the host meanwhile). A failure is reported,
    never fatal to the RCCL line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    steps = min(args.steps, 100)
    cmd = [sys.executable, os.path.abspath(__file__), "--engine", "multipart", "--gpus", str(world),
           "--devices", ",".join(str(d) for d in range(world)), "--size", "%dx%d" % (W, Hh), "--workload", args.workload,
           "--steps", str(steps), "--warmup", str(min(args.warmup, 10)), "--cpu-budget", "0", "--no-pmc"]
    if args.no_check:
        cmd.append("--no-check")
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
        if r.returncode != 0:
            return {"error": "exit %d: %s" % (r.returncode, r.stderr[-300:])}
        d = json.loads(r.stdout.strip().splitlines()[-1])
        return {k: d.get(k) for k in ("value", "unit", "ms_per_step", "steps", "parts_seen", "devices", "kernel_ms",
                                      "n_gpu_bitexact", "n_gpu_check")}
    except Exception as e:   # noqa: BLE001 - reported in the line
        return {"error": repr(e)[-300:]}


# ------------------------------------------------------------------------------ N-GPU per-rank detail
def rank_fields(rows):
    """The line's `rank_detail` from one row per rank: [path-tracing kernel ms, halo exchange ms,
    band gather ms, bands owned] (NaN = not measured). A load imbalance shows as a spread of the kernel
    ms (and a slowest rank), a slow collective as its ms against the frame's."""
    def mm(i):
        v = [r[i] for r in rows if r[i] == r[i]]
        return {"min": round(min(v), 4), "max": round(max(v), 4)} if v else None
    k = [r[0] for r in rows]
    return {"pathtrace_kernel_ms": mm(0), "halo_ms": mm(1), "gather_ms": mm(2),
            "bands_per_rank": [int(r[3]) for r in rows],
            "slowest_rank": int(max(range(len(rows)), key=lambda i: k[i])) if all(x == x for x in k) else None,
            "method": ("path-tracing kernel: each rank's HIP-event windows in the timed region; halo exchange "
                       "(RCCL P2P) and RGBA8 band gather: timed alone after the timed region, CUDA events around "
                       "10 of each on the rank's stream")}


def rank_detail(dist, torch, device, row):
    """Every rank passes its row (rank_fields); rank 0 gets the assembled rank_detail, the others None."""
    t = torch.tensor([float(x) for x in row], dtype=torch.float64, device=device)
    g = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(g, t)
    return rank_fields([x.cpu().tolist() for x in g]) if dist.get_rank() == 0 else None


def collective_costs(dist, torch, bp, acc_t, halo, gather, world, rank, reps=10):
    """N > 1, after the timed region: ms per halo exchange and per RGBA8 band gather, each timed alone
    (CUDA events on this rank's stream around `reps` of them, every rank in step)."""
    def timed(fn):
        torch.cuda.synchronize()
        dist.barrier()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    def one_gather():
        gather.target()
        gather.submit()
        gather.drain()

    return (timed(lambda: bp.exchange_halos(dist, acc_t, world, rank, halo)), timed(one_gather))


def nrank_check(dist, torch, engine, player, route, barrier_sync, gather, acc_t, workload, W, Hh, world, rank, device):
    """After the timed region: the first PARITY_FRAMES recorded frames (the first clears the history)
    through the N-rank route - path tracing of each rank's bands, RCCL halos, screenOutput of own
    bands, the RGBA8 gather - and every rank's RGBA32F bands gathered to rank 0 too; rank 0 renders the
    same frames whole on its own GPU in a fresh context and compares both bit for bit."""
    import babylon_pt as bp
    for i in range(PARITY_FRAMES):
        route(player.meta["frames"][i])
    barrier_sync()
    share = bp.band_view(acc_t, world)[:, rank]
    send = torch.empty_like(share)
    glist = [torch.empty_like(share) for _ in range(world)] if rank == 0 else None
    full = torch.zeros_like(acc_t) if rank == 0 else None
    bp.gather_bands(dist, acc_t, world, rank, send, glist, full)
    torch.cuda.synchronize()
    res = None
    if rank == 0:
        canvas = gather.last_frame()[:Hh].cpu().numpy()
        acc = full[:Hh].cpu().numpy()
        res = compare_frames(canvas, acc, *one_gpu_reference(workload, W, Hh, device, range(PARITY_FRAMES)))
        res["frames"] = PARITY_FRAMES
    dist.barrier()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100,
                    help="untimed frames first (>= 73 lets the late-bounce compaction trial finish)")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-oracle baseline (0 = skip)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    ap.add_argument("--no-output", action="store_true", help="time pathTracing+copy only (no screenOutput/gather)")
    ap.add_argument("--check-launch", action="store_true", help="start the ranks, report the world size, render nothing")
    ap.add_argument("--workload", choices=("dragon", "bunny", "helmet", "sky_dragon", "bunny16"), default="dragon",
                    help="dragon (default): BASELINE.json's metric on the StanfordDragon stand-in; bunny: configs[1]; "
                         "helmet: configs[2] (real PBR maps); sky_dragon: configs[4] (physical sky + dragon, 4K); "
                         "bunny16: the StanfordBunny split x16 (485,408 triangles, the scan-like dragon-sized stand-in)")
    ap.add_argument("--engine", choices=("ranks", "multipart"), default="ranks",
                    help="ranks (default): one process per GPU, RCCL halos + gather; multipart: one process over a "
                         "pt_ctx_create_devices context of --gpus parts (the Node host's route; parts share device 0 "
                         "when fewer GPUs are visible)")
    ap.add_argument("--devices", default=None, help="multipart: comma-separated device of each part")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="N > 1: strong (default) = one 3840x2160 frame split over the GPUs (BASELINE configs[3]); "
                         "weak = N x 2.07 MP (1920x1080, 3840x1080, 3840x2160, 7680x2160)")
    ap.add_argument("--no-anchors", action="store_true",
                    help="N = 1: skip the 4K, scan-like and converged-run fields beside the headline")
    ap.add_argument("--no-multipart", action="store_true", help="N > 1: skip the multipart curve beside the RCCL one")
    ap.add_argument("--no-check", action="store_true",
                    help="N > 1: skip the bitwise check of the N-GPU frame against a one-GPU render (n_gpu_bitexact)")
    ap.add_argument("--event-every", type=int, default=None, metavar="K",
                    help="time the kernels with HIP events around every K-th frame of the timed region "
                         "(default: steps // 10, so that about 10 draws are bracketed whatever --steps is)")
    ap.add_argument("--dump-canvas", default=None, metavar="PATH",
                    help="rank 0 saves the last timed frame's RGBA8 canvas (.npy) - e.g. to compare an N-rank "
                         "frame with a one-rank render of the same size")
    ap.add_argument("--size", default=None,
                    help="WxH frame size (e.g. 3840x2160 for the 4K configs); at N > 1 the same frame is split over "
                         "the GPUs (strong scaling)")
    args = ap.parse_args()
    event_every = plan(args, 1)["event_every"]

    if args.engine == "multipart":
        return multipart_main(args, event_every)
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
        # an explicit timeout: a rank that stops answering fails the run (the watchdog aborts the
        # process) instead of holding the driver's run until its own limit
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                 timeout=datetime.timedelta(seconds=PG_TIMEOUT_S))
        dist = tdist
        # one dedicated stream per rank for libpt draws and torch/RCCL work alike (the legacy default
        # stream would not order them: libpt's own stream is non-blocking)
        stream = torch.cuda.Stream(device=local)
        torch.cuda.set_stream(stream)

    import babylon_pt as bp

    p = plan(args, world)
    W, Hh = p["width"], p["height"]
    engine = bp.Engine(local)

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
    player, program, tris = make_player(engine, args.workload, W, Hh, rt_ptrs)
    engine.resize_canvas(W, Hh)
    engine.set_row_partition(world, rank)

    if dist is not None:
        # the canvas is the first H rows of a band-padded uint8 tensor: screenOutput writes this
        # rank's bands there, and they are gathered to rank 0's full canvas - asynchronously, two
        # canvases alternating, so frame k's gather overlaps frame k+1's path tracing
        engine.set_output_partition(True)
        halo = bp.halo_buffers(acc_t, world)
        gather = bp.PipelinedBandGather(dist, world, rank, pad_bands * 16, W, "cuda")

    def route(frame):
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

    def step(k):
        route(player.synth_frame(k))

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
    # kernel durations from HIP event pairs around every event_every-th frame's draws (an event
    # record costs ~5 us of stream time between kernels: bracketing every draw slowed the dragon
    # stand-in's frame by 1.7 %, the bunny's by 3.8 %)
    elapsed, kernel_ms, pt_n, lat = timed_region(engine, step, args.warmup, args.steps, event_every, barrier_sync,
                                                 program)
    if args.dump_canvas:
        import numpy as np
        if dist is None:
            np.save(args.dump_canvas, engine.read_canvas(W, Hh))
        elif rank == 0:
            np.save(args.dump_canvas, gather.last_frame()[:Hh].cpu().numpy())

    check = None
    if dist is not None and p["parity_frames"]:
        check = nrank_check(dist, torch, engine, player, route, barrier_sync, gather, acc_t, args.workload, W, Hh,
                            world, rank, local)

    detail = None
    if dist is not None:
        import babylon_pt as bp
        halo_ms, gather_ms = (float("nan"), float("nan")) if args.no_output else \
            collective_costs(dist, torch, bp, acc_t, halo, gather, world, rank)
        detail = rank_detail(dist, torch, "cuda", [kernel_ms["pathtrace"], halo_ms, gather_ms,
                                                   bp.bands_owned(Hh, world, rank)])

    ranks_seen = world
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ranks_seen = dist.get_world_size()

    comp = compaction(engine)   # (before the counting replay: counting draws never compact)
    # algorithmic bytes of the measured frames: a counted (untimed) replay of the same frames
    bytes_per_launch, counts = counted_frame(engine, player, args.warmup, min(args.steps, 5))
    layout = engine.bvh_layout_used()

    anchors = {}
    if world == 1 and not args.no_anchors and args.workload == "dragon" and args.size is None:
        anchors = run_anchors(engine, args)

    if rank != 0:
        if not args.no_multipart:
            # rank 0's multipart curve runs in a child process on these GPUs meanwhile: wait on the
            # host (the rendezvous store), not in a device-side RCCL barrier that would hold CUs
            dist.barrier()
            dist.distributed_c10d._get_default_store().wait(["bench_multipart_done"],
                                                            datetime.timedelta(seconds=PG_TIMEOUT_S))
        dist.barrier()
        dist.destroy_process_group()
        return 0

    paths = W * Hh * args.steps
    value = paths / elapsed / 1e6
    avg_span_ms = max(kernel_ms["pathtrace"], 1e-9)
    wname = {"bunny": "bunny", "helmet": "helmet_pbr", "dragon": "dragon_standin", "sky_dragon": "dragon_standin",
             "bunny16": "bunny_split16"}
    workload = "%s_%s_%dx%d" % (program, wname[args.workload], W, Hh)
    kernel = kernel_name(layout, program, args.workload)
    traffic, valu, note = None, None, "N > 1: not collected"
    if world == 1:
        note = pmc_note(args)
        if note is None:
            traffic, valu, note = live_traffic(args.workload, W, Hh)
    ms_per_step = elapsed / args.steps * 1e3
    roofline = roofline_object(bytes_per_launch, counts, avg_span_ms, ms_per_step, traffic, valu,
                               "%s (+ pt_cont<...> when the draws compact) of one frame" % kernel, note)
    roofline["kernel"] = kernel
    roofline["bvh_walk"] = layout
    line = {
        "metric": baseline_metric() if args.workload == "dragon" else METRICS[args.workload],
        "value": round(value, 2),
        "unit": "Mpaths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": p["scaling"],
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: " + DATA[args.workload] + "; continued with fresh uRandomVec2 per frame",
        "config": {"workload": workload, "width": W, "height": Hh, "spp_per_frame": 1, "max_bounces": 6,
                   "triangles": tris, "parallelism": "row-bands x%d" % world, "ranks_seen": ranks_seen,
                   "gather": ("per frame: 2-row halo exchange with band neighbours (RCCL P2P), screenOutput "
                              "of own bands, async RCCL gather of RGBA8 bands to rank 0 overlapping the next "
                              "frame") if world > 1 else None},
        "pathtrace_span_mpaths_per_s": round(W * Hh / (avg_span_ms * 1e-3) / 1e6 * world, 2),
        **timing_fields(kernel_ms, pt_n, lat, ms_per_step, event_every),
        "late_bounce_compaction": comp,
        "roofline": roofline,
    }
    line.update(anchors)
    if detail is not None:
        line["rank_detail"] = detail
    if check is not None:
        line["n_gpu_bitexact"] = check["n_gpu_bitexact"]
        line["n_gpu_check"] = check
    if args.workload == "sky_dragon":
        line["converge_%dspp_s" % CONVERGED_SPP] = round(CONVERGED_SPP * elapsed / args.steps, 3)
        line["converge_note"] = ("%d frames timed; seconds for %d progressive frames = %s"
                                 % (args.steps, CONVERGED_SPP, "measured" if args.steps == CONVERGED_SPP
                                    else "ms_per_step x %d" % CONVERGED_SPP))
    if world > 1 and not args.no_multipart:
        dist.barrier()   # every rank's GPU work is done; they wait on the host while the child runs
        try:
            line["multipart"] = multipart_child(args, world, W, Hh)
        finally:
            dist.distributed_c10d._get_default_store().set("bench_multipart_done", "1")
    if args.cpu_budget > 0:
        line["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_budget) if world == 1 else None
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    try:
        rc = main()
    except SystemExit:      # argparse's --help and usage errors exit as they always do
        raise
    except BaseException:   # noqa: BLE001 - any failure of a rank ends it at once, non-zero
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)          # no interpreter teardown (a process group torn down mid-collective can hang)
    sys.exit(rc)
