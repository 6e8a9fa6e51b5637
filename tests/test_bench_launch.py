"""bench.py's multi-GPU launch contract, on CPU: `--gpus N` without a launcher starts N ranks itself
(torch.distributed.run, 127.0.0.1) and the line reports the rank count the backend saw; under a
launcher, WORLD_SIZE must equal --gpus. `--check-launch` brings the process group up exactly as the
bench does (gloo here: no GPU) and renders nothing."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--check-launch"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout       # one line, from rank 0
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2 and lines[0]["backend"] == "gloo"


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--check-launch"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_single_rank_default():
    r = subprocess.run([sys.executable, BENCH, "--check-launch"], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_cpu_baseline_uses_every_job_cpu_pinned():
    """The CPU baseline runs the oracle in a taskset-pinned child on every CPU of the job and
    reports the thread count, nproc and the CPU model."""
    sys.path.insert(0, ROOT)
    import bench
    cpus, _ = bench.job_cpus()
    r = bench.cpu_baseline("bunny", 0.5)
    assert r["value"] and r["value"] > 0, r
    assert r["cores"] == len(cpus) == r["job_cpus"] and r["nproc"] == os.cpu_count()
    assert "taskset" in r["sample"] and r["kind"] == "port"


def _plan(argv, world):
    sys.path.insert(0, ROOT)
    import bench
    import argparse
    ap = argparse.ArgumentParser()
    for a, kw in (("--size", {}), ("--workload", {"default": "dragon"}), ("--scaling", {"default": "strong"}),
                  ("--steps", {"type": int, "default": 200}), ("--event-every", {"type": int, "default": None}),
                  ("--no-check", {"action": "store_true"}), ("--no-output", {"action": "store_true"})):
        ap.add_argument(a, **kw)
    return bench.plan(ap.parse_args(argv), world)


def test_plan_headline_and_scaling_configs():
    """N = 1: the metric's 1080p frame; N > 1 (the driver's `--gpus N`, no other flags): BASELINE
    configs[3]'s 3840x2160 frame split over the GPUs (strong scaling), the frame the N = 1 line's
    dragon_4k_1gpu field renders on one GPU; --scaling weak keeps N x 2.07 MP; --size and the sky
    workload fix the frame."""
    assert _plan([], 1) == {"width": 1920, "height": 1080, "scaling": None, "event_every": 20, "parity_frames": 0}
    for n in (2, 4, 8):
        p = _plan([], n)
        assert (p["width"], p["height"], p["scaling"]) == (3840, 2160, "strong")
        assert p["parity_frames"] == 2          # the N-GPU frame is checked against one GPU after the timed region
    assert (_plan(["--scaling", "weak"], 8)["width"], _plan(["--scaling", "weak"], 8)["height"]) == (7680, 2160)
    assert _plan(["--scaling", "weak"], 8)["scaling"] == "weak"
    assert (_plan(["--size", "640x480"], 2)["width"], _plan(["--size", "640x480"], 2)["scaling"]) == (640, "strong")
    assert (_plan(["--workload", "sky_dragon"], 1)["width"], _plan(["--workload", "sky_dragon"], 1)["height"]) == (3840, 2160)
    assert _plan(["--no-check"], 8)["parity_frames"] == 0
    assert _plan(["--no-output"], 8)["parity_frames"] == 0   # no canvas gathered: nothing to compare
    assert _plan([], 8)["parity_frames"] > 0


def test_compare_frames_reports_bitwise_equality():
    """n_gpu_bitexact: the N-GPU canvas and accumulation against the one-GPU render, bit for bit
    (a -0.0 / +0.0 or NaN-payload difference counts; a canvas byte counts)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    rng = np.random.default_rng(1)
    can = rng.integers(0, 256, (18, 20, 4), dtype=np.uint8)
    acc = rng.standard_normal((18, 20, 4)).astype(np.float32)
    r = bench.compare_frames(can, acc, can.copy(), acc.copy())
    assert r["n_gpu_bitexact"] is True and r["canvas_pixels_differing"] == 0 and r["pixels"] == 360
    acc2 = acc.copy()
    acc2[3, 4, 1] = -acc2[3, 4, 1] if acc2[3, 4, 1] == 0 else np.nextafter(acc2[3, 4, 1], np.float32(np.inf))
    acc2[0, 0, 0] = 0.0
    acc3 = acc2.copy()
    acc3[0, 0, 0] = -0.0
    r = bench.compare_frames(can, acc3, can, acc2)
    assert r["n_gpu_bitexact"] is False and r["accumulation_pixels_differing"] == 1
    can2 = can.copy()
    can2[17, 19, 3] ^= 1
    r = bench.compare_frames(can2, acc, can, acc)
    assert r["n_gpu_bitexact"] is False and r["canvas_pixels_differing"] == 1
    assert bench.compare_frames(can[:4], acc, can, acc)["n_gpu_bitexact"] is False


def test_kernel_timing_brackets_about_ten_draws():
    """HIP-event windows bracket every (steps // 10)-th frame: ~10 draws at the driver's --steps 20
    as at 200 (round 2 bracketed 2 at --steps 20); --event-every overrides."""
    for steps, every in ((20, 2), (200, 20), (5, 1), (1000, 100)):
        p = _plan(["--steps", str(steps)], 1)
        assert p["event_every"] == every and len(range(0, steps, every)) >= min(steps, 10)
    assert _plan(["--steps", "20", "--event-every", "7"], 1)["event_every"] == 7


def test_gpus_n_check_launch_reports_the_4k_strong_config():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--check-launch", "--steps", "20"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert (d["width"], d["height"], d["scaling"], d["event_every"], d["ranks_seen"]) == (3840, 2160, "strong", 2, 2)


def test_multipart_devices_fall_back_to_device_zero(monkeypatch):
    """--engine multipart: one part per visible GPU, or every part on device 0 when fewer are visible
    (the one-GPU rehearsal of the multi-device route); --devices fixes them."""
    sys.path.insert(0, ROOT)
    import bench
    import argparse
    import torch
    a = argparse.Namespace(devices=None, gpus=3)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.multipart_devices(a) == [0, 0, 0]          # fewer GPUs visible than parts
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.multipart_devices(a) == [0, 1, 2]
    assert bench.multipart_devices(argparse.Namespace(devices="0,1", gpus=2)) == [0, 1]


def test_roofline_fracs_formulas():
    """The roofline's bounds (bench.roofline_fracs) on round 5's dragon stand-in numbers: every
    rate over ms_per_step (frac = reference-priced bytes per displayed frame, counter_frac from the PMC
    bytes of pt_trace + pt_cont, pipe_frac from the walk's lane-steps priced by the td_width microbenchmark,
    valu_frac from SQ_INSTS_VALU), the per-span figure under its own name, and the bound the largest
    fraction names."""
    sys.path.insert(0, ROOT)
    import bench
    counts = {"node_fetches": 90965227.8, "leaf_tests": 4669916.4}
    f = bench.roofline_fracs(3285147468, counts, 1.0896, 0.8089, 1289260064)
    assert f["frac"] == round(3285147468 / 0.8089e-3 / 8e12, 4) == 0.5077
    assert f["frac_span"] == round(3285147468 / 1.0896e-3 / 8e12, 4)
    assert f["counter_frac"] == round(1289260064 / 0.8089e-3 / 8e12, 4) == 0.1992
    cyc = 90965227.8 / 2 * 243.8 / 64 + 4669916.4 * 189.2 / 64
    assert f["pipe_frac"] == round(cyc / (256 * 0.8089e-3 * 2.4e9), 4)
    assert 0.37 < f["pipe_frac"] < 0.38 and f["pipe_model"]["lane_steps_per_launch"] == int(90965227.8 / 2 + 4669916.4)
    assert (f["bound"], f["bound_by"]) == ("hbm", "frac")          # without the VALU count, the bytes lead
    assert bench.roofline_fracs(1.0, counts, 1.0, 1.0, None)["counter_frac"] is None
    assert bench.roofline_fracs(1.0, counts, 1.0, 1.0, None)["valu_frac"] is None
    v = bench.roofline_fracs(3285147468, counts, 1.0896, 0.8089, 1289260064, 509562504)
    assert v["valu_frac"] == round(509562504 * 2 / (1024 * 0.8089e-3 * 2.4e9), 4) == 0.5127
    assert (v["bound"], v["bound_by"]) == ("valu", "valu_frac")   # round 5's line: VALU issue, not HBM
    # a walk-bound frame (pipe_frac largest)
    w = bench.roofline_fracs(1e6, {"node_fetches": 4e8, "leaf_tests": 1e7}, 1.0, 1.0, 1e6, 1e6)
    assert w["bound"] == "vmem"
    o = bench.roofline_object(3285147468, counts, 1.0896, 0.8089, 1289260064, 509562504, "pt_trace + pt_cont", None)
    assert o["achieved"] == round(3285147468 / 0.8089e-3 / 1e9, 1) and o["frac"] == 0.5077
    assert o["achieved_counter_gbs"] == round(1289260064 / 0.8089e-3 / 1e9, 1)
    assert o["bound"] == "valu" and o["peak"] == 8000.0 and o["unit"] == "GB/s"
    assert "ms_per_step" in o["rates_over"]


def test_frame_latency_summary():
    """frame_latency_ms: p50 / max of the per-frame latencies the timing window pairs up
    (pt_timing_latency), and the p50 in frame times."""
    sys.path.insert(0, ROOT)
    import bench
    s = bench.latency_summary([2.0, 3.0, 2.5, 9.0], 1.0)
    assert (s["p50"], s["max"], s["frames"], s["p50_per_step"]) == (2.75, 9.0, 4, 2.75)
    assert bench.latency_summary([1.5, 0.5, 1.0], 0.5)["p50"] == 1.0
    assert bench.latency_summary([], 1.0) is None


class _FakeEngine:
    """timing_begin / timing_end / timing_latency as libpt's window reports them (no GPU)."""
    def __init__(self):
        self.began = False

    def timing_begin(self):
        self.began = True

    def timing_end(self, kind):
        return {"gltf": (10.0, 5), "screenCopy": (0.0, 0), "screenOutput": (0.5, 5)}[kind]

    def timing_latency(self, kind):
        return [2.0, 2.5, 2.25, 3.0, 2.1]


def test_every_line_carries_frame_latency():
    """The timed region returns the window's per-frame latencies, and the line's timing fields (bench.py
    timing_fields, shared by the headline) carry frame_latency_ms {p50, max} next to the kernel spans."""
    sys.path.insert(0, ROOT)
    import bench
    e = _FakeEngine()
    steps = []
    el, km, n, lat = bench.timed_region(e, steps.append, 5, 4, 1, lambda: None, "gltf")
    assert e.began and steps == [5, 6, 7, 8] and n == 5 and km["pathtrace"] == 2.0 and len(lat) == 5
    f = bench.timing_fields(km, n, lat, 0.8, 1)
    assert f["frame_latency_ms"]["p50"] == 2.25 and f["frame_latency_ms"]["max"] == 3.0
    assert f["frame_latency_ms"]["p50_per_step"] == round(2.25 / 0.8, 3)
    assert f["kernel_sum_exceeds_step"] is True and f["kernel_ms"] is km
