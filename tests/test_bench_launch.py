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
