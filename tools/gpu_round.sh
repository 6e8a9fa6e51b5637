#!/bin/bash
# One GPU session: parity tests, bench on every workload (default = the dragon stand-in), a
# rocprofv3 kernel trace + stats of the default bench. Every GPU step has its own time limit; a
# crash/timeout (anything but pytest's 0/1) ends the session.
# usage: gpu_round.sh TAG [pytest -k expression]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for W in dragon sky_dragon helmet bunny bunny16; do
  timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --cpu-budget 0 --no-pmc --no-anchors > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
echo "prof rc=0" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"
