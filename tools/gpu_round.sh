#!/bin/bash
# One GPU session: parity tests, bench (default workload = the dragon stand-in, then the bunny),
# rocprofv3 kernel trace + stats of the default bench, PMC passes for both meshes. Every GPU step
# has its own time limit; a crash/timeout (anything but pytest's 0/1) ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-budget 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 300 python bench.py --workload bunny --steps 50 --warmup 5 --cpu-budget 10 > gpurun_out/bench_${TAG}_bunny.json 2> gpurun_out/bench_${TAG}_bunny.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --cpu-budget 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
echo "prof rc=0" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_pmc.sh ${TAG}_dragon --dragon || exit $?
bash tools/gpu_pmc.sh ${TAG}_bunny
