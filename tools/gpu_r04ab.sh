#!/bin/bash
# the tree with the sky + mesh G-buffer out of LDS: smoke, GPU parity suite, sky + dragon and exact bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r04ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ab.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --workload sky_dragon > gpurun_out/bench_r04ab_sky_dragon.json 2> gpurun_out/bench_r04ab_sky_dragon.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04ab_exact.json 2> gpurun_out/bench_r04ab_exact.err || exit $?
