#!/bin/bash
# the driver's default bench command on the final tree (bench.py JSON sanity after the roofline note)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r04z_default.json 2> gpurun_out/bench_r04z_default.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04z_exact.json 2> gpurun_out/bench_r04z_exact.err || exit $?
