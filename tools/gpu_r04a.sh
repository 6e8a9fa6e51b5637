#!/bin/bash
# round-4 first session: the pruned tree's parity suite, the driver's exact bench command, and the
# child-pair walk's load coherence (secprof variant)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r04a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench_exact.json 2> gpurun_out/r04a_bench_exact.err || exit $?
PT_LIBPT=$PWD/build_variants/secprof/libpt.so timeout -k 10 300 python3 tools/walkstat.py dragon bunny helmet sky_dragon bunny16 > gpurun_out/r04a_walkstat.jsonl 2> gpurun_out/r04a_walkstat.err || exit $?
