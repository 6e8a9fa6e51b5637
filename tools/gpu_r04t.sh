#!/bin/bash
# wave timelines and walk statistics of the round-4 tree (instrumented build)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04t
PT_LIBPT=build_variants/secprof/libpt.so timeout -k 10 300 python3 tools/wavetime.py gpurun_out/r04t helmet dragon bunny > gpurun_out/r04t/wavetime.log 2>&1 || exit $?
PT_LIBPT=build_variants/secprof/libpt.so timeout -k 10 300 python3 tools/walkstat.py dragon helmet > gpurun_out/r04t/walkstat.jsonl 2> gpurun_out/r04t/walkstat.err || exit $?
