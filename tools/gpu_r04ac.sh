#!/bin/bash
# PState counters and flags as bit-fields of one register (build_variants/pstate): GPU parity suite on
# it, kernel time against the tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=build_variants/pstate/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ac.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04ac.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04ac "dragon bunny helmet sky_dragon bunny16" 3 "-" "PT_LIBPT=build_variants/pstate/libpt.so"
