#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r04e_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
B=$PWD/build_variants
bash tools/gpu_env_matrix.sh r04e "dragon bunny helmet sky_dragon bunny16" 2 "PT_LIBPT=$B/base/libpt.so" "-" "PT_LIBPT=$B/gout2/libpt.so" "PT_LIBPT=$B/gout0/libpt.so"
