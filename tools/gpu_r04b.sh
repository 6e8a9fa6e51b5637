#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r04b_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04b "dragon bunny helmet sky_dragon bunny16" 2 "PT_CONT=0" "PT_CONT=1" "PT_CONT_BOUNCE=2" "PT_CONT_LANES=32" "PT_CONT_LANES=8" "PT_CONT_WAVES=8"
