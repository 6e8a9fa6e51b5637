#!/bin/bash
# analytic objects' attributes selected per lane from scalar loads (build_variants/kargsel) instead of
# vector loads from the kernarg segment: GPU parity suite on it, kernel time against the tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=build_variants/kargsel/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04w.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04w.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04w "dragon bunny helmet sky_dragon bunny16" 3 "-" "PT_LIBPT=build_variants/kargsel/libpt.so"
