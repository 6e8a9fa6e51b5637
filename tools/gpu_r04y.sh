#!/bin/bash
# any-hit for the sixth segment in the textured variants (past the first diffuse bounce, sharpness 0):
# GPU parity suite on build_variants/anyhitpbr, kernel time against the tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=build_variants/anyhitpbr/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04y.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04y.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04y "helmet dragon" 4 "-" "PT_LIBPT=build_variants/anyhitpbr/libpt.so"
