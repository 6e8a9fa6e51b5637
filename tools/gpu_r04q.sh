#!/bin/bash
# any-hit for eligible last segments (all variants): GPU parity suite on build_variants/lastbounce,
# kernel time against build_variants/base_p (shadow rays only, textured variants only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=build_variants/lastbounce/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04q.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04q.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04q "dragon bunny helmet sky_dragon bunny16" 3 "PT_LIBPT=build_variants/base_p/libpt.so" "PT_LIBPT=build_variants/lastbounce/libpt.so"
