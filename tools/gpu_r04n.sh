#!/bin/bash
# field-major G-buffer fields: GPU parity suite, kernel time against build_variants/lean (the tree before)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04n.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04n.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04n "dragon bunny helmet sky_dragon bunny16" 3 "PT_LIBPT=build_variants/lean/libpt.so" "-"
