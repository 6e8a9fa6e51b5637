#!/bin/bash
# any-hit shadow rays: the GPU parity suite on the new tree, then path-tracing kernel time against
# the tree before it (build_variants/lean), alternating
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04k.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04k.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04k "dragon bunny helmet sky_dragon bunny16" 3 "PT_LIBPT=build_variants/lean/libpt.so" "-"
