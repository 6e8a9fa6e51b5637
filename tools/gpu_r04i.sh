#!/bin/bash
# is the round-4 slowdown the box or the code? path-tracing kernel time of the pre-ride tree (92a4406),
# the current tree without the riding screenOutput call, and the current tree, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_env_matrix.sh r04i "dragon bunny helmet" 3 "PT_LIBPT=build_variants/pre/libpt.so" "PT_LIBPT=build_variants/noride/libpt.so" "-"
