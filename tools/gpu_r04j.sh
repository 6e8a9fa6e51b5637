#!/bin/bash
# the lean tree (ride / prefetch / priority / XCD-order code removed) against the scalar-cache record
# read (all variants, or the texture-free ones), then the evidence session of the lean tree
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_env_matrix.sh r04j "dragon bunny helmet sky_dragon bunny16" 3 "-" "PT_LIBPT=build_variants/scalar/libpt.so" "PT_LIBPT=build_variants/scalar_notex/libpt.so" || exit $?
bash tools/gpu_evidence.sh r04j
