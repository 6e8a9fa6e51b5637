#!/bin/bash
# the sky + mesh scene's G-buffer fields out of LDS now that the colour is recomputed (kGoutLdsSky 3:
# normal in LDS, 8 stack levels; 0: normal in memory, 10 levels): parity subset, kernel time
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in sky3 sky0; do
  PT_LIBPT=build_variants/$v/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "sky" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04aa_$v.log 2>&1 || exit $?
done
bash tools/gpu_env_matrix.sh r04aa "sky_dragon" 4 "-" "PT_LIBPT=build_variants/sky3/libpt.so" "PT_LIBPT=build_variants/sky0/libpt.so"
