#!/bin/bash
# Timing sweep over library variants built into build_variants/<name>/libpt.so (plus the in-tree
# build as "base"): bunny 1080p, megakernel, both BVH layouts.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/variants_${1:-x}.log
: > $OUT
echo "== base" >> $OUT
timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel >> $OUT 2>&1 || exit $?
for d in build_variants/*/; do
  n=$(basename $d)
  echo "== $n" >> $OUT
  PT_LIBPT=$PWD/$d/libpt.so timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel >> $OUT 2>&1 || exit $?
done
