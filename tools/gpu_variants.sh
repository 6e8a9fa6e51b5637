#!/bin/bash
# Timing sweep over library variants built into build_variants/<name>/libpt.so (plus the in-tree
# build as "base"): megakernel + child-pair walk, per-launch path-tracing time on each bench
# workload, twice each in alternating order (base, variants, base, variants) so that box drift
# shows. usage: gpu_variants.sh TAG ["workload ..."]   (summary: tools/variants_summary.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/variants_${1:-x}.log
WLS=${2:-"dragon bunny helmet sky_dragon"}
: > $OUT
for round in 1 2; do
  for d in base build_variants/*/; do
    n=$(basename $d)
    lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
    for w in $WLS; do
      echo "== $n $w (round $round)" >> $OUT
      PT_LIBPT=$lib timeout -k 10 120 python tools/exp_timing.py --workload $w --frames 20 --backends megakernel --layouts pairs --no-mesh-variant >> $OUT 2>&1 || exit $?
    done
  done
done
