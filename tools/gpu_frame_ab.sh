#!/bin/bash
# Whole-frame A/B (ms per step and every kernel's time) of the in-tree build against each
# build_variants/<name>/libpt.so, three alternating rounds. usage: gpu_frame_ab.sh TAG "workloads"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-frame}; WLS=${2:-"dragon"}
OUT=gpurun_out/frame_ab_$TAG.log; : > $OUT
for round in 1 2 3; do
  for d in base build_variants/*/; do
    n=$(basename $d); lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
    for w in $WLS; do
      PT_LIBPT=$lib timeout -k 10 200 python bench.py --workload $w --steps 200 --warmup 10 --cpu-budget 0 --no-pmc > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
      python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('$n $w r$round', d['ms_per_step'], d['kernel_ms'])" >> $OUT
    done
  done
done
