#!/bin/bash
# A/B of whole-frame bench lines: the in-tree build and each build_variants/<name>/libpt.so,
# dragon and bunny, two alternating rounds. usage: gpu_bench_ab.sh TAG [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-ab}; shift
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.log
: > $OUT
for round in 1 2; do
  for d in base build_variants/*/; do
    n=$(basename $d)
    lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
    for w in dragon bunny; do
      PT_LIBPT=$lib timeout -k 10 200 python bench.py --workload $w --steps 30 --warmup 3 --cpu-budget 0 "$@" > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); print('$n $w r$round', d['value'], d['ms_per_step'], d['kernel_ms']['pathtrace'])" >> $OUT
    done
  done
done
