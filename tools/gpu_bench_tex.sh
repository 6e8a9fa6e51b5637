#!/bin/bash
# helmet (textured variant) bench: in-tree build vs build_variants/<name>, alternating twice
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/bench_tex_${1:-x}.log
: > $OUT
for round in 1 2; do
  for d in base build_variants/*/; do
    n=$(basename $d); lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
    echo "== $n (round $round)" >> $OUT
    PT_LIBPT=$lib timeout -k 10 200 python bench.py --workload helmet --steps 30 --warmup 5 --cpu-budget 0 >> $OUT 2>/dev/null || exit $?
  done
done
