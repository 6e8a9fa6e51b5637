#!/bin/bash
# pt_persist tuning sweep: wave-list length x refill threshold (bunny 1080p, pairs layout)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/persist_${1:-x}.log
: > $OUT
for lib in "" build_variants/w5/libpt.so; do
  for t in ${TILES:-1 2 4 8 16}; do
    for r in ${REFILLS:-8 16 32}; do
      echo "== lib=${lib:-base} tiles=$t refill=$r" >> $OUT
      PT_LIBPT=${lib:+$PWD/$lib} PT_PERSIST_TILES=$t PT_PERSIST_REFILL=$r timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends persistent --layouts pairs >> $OUT 2>&1 || exit $?
    done
  done
done
