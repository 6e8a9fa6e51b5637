#!/bin/bash
# the persistent path-regeneration backend against the megakernel (tile-list length x refill threshold)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/persist_r04d.log
: > $OUT
for w in dragon bunny helmet; do
  echo "$w mega $(PT_CONT=0 timeout -k 10 120 python tools/exp_timing.py --workload $w --frames 20 --backends megakernel --layouts pairs --no-mesh-variant | tail -1)" >> $OUT || exit 1
  for t in 2 4 8; do for r in 8 16 32 48; do
    echo "$w persist T=$t R=$r $(PT_PERSIST_TILES=$t PT_PERSIST_REFILL=$r timeout -k 10 120 python tools/exp_timing.py --workload $w --frames 20 --backends persistent --layouts pairs --no-mesh-variant | tail -1)" >> $OUT || exit 1
  done; done
done
