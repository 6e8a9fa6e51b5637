#!/bin/bash
# Tile splitting (pt_trace / pt_order_build): kernel time per split cap (PT_SPLIT_TILES; 0 = off)
# over the bench workloads, two alternating rounds. usage: gpu_split_ab.sh "caps" "workloads"
cd "$GRAFT_REPO_ROOT" || exit 1
CAPS=${1:-"0 16 32 64"}; WLS=${2:-"helmet dragon bunny sky_dragon"}
OUT=gpurun_out/split_ab.log; : > $OUT
for round in 1 2; do
for k in $CAPS; do
  for w in $WLS; do
    PT_SPLIT_TILES=$k timeout -k 10 200 python bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('split$k $w r$round', d['value'], d['ms_per_step'], d['kernel_ms']['pathtrace'])" >> $OUT
  done
done
done
