#!/bin/bash
# Split-tile knobs (PT_SPLIT_NEAR buckets : PT_SPLIT_TILES cap) over workloads, bench.py kernel time,
# two alternating rounds. usage: gpu_split_sweep.sh "3:32 5:64 ..." "workloads"
cd "$GRAFT_REPO_ROOT" || exit 1
COMBOS=${1:-"3:32 5:64"}; WLS=${2:-"helmet"}
OUT=gpurun_out/split_sweep.log; : > $OUT
for round in 1 2; do
for c in $COMBOS; do
  nb=${c%%:*}; cap=${c##*:}
  for w in $WLS; do
    PT_SPLIT_NEAR=$nb PT_SPLIT_TILES=$cap timeout -k 10 200 python bench.py --workload $w --steps 200 --warmup 10 --cpu-budget 0 --no-pmc > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('$c $w r$round', d['value'], d['ms_per_step'], d['kernel_ms']['pathtrace'])" >> $OUT
  done
done
done
