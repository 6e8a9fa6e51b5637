#!/bin/bash
# A/B of one environment knob over workloads (bench.py kernel time), two alternating rounds.
# usage: gpu_env_ab.sh VAR "v1 v2 ..." "workloads"
cd "$GRAFT_REPO_ROOT" || exit 1
VAR=$1; VALS=$2; WLS=${3:-"helmet dragon bunny"}
OUT=gpurun_out/env_ab_$VAR.log; : > $OUT
for round in 1 2; do
for v in $VALS; do
  for w in $WLS; do
    env $VAR=$v timeout -k 10 200 python bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('$VAR=$v $w r$round', d['value'], d['ms_per_step'], d['kernel_ms']['pathtrace'])" >> $OUT
  done
done
done
