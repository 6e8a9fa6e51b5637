#!/bin/bash
# Quick GPU check after a kernel change: a parity subset, then bench lines (no CPU baseline, no PMC)
# usage: gpu_quick.sh TAG "pytest -k expression" "workload ..."
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; K=$2; WLS=${3:-"dragon helmet bunny"}
mkdir -p gpurun_out
OUT=gpurun_out/quick_$TAG.log
: > $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" >> $OUT 2>&1 || { echo "pytest rc=$?" >> $OUT; exit 1; }
fi
for W in $WLS; do
  timeout -k 10 300 python bench.py --workload $W --steps 100 --warmup 10 --cpu-budget 0 --no-pmc > gpurun_out/quick_${TAG}_$W.json 2>> $OUT || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['kernel_ms'])" gpurun_out/quick_${TAG}_$W.json $W >> $OUT
done
