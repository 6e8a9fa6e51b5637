#!/bin/bash
# Tuning sweep: parity subset under one env setting, then exp_timing (megakernel, child-pair walk)
# on the bunny and the dragon stand-in for each setting of an environment knob.
# usage: gpu_sweep.sh TAG VAR "v1 v2 ..." [pytest -k expression] [parity value]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; VAR=$2; VALS=$3; K=${4:-"megakernel-pairs and (stream or bunny or dragon or overflow or multimesh)"}
PV=${5:-$(echo $VALS | awk '{print $NF}')}
mkdir -p gpurun_out
env $VAR=$PV timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -rf -k "$K" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc ($VAR=$PV)" >> gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OUT=gpurun_out/sweep_$TAG.log
: > $OUT
for v in $VALS; do
  for extra in "" "--dragon"; do
    echo "== $VAR=$v $extra" >> $OUT
    env $VAR=$v timeout -k 10 180 python tools/exp_timing.py --frames 20 --backends megakernel --layouts pairs --no-mesh-variant $extra >> $OUT 2>&1 || exit $?
  done
done
