#!/bin/bash
# Deferred-schedule sweep: parity of the child-pair programs first, then megakernel timings for
# PT_DEFER_RATIO / PT_DEFER_MIN settings on the bunny and the dragon stand-in, per library variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/defer_${1:-x}.log
: > $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "megakernel-pairs" >> $OUT 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# maximal interleaving: leave the walk phase after every step
PT_DEFER_RATIO=0 PT_DEFER_MIN=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "megakernel-pairs" >> $OUT 2>&1
rc=$?; echo "pytest (ratio 0) rc=$rc" >> $OUT
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for d in base build_variants/*/; do
  n=$(basename $d)
  lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
  for cfg in "1e9 4" "1 4" "0.5 4" "2 4" "1 16"; do
    set -- $cfg
    for extra in "" "--dragon"; do
      echo "== $n ratio=$1 min=$2 $extra" >> $OUT
      PT_DEFER_RATIO=$1 PT_DEFER_MIN=$2 PT_LIBPT=$lib timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel --layouts pairs $extra >> $OUT 2>&1 || exit $?
    done
  done
done
