#!/bin/bash
# the restart-trail walk with the G-buffer's LDS as ring entries (10 for the glTF / HDRI scenes):
# GPU parity suite, then trail vs the stack walk in this tree and the trail of the tree before
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04p.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04p.log
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=gpurun_out/envmx_r04p.log
: > $OUT
for r in 1 2 3; do
  for cfg in "- pairs" "- trail" "PT_LIBPT=build_variants/lean/libpt.so trail"; do
    set -- $cfg
    for w in dragon bunny helmet sky_dragon bunny16; do
      envs=""; [ "$1" != "-" ] && envs="$1"
      res=$(env $envs timeout -k 10 120 python tools/exp_timing.py --workload $w --frames 30 --backends megakernel --layouts $2 --no-mesh-variant 2>&1 | tail -1) || { echo "FAIL $cfg $w: $res" >> $OUT; exit 1; }
      echo "r$r [$1 $2] $w $res" >> $OUT
    done
  done
done
