#!/bin/bash
# screenOutput occupancy (order build at 32 held tiles per thread): parity, then whole-frame bench
# against the tree before it (build_variants/lean), alternating
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04l.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04l.log
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=gpurun_out/r04l_ab.log
: > $OUT
for r in 1 2; do
  for cfg in PT_LIBPT=build_variants/lean/libpt.so -; do
    for w in dragon bunny helmet sky_dragon; do
      envs=""; [ "$cfg" != "-" ] && envs="$cfg"
      env $envs timeout -k 10 200 python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc --no-anchors > gpurun_out/r04l_tmp.json 2> gpurun_out/r04l_tmp.err || exit $?
      echo "r$r $cfg $w $(tail -1 gpurun_out/r04l_tmp.json)" >> $OUT
    done
  done
done
