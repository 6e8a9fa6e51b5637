#!/bin/bash
# screenOutput over 32x16 tiles (build_variants/outwide): GPU parity suite on it, whole-frame A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=build_variants/outwide/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04v.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04v.log
if [ $rc -ne 0 ]; then exit $rc; fi
OUT=gpurun_out/r04v_ab.log
: > $OUT
for r in 1 2; do
  for cfg in - PT_LIBPT=build_variants/outwide/libpt.so; do
    for w in dragon helmet sky_dragon; do
      envs=""; [ "$cfg" != "-" ] && envs="$cfg"
      env $envs timeout -k 10 200 python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc --no-anchors > gpurun_out/r04v_tmp.json 2> gpurun_out/r04v_tmp.err || exit $?
      echo "r$r $cfg $w $(tail -1 gpurun_out/r04v_tmp.json)" >> $OUT
    done
  done
done
