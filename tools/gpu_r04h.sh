#!/bin/bash
# screenOutput riding: its parity tests, then whole-frame A/B (PT_RIDE=0/1, bench.py), the walk knobs
# (kernel time), and the evidence session of the tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "rides or deferred or stream" --timeout 120 --timeout-method thread > gpurun_out/r04h_pytest_ride.log 2>&1 || exit $?
OUT=gpurun_out/r04h_ride_ab.log
: > $OUT
for r in 1 2; do
  for cfg in PT_RIDE=0 PT_RIDE=1; do
    for w in dragon bunny helmet; do
      env $cfg timeout -k 10 200 python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc --no-anchors > gpurun_out/r04h_tmp.json 2> gpurun_out/r04h_tmp.err || exit $?
      echo "r$r $cfg $w $(tail -1 gpurun_out/r04h_tmp.json)" >> $OUT
    done
  done
done
bash tools/gpu_env_matrix.sh r04h "dragon bunny helmet" 2 "-" "PT_WALK_PREFETCH=1" "PT_WALK_PRIO=1" || exit $?
bash tools/gpu_evidence.sh r04h
