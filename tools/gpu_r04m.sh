#!/bin/bash
# pt_order_build: its share of screenOutput (fused) or alone (PT_FUSE_ORDER=0), and the wave-aggregated
# bucket atomics (build_variants/order_agg): parity subset, kernel traces, whole-frame A/B
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
PT_LIBPT=build_variants/order_agg/libpt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "stream or dragon or sky" --timeout 200 --timeout-method thread > gpurun_out/pytest_r04m.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for lib in lean agg; do
  for cfg in "dragon 1" "dragon 0" "sky_dragon 1"; do
    set -- $cfg
    L=""; [ $lib = agg ] && L="$R/build_variants/order_agg/libpt.so"
    PT_LIBPT=$L PT_FUSE_ORDER=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r04m_${lib}_$1_f$2" -o run -- python3 "$R/bench.py" --workload $1 --steps 50 --warmup 5 --cpu-budget 0 --no-pmc --no-anchors > "$R/gpurun_out/prof_r04m_${lib}_$1_f$2.log" 2>&1 || exit $?
  done
done
cd "$R"
OUT=gpurun_out/r04m_ab.log
: > $OUT
for r in 1 2; do
  for cfg in - PT_LIBPT=build_variants/order_agg/libpt.so; do
    for w in dragon bunny sky_dragon; do
      envs=""; [ "$cfg" != "-" ] && envs="$cfg"
      env $envs timeout -k 10 200 python3 bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc --no-anchors > gpurun_out/r04m_tmp.json 2> gpurun_out/r04m_tmp.err || exit $?
      echo "r$r $cfg $w $(tail -1 gpurun_out/r04m_tmp.json)" >> $OUT
    done
  done
done
