#!/bin/bash
# One GPU session (run through gpurun): a list of steps, each under its own time limit; the first
# failing step ends the session (no GPU step after a fault, abort, or time limit). Every step's
# output lands in gpurun_out/<TAG>_<n>_<step>.log; the session log lists the steps and their exit codes.
#
# usage: tools/gpu_session.sh TAG STEP [STEP ...]
#   smoke                      __graft_entry__.smoke()
#   pytest[:K[:ENV]]           the GPU parity suite (pytest -m gpu), or only the tests matching -k K (- = all),
#                              under environment ENV (K=V[,K=V])
#   exact                      the driver's exact bench command (bench.py --gpus 1 --steps 20 --warmup 5)
#   bench:W[:ARGS]             bench.py --workload W (ARGS: extra bench flags, commas for spaces)
#   envmx:ROUNDS:WLS:ENVS      path-tracing kernel ms per workload under environment settings, alternating
#                              rounds (WLS comma-separated; ENVS '|'-separated, each space-free K=V[,K=V] or -)
#   fshort:ROUNDS:WLS:ENVS     frames with the driver's short run (--steps 20 --warmup 5)
#   frames:ROUNDS:WLS:ENVS     the same for whole frames (bench.py --no-pmc --cpu-budget 0 per setting);
#                              a workload W@WxH runs at that frame size
#   wavetime:LIB:WLS           wave timeline + CU occupancy of a -DPT_SECPROF build (tools/wavetime.py)
#   prof                       rocprofv3 --kernel-trace --stats of the exact command's workload (20 steps + 5 warmup)
#   pmc[:W[:WxH]]              the five PMC passes over tools/prof_frames.py (default workload dragon), at a frame size
#   movpx:ROUNDS:ENVS          tools/moving_proxy.py (the moving-camera anchor) per setting
#   rankpx:ROUNDS:WORLD:ENVS   tools/rank_proxy.py (rank 0's share of the 4K dragon frame at N = WORLD) per setting
#   profw:W[:WxH]              rocprofv3 kernel trace + stats of bench.py --workload W (50 frames after 100)
#   ktrace:K                   rocprofv3 --kernel-trace --stats over the GPU tests matching -k K
set -o pipefail   # a step's status is its GPU command's, not that of a `| tail` after it
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
SLOG=gpurun_out/${TAG}_session.log
: > "$SLOG"
n=0
run() {   # run LIMIT LOG CMD...  (the step's own time limit)
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
}
for step in "$@"; do
  n=$((n + 1))
  IFS=':' read -r kind a1 a2 a3 <<< "$step"
  LOG="gpurun_out/${TAG}_${n}_${kind}.log"
  echo "step $n: $step" >> "$SLOG"
  case $kind in
    smoke) run 300 "$LOG" python -u -c 'import __graft_entry__ as g; g.smoke()' ;;
    pytest)
      envs=""; [ -n "$a2" ] && envs="${a2//,/ }"
      if [ -n "$a1" ] && [ "$a1" != "-" ]; then run 900 "$LOG" env $envs python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -k "$a1"
      else run 900 "$LOG" env $envs python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread; fi ;;
    exact) run 300 "$LOG" python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench) run 400 "$LOG" python3 bench.py --workload "$a1" ${a2//,/ } ;;
    envmx|frames|fshort)
      : > "$LOG"; rc=0
      for r in $(seq "$a1"); do
        IFS='|' read -ra ENVS <<< "$a3"
        for cfg in "${ENVS[@]}"; do
          for w in ${a2//,/ }; do
            envs=""; [ "$cfg" != "-" ] && envs="${cfg//,/ }"
            wl=${w%@*}; sz=""; [ "$wl" != "$w" ] && sz="--size ${w#*@}"
            if [ $kind = envmx ]; then
              res=$(set -o pipefail; env $envs timeout -k 10 120 python tools/exp_timing.py --workload "$wl" --frames 30 --backends megakernel --layouts pairs --no-mesh-variant 2>&1 | tail -1); rc=$?
            else
              short=""; [ $kind = fshort ] && short="--steps 20 --warmup 5"
              res=$(set -o pipefail; env $envs timeout -k 10 200 python3 bench.py --workload "$wl" $sz $short --no-pmc --cpu-budget 0 --no-check --no-anchors 2>&1 | tail -1); rc=$?
            fi
            echo "r$r [$cfg] $w $res" >> "$LOG"
            [ $rc -ne 0 ] && break 3
          done
        done
      done
      (exit $rc) ;;
    rankpx)   # rankpx:ROUNDS:WORLD:ENVS - tools/rank_proxy.py (rank 0's share of the 4K dragon frame) per setting
      : > "$LOG"; rc=0
      for r in $(seq "$a1"); do
        IFS='|' read -ra ENVS <<< "$a3"
        for cfg in "${ENVS[@]}"; do
          envs=""; [ "$cfg" != "-" ] && envs="${cfg//,/ }"
          res=$(set -o pipefail; env $envs timeout -k 10 200 python3 tools/rank_proxy.py --world "$a2" 2>&1 | tail -1); rc=$?
          echo "r$r [$cfg] n$a2 $res" >> "$LOG"
          [ $rc -ne 0 ] && break 2
        done
      done
      (exit $rc) ;;
    movpx)    # movpx:ROUNDS:ENVS - tools/moving_proxy.py (the moving-camera anchor) per setting
      : > "$LOG"; rc=0
      for r in $(seq "$a1"); do
        IFS='|' read -ra ENVS <<< "$a2"
        for cfg in "${ENVS[@]}"; do
          envs=""; [ "$cfg" != "-" ] && envs="${cfg//,/ }"
          res=$(set -o pipefail; env $envs timeout -k 10 200 python3 tools/moving_proxy.py 2>&1 | tail -1); rc=$?
          echo "r$r [$cfg] $res" >> "$LOG"
          [ $rc -ne 0 ] && break 2
        done
      done
      (exit $rc) ;;
    wavetime) mkdir -p "gpurun_out/wt_$TAG"; PT_LIBPT=$a1 run 300 "$LOG" python3 tools/wavetime.py "gpurun_out/wt_$TAG" ${a2//,/ } ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-budget 0 --no-pmc --no-anchors) > "$LOG" 2>&1 ;;
    profw)    # profw:W - rocprofv3 kernel trace + stats of bench.py --workload W (50 frames after 100)
      sz=""; [ -n "$a2" ] && sz="--size $a2"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof_${TAG}_$a1" -o run -- python3 "$R/bench.py" --workload "$a1" $sz --steps 50 --warmup 100 \
        --cpu-budget 0 --no-pmc --no-anchors) > "$LOG" 2>&1 ;;
    ktrace)   # rocprofv3 --kernel-trace --stats over the GPU tests matching -k a1
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/ktrace_$TAG" -o run -- python3 -m pytest "$R/tests" -m gpu -q -x -p no:cacheprovider \
        --timeout 300 --timeout-method thread -k "$a1") > "$LOG" 2>&1 ;;
    pmc)
      W=${a1:-dragon}; OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"; i=0; rc=0
      SZ=""; [ -n "$a2" ] && SZ="--width ${a2%x*} --height ${a2#*x}"   # pmc:W[:WxH]
      for C in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
               "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
        i=$((i + 1))
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run \
          -- python3 "$R/tools/prof_frames.py" --workload "$W" $SZ --frames 10) > "$OUT/p$i.log" 2>&1 || { rc=$?; break; }
      done
      (exit $rc) ;;
    *) echo "unknown step $step" >> "$SLOG"; exit 2 ;;
  esac
  rc=$?
  echo "step $n rc=$rc" >> "$SLOG"
  if [ $rc -ne 0 ]; then tail -30 "$LOG"; exit $rc; fi
done
echo "session $TAG done" >> "$SLOG"
