#!/bin/bash
# PMC passes over the profiling driver (separate passes, counters only with --kernel-trace).
# usage: gpu_pmc.sh TAG [prof_frames.py args, e.g. --dragon]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_frames.py" --frames 10 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
