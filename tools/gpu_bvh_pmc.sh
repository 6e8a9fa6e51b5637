#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
OUT="$GRAFT_REPO_ROOT/gpurun_out/bvhpmc_$TAG"
mkdir -p "$OUT"
PT_QSTATS=1 timeout -k 10 120 python3 tools/prof_frames.py --frames 3 > "$OUT/qstats.txt" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_frames.py" --frames 3 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
