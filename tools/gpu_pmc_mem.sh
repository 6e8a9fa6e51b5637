#!/bin/bash
# Memory-pipeline PMC passes (TA / TD / TCP: address unit, data unit, L1) over the profiling driver:
# L1->L2 read latency, TLB hits and misses, address-unit busy and stalls. One rocprofv3 run per pass.
# usage: gpu_pmc_mem.sh TAG [prof_frames.py args, e.g. --workload dragon]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-mem}
shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcmem_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_RW_READ_REQ_sum TA_BUFFER_READ_WAVEFRONTS_sum TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_frames.py" --frames 10 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
