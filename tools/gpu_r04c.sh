#!/bin/bash
# per-kernel split of the late-bounce compaction: rocprofv3 kernel trace of the profiling driver
# under PT_CONT settings (pt_trace vs pt_cont time per frame)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/kt
cd /tmp && export TMPDIR=/tmp
for cfg in "PT_CONT=0" "PT_CONT_LANES=16" "PT_CONT_LANES=64" "PT_CONT_LANES=64 PT_CONT_BOUNCE=2" "PT_CONT_LANES=64 PT_CONT_BOUNCE=4" "PT_CONT_LANES=64 PT_CONT_BOUNCE=5"; do
  tag=$(echo "$cfg" | tr ' =' '__')
  for w in dragon helmet; do
    d="$R/gpurun_out/kt_${tag}_${w}"
    env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- python3 "$R/tools/prof_frames.py" --workload $w --frames 20 > "$R/gpurun_out/kt/${tag}_${w}.log" 2>&1 || exit $?
    f=$(find "$d" -name "*kernel_stats.csv" | head -1)
    [ -n "$f" ] && cp "$f" "$R/gpurun_out/kt/${tag}_${w}.csv"
    rm -rf "$d"
  done
done
