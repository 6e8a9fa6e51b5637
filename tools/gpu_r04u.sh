#!/bin/bash
# 4K screenOutput: with the order build fused (default) or alone (PT_FUSE_ORDER=0), kernel traces
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  PT_FUSE_ORDER=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r04u_sky_f$f" -o run -- python3 "$R/bench.py" --workload sky_dragon --steps 50 --warmup 5 --cpu-budget 0 --no-pmc --no-anchors > "$R/gpurun_out/prof_r04u_sky_f$f.log" 2>&1 || exit $?
done
