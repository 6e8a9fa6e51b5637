set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PT_CONT_SORT=1
for W in dragon helmet; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r06s_$W" -o run -- python3 "$R/bench.py" --workload $W --steps 50 --warmup 100 --cpu-budget 0 --no-pmc --no-anchors --no-check > "$R/gpurun_out/r06s_$W.log" 2>&1 || exit 1
done
