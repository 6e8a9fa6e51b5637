cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh r03f || exit $?
bash tools/gpu_pmc.sh r03f --workload dragon || exit $?
