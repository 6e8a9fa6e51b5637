cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh r03g || exit $?
bash tools/gpu_pmc.sh r03g --workload dragon || exit $?
