cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_r01l.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r01l.log
exit $rc
