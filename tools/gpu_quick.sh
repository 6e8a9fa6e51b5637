cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_r01f.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r01f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/exp_timing.py --frames 20 > gpurun_out/exp2.log 2>&1
