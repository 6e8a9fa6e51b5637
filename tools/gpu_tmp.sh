cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_r01o.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r01o.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel --layouts pairs > gpurun_out/exp5.log 2>&1
