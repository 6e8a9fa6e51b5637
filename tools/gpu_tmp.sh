cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu_r01k.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r01k.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel,wavefront,persistent --layouts pairs > gpurun_out/exp3.log 2>&1
