cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gout.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gout.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab.sh gout "dragon bunny sky_dragon bunny16" 2 || exit $?
