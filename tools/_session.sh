cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PT_LIBPT=$GRAFT_REPO_ROOT/build_variants/sky4/libpt.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "sky" > gpurun_out/pytest_sky4.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_sky4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab.sh sky "sky_dragon" 3 || exit $?
