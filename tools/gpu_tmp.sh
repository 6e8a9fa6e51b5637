cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel --layouts pairs > gpurun_out/exp7.log 2>&1 || exit $?
timeout -k 10 120 python tools/exp_timing.py --frames 20 --backends megakernel --layouts pairs --dragon >> gpurun_out/exp7.log 2>&1
