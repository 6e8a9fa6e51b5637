cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prio_sweep.log; : > $OUT
for P in 0 16 64 256 1024; do
  for W in helmet dragon bunny sky_dragon; do
    echo "P=$P W=$W base $(PT_PRIO_TILES=$P timeout -k 10 120 python tools/exp_timing.py --workload $W --backends megakernel --layouts pairs --no-mesh-variant --frames 30 2>&1 | tail -1)" >> $OUT || exit 1
  done
  echo "P=$P W=helmet tex4 $(PT_LIBPT=$PWD/build_variants/tex4/libpt.so PT_PRIO_TILES=$P timeout -k 10 120 python tools/exp_timing.py --workload helmet --backends megakernel --layouts pairs --no-mesh-variant --frames 30 2>&1 | tail -1)" >> $OUT || exit 1
done
