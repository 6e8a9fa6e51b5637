#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the path-tracing kernel: the tree against build_variants/lean (AoS G-buffer)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in lean tree; do
  L=""; [ $lib = lean ] && L="$R/build_variants/lean/libpt.so"
  for w in dragon bunny; do
    i=0
    for C in "WRITE_SIZE" "FETCH_SIZE"; do
      i=$((i+1))
      PT_LIBPT=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$R/gpurun_out/pmc_r04o_${lib}_$w/p$i" -o run -- python3 "$R/tools/prof_frames.py" --workload $w --frames 10 > "$R/gpurun_out/pmc_r04o_${lib}_$w.p$i.log" 2>&1 || exit $?
    done
  done
done
