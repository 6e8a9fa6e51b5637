#!/bin/bash
# objectColor recomputed from the bounce-0 id instead of stored (build_variants/colid) against the
# tree before (build_variants/base_s): GPU parity suite, kernel time, WRITE_SIZE / FETCH_SIZE
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
PT_LIBPT=build_variants/colid/libpt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r04s.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_r04s.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_env_matrix.sh r04s "dragon bunny bunny16" 3 "PT_LIBPT=build_variants/base_s/libpt.so" "PT_LIBPT=build_variants/colid/libpt.so" || exit $?
cd /tmp && export TMPDIR=/tmp
for lib in base_s colid; do
  for w in dragon bunny; do
    i=0
    for C in "WRITE_SIZE" "FETCH_SIZE"; do
      i=$((i+1))
      PT_LIBPT=$R/build_variants/$lib/libpt.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$R/gpurun_out/pmc_r04s_${lib}_$w/p$i" -o run -- python3 "$R/tools/prof_frames.py" --workload $w --frames 10 > "$R/gpurun_out/pmc_r04s_${lib}_$w.p$i.log" 2>&1 || exit $?
    done
  done
done
