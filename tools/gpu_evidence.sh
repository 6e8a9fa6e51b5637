#!/bin/bash
# One evidence session for a tree: smoke(), the GPU parity suite, the driver's exact bench command, bench.py on
# every workload, a rocprofv3 kernel trace + stats of the default bench, and the PMC passes of the
# dragon stand-in (tools/gpu_pmc.sh groups). Every GPU step has its own time limit; anything but
# pytest's 0 ends the session. usage: gpu_evidence.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_exact.json 2> gpurun_out/bench_${TAG}_exact.err || exit $?
for W in helmet bunny sky_dragon bunny16; do
  timeout -k 10 300 python3 bench.py --workload $W > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || exit $?
done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_dragon.json 2> gpurun_out/bench_${TAG}_dragon.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 --cpu-budget 0 --no-pmc --no-anchors > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/prof_frames.py" --workload dragon --frames 10 > "$OUT/p$i.log" 2>&1 || exit $?
done
echo "evidence $TAG done" > "$R/gpurun_out/evidence_$TAG.done"
