cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; O=gpurun_out/ev_ab.log; : > $O
for r in 1 2 3; do for w in dragon bunny; do for e in "" 1; do
PT_BENCH_NO_EVENTS=$e timeout -k 10 200 python bench.py --workload $w --steps 400 --warmup 20 --cpu-budget 0 --no-pmc > gpurun_out/ev_tmp.json 2>>$O || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/ev_tmp.json').read().strip().splitlines()[-1]); print('$w noev=$e r$r', d['ms_per_step'])" >> $O
done; done; done
