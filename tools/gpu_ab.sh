#!/bin/bash
# A/B of the path-tracing kernel time over workloads: the in-tree build and every
# build_variants/<name>/libpt.so, alternating rounds (bench.py, no CPU baseline, no PMC).
# usage: gpu_ab.sh TAG "dragon helmet bunny" [rounds]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-ab}; WLS=${2:-"dragon helmet bunny"}; ROUNDS=${3:-2}
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.log
: > $OUT
for round in $(seq $ROUNDS); do
  for d in base build_variants/*/; do
    n=$(basename $d)
    [ "$n" = secprof ] && continue
    lib=""; [ "$d" != base ] && lib=$PWD/$d/libpt.so
    for w in $WLS; do
      PT_LIBPT=$lib timeout -k 10 200 python bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 0 --no-pmc --no-anchors > gpurun_out/ab_tmp.json 2>>$OUT || exit $?
      python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); print('$n $w r$round', d['value'], d['ms_per_step'], d['kernel_ms']['pathtrace'], d['kernel_ms']['screen_output'], d['kernel_ms']['screen_copy'])" >> $OUT
    done
  done
done
python3 - "$OUT" <<'PY' >> $OUT
import sys, collections
r = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 6 and p[2].startswith('r'):
        r[(p[0], p[1])].append(float(p[5]))
print("summary (min kernel ms over rounds):")
for (n, w), v in sorted(r.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print("  %-12s %-10s %.4f" % (w, n, min(v)))
PY
