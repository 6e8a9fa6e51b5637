#!/usr/bin/env python3
"""Summarise a tools/gpu_variants.sh log: per variant and workload, the per-launch path-tracing ms
of each round and their mean. usage: variants_summary.py gpurun_out/variants_TAG.log"""
import collections
import json
import sys

runs = collections.defaultdict(list)
key = None
for line in open(sys.argv[1]):
    if line.startswith("== "):
        name, wl = line.split()[1:3]
        key = (name, wl)
    elif line.startswith("{") and key:
        runs[key].append(json.loads(line)["ms_per_launch"])
wls = sorted({k[1] for k in runs})
names = sorted({k[0] for k in runs}, key=lambda n: (n != "base", n))
print("%-16s" % "variant" + "".join("%22s" % w for w in wls))
for n in names:
    cells = []
    for w in wls:
        v = runs.get((n, w), [])
        cells.append("%22s" % ("%.4f (%s)" % (sum(v) / len(v), "/".join("%.3f" % x for x in v)) if v else "-"))
    print("%-16s" % n + "".join(cells))
