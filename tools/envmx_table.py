#!/usr/bin/env python3
"""Table of a gpu_env_matrix.sh log: min ms per launch per (setting, workload) over the rounds."""
import collections
import json
import re
import sys

d = collections.defaultdict(list)
cfgs, wls = [], []
for line in open(sys.argv[1]):
    m = re.match(r'r(\d+) \[(.*?)\] (\S+) (\{.*\})', line)
    if not m:
        continue
    cfg = m.group(2).split('/')[-2] if 'LIBPT' in m.group(2) else m.group(2)
    if cfg not in cfgs:
        cfgs.append(cfg)
    if m.group(3) not in wls:
        wls.append(m.group(3))
    d[(cfg, m.group(3))].append(json.loads(m.group(4))['ms_per_launch'])
print("%-22s" % "ms (min of rounds)" + "".join("%12s" % w for w in wls))
for c in cfgs:
    print("%-22s" % c + "".join("%12.4f" % min(d[(c, w)]) if d[(c, w)] else "%12s" % "-" for w in wls))
