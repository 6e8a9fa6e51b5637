#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output into profiles/pmc_<workload>.json.

Per kernel: every counter averaged over its dispatches (the passes are separate runs of the same
frames). For the path-tracing kernel (the bench's roofline kernel) the HBM traffic per launch is
derived as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) doubled (gfx950 tallies 128-B
read requests at 64 B) plus WRITE_SIZE (KiB), times 1024. FETCH_SIZE counts L2 misses that the
Infinity Cache serves too, so this is L2-to-fabric traffic, an upper bound on HBM bytes.

usage: pmc_summary.py <gpurun_out/pmc_TAG> <workload> [note]
"""
import collections
import csv
import glob
import json
import os
import sys

src, workload = sys.argv[1], sys.argv[2]
note = sys.argv[3] if len(sys.argv) > 3 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = int(r["Dispatch_Id"])
            names[key] = r["Kernel_Name"]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, cs in per.items():
        for c, v in cs.items():
            acc[names[d]][c].append(v)

kernels = {}
for k, cs in acc.items():
    kernels[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    kernels[k]["dispatches"] = max(len(v) for v in cs.values())

trace = [k for k in kernels if "pt_trace<" in k or "pt_persist<" in k]
main = max(trace, key=lambda k: kernels[k].get("GRBM_GUI_ACTIVE", 0.0)) if trace else None
out = {"note": note or "rocprofv3 --pmc passes of tools/gpu_pmc.sh (tools/prof_frames.py, bench workload)",
       "workload": workload, "kernel": main, "kernels": kernels}
if main and "FETCH_SIZE" in kernels[main] and "WRITE_SIZE" in kernels[main]:
    m = kernels[main]
    out["hbm_bytes_per_launch"] = int((2.0 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024)
    out["hbm_bytes_formula"] = "(2 x FETCH_SIZE + WRITE_SIZE) x 1024, per launch"
    if "TCC_HIT_sum" in m:
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_%s.json" % workload)
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", dst, "kernel", main, "hbm_bytes_per_launch", out.get("hbm_bytes_per_launch"))
