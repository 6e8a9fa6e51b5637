#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy of a HIP source (clang's kernel-resource-usage remarks)."""
import re
import subprocess
import sys

src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-fast-math", "-c", "-o", "/tmp/kres.o", src, "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
for r in rows:
    print("%-70s vgpr %3s scratch %4s occ %s lds %s" % (r["name"][:70], r.get("VGPRs"), r.get("ScratchSize"),
                                                       r.get("Occupancy"), r.get("LDS")))
