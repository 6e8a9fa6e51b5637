#!/usr/bin/env python3
"""BVH build time: the host builder (pt_bvh_build, one core) against the device build
(pt_bvh_build_gpu: device time of the level loop, and wall time with uploads and read-back),
bit-identical outputs checked, for the reference meshes and the 524,288-triangle dragon stand-in.
One JSON line per mesh."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import babylon_pt as bp  # noqa: E402
import helpers as H      # noqa: E402

meshes = {k: np.load(os.path.join(H.GOLD, "mesh_%s.npz" % k))["aabb_in"] for k in ("teapot", "helmet", "bunny")}
meshes["dragon_standin"] = H.synthetic_dragon()["aabb_in"]
bp.bvh_build_gpu(meshes["teapot"])   # device init outside the timings
for name, aabb in meshes.items():
    t0 = time.perf_counter(); host = bp.bvh_build(aabb); t_host = time.perf_counter() - t0
    walls, devs = [], []
    for _ in range(5):
        t0 = time.perf_counter(); dev, ms = bp.bvh_build_gpu(aabb); walls.append(time.perf_counter() - t0); devs.append(ms)
    print(json.dumps({"mesh": name, "triangles": int(aabb.shape[0]), "nodes": int(host.shape[0]),
                      "bit_identical": bool(np.array_equal(host.view(np.uint32), dev.view(np.uint32))),
                      "host_ms": round(t_host * 1e3, 2), "device_ms": round(min(devs), 3),
                      "device_wall_ms": round(min(walls) * 1e3, 2)}), flush=True)
