"""The native BVH builder (libpt pt_bvh_build, csrc/pt_bvh_build.cpp) against the reference's own
BVH_Fast_Builder.js output: same input (the per-triangle AABB array the setup script hands to
BVH_Build_Iterative, captured by tests/golden/gen), same tree, bit for bit. Host code: runs on CPU."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import helpers as H


@pytest.mark.parametrize("key", ["teapot", "duck", "helmet", "bunny"])
def test_native_builder_matches_reference_bits(key):
    import babylon_pt as bp
    m = np.load(os.path.join(H.GOLD, "mesh_%s.npz" % key))
    out = bp.bvh_build(m["aabb_in"])
    assert out.shape == m["bvh"].shape
    assert np.array_equal(out.view(np.uint32), m["bvh"].view(np.uint32))


def test_native_builder_degenerate_inputs():
    """Coincident centroids (no axis separates them: the alternate deal) and a single triangle."""
    import babylon_pt as bp
    box = np.array([0, 0, 0, 1, 1, 1, 0.5, 0.5, 0.5], np.float32)
    same = np.tile(box, (5, 1))
    out = bp.bvh_build(same)
    assert out.shape == (9, 8)
    # alternate deals: {0..4} -> {0,2,4} | {1,3}; {0,2,4} -> {0,4} | {2}; depth-first, left first
    assert out[:, 0].tolist() == [-1, -1, -1, 0, 4, 2, -1, 1, 3]
    assert out[:, 4].tolist() == [6, 5, 4, -1, -1, -1, 8, -1, -1]
    one = bp.bvh_build(box[None])
    assert one.shape == (1, 8) and one[0, 0] == 0 and one[0, 4] == -1


REF = os.environ.get("PT_REFERENCE", "/root/reference")


@pytest.mark.skipif(not (os.path.isdir(os.path.join(REF, "js")) and shutil.which("node")),
                    reason="needs the reference scripts and node (build container)")
def test_setup_script_with_native_builder_uploads_the_same_texture():
    """The unmodified glTF setup script with BVH_Build_Iterative swapped for the native builder
    uploads exactly the tAABBTexture the reference builder produced."""
    import hashlib
    meta = H.stream("gltf_teapot_320x180")
    cmd = ["node", os.path.join(H.ROOT, "tests", "js", "dropin_check.js"), "gltf", "320", "180", "3",
           str(meta["seed"]), meta["model"]]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, PT_NATIVE_BVH="1")).stdout
    got = json.loads(out)
    payload = H.texture_payloads(meta, H.mesh(meta))
    assert hashlib.sha256(payload["bvh"].tobytes()).hexdigest() in got["raw_sha256"]
