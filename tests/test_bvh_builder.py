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


# ---- the device build (pt_bvh_build_gpu, csrc/pt_bvh_gpu.hip): the same tree, bit for bit

def _same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["teapot", "duck", "helmet", "bunny"])
def test_gpu_builder_matches_reference_bits(key):
    import babylon_pt as bp
    m = np.load(os.path.join(H.GOLD, "mesh_%s.npz" % key))
    out, ms = bp.bvh_build_gpu(m["aabb_in"])
    assert _same_bits(out, m["bvh"])
    assert ms > 0.0


@pytest.mark.gpu
def test_gpu_builder_dragon_standin_matches_host_builder():
    """524,288 triangles: the bench's mesh, device build == host build."""
    import babylon_pt as bp
    d = H.synthetic_dragon()
    out, ms = bp.bvh_build_gpu(d["aabb_in"])
    assert _same_bits(out, d["bvh"])


def _aabbs(lo, hi):
    c = (lo + hi) * np.float32(0.5)
    return np.concatenate([lo, hi, c], 1).astype(np.float32)


@pytest.mark.gpu
def test_gpu_builder_degenerate_and_edge_inputs():
    """Coincident centroids (alternate deals), one and two triangles, a permuted and partial work
    list, duplicates, signed zeros, infinities and NaN bounds: device == host, bit for bit."""
    import babylon_pt as bp
    rng = np.random.default_rng(7)
    cases = []
    box = np.array([0, 0, 0, 1, 1, 1, 0.5, 0.5, 0.5], np.float32)
    cases.append((np.tile(box, (5, 1)), None))
    cases.append((box[None], None))
    cases.append((np.tile(box, (2, 1)), None))
    lo = rng.normal(size=(3000, 3)).astype(np.float32)
    hi = lo + rng.random((3000, 3)).astype(np.float32)
    a = _aabbs(lo, hi)
    cases.append((a, None))
    cases.append((a, rng.permutation(3000).astype(np.uint32)))           # permuted work list
    cases.append((a, rng.permutation(3000)[:1777].astype(np.uint32)))    # a subset
    dup = a.copy(); dup[1000:2000] = dup[0]                                # duplicates
    cases.append((dup, None))
    z = a.copy(); z[::7, 0] = -0.0; z[1::7, 3] = 0.0; z[2::7, 0] = 0.0; z[3::7, 3] = -0.0   # signed zeros
    cases.append((z, None))
    inf = a.copy(); inf[5, 3] = np.inf; inf[9, 1] = -np.inf
    cases.append((inf, None))
    nan = a.copy(); nan[17, 2] = np.nan; nan[400, 4] = np.nan; nan[2500, 7] = np.nan   # NaN bounds, a NaN centroid
    cases.append((nan, None))
    clus = _aabbs(*(lambda l: (l, l + np.float32(1e-3)))(np.repeat(rng.normal(size=(20, 3)), 100, 0).astype(np.float32)))
    cases.append((clus, None))
    for aabb, work in cases:
        want = bp.bvh_build(aabb, work)
        got, _ = bp.bvh_build_gpu(aabb, work)
        assert _same_bits(got, want), (aabb.shape, None if work is None else work.shape)
