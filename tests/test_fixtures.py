"""The reference-run fixtures (tests/golden, made by tests/golden/gen from the reference's own
JavaScript) are intact and have the layout the hot path relies on.

These pin the data-format side of the oracle: the BVH / triangle textures are exactly what
BVH_Build_Iterative (js/BVH_Fast_Builder.js:327-407) and Prepare_Model_For_PathTracing
(js/GLTF_Model_Path_Tracing.js:287-497) produce, and the uniform streams are exactly what the
setup scripts push through effect.set* (js/GLTF_Model_Path_Tracing.js:813-848).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import helpers as H

MANIFEST = json.load(open(os.path.join(H.GOLD, "MANIFEST.json")))
MESHES = ["teapot", "bunny", "duck", "helmet"]


@pytest.mark.parametrize("key", MESHES)
def test_mesh_hashes(key):
    m = H.mesh(key)
    man = MANIFEST["mesh_" + key]
    assert hashlib.sha256(m["bvh"].tobytes()).hexdigest() == man["sha256_bvh"]
    assert hashlib.sha256(m["tri"].tobytes()).hexdigest() == man["sha256_tri"]
    assert m["tri"].shape == (man["triangles"], 32)
    assert m["bvh"].shape == (2 * man["triangles"] - 1, 8)


@pytest.mark.parametrize("key", MESHES)
def test_bvh_layout_invariants(key):
    """Depth-first order, left child = n+1, right child index in texel .x of slot 1, one triangle
    per leaf, every triangle in exactly one leaf, leaf box = its triangle's f32 bounds, inner box
    = union of children, depth within stackLevels[28]."""
    m = H.mesh(key)
    bvh, tri = m["bvh"], m["tri"]
    n = bvh.shape[0]
    inner = bvh[:, 0] < 0
    leaves = np.nonzero(~inner)[0]
    ids = bvh[leaves, 0].astype(np.int64)
    assert np.array_equal(np.sort(ids), np.arange(tri.shape[0]))
    assert np.all(bvh[leaves, 4] == -1)
    right = bvh[inner, 4].astype(np.int64)
    idx = np.nonzero(inner)[0]
    assert np.all(right > idx + 1) and np.all(right < n)
    for node, r in zip(idx, right):
        for c in (node + 1, r):
            assert np.all(bvh[node, 1:4] <= bvh[c, 1:4]) and np.all(bvh[node, 5:8] >= bvh[c, 5:8])
    p = tri[ids][:, :9].reshape(-1, 3, 3)
    assert np.array_equal(bvh[leaves, 1:4], p.min(axis=1))
    assert np.array_equal(bvh[leaves, 5:8], p.max(axis=1))
    assert MANIFEST["mesh_" + key]["depth"] <= 28


@pytest.mark.parametrize("key", MESHES)
def test_triangle_records(key):
    """32-float records: normals unit length, unused PBR slots zero (js/GLTF_Model_Path_Tracing.js:374-423)."""
    tri = H.mesh(key)["tri"]
    for a, b in ((9, 12), (12, 15), (15, 18)):
        nrm = np.linalg.norm(tri[:, a:b].astype(np.float64), axis=1)
        assert np.all(np.abs(nrm - 1.0) < 1e-5)
    assert np.all(tri[:, 24:32] == 0)


def test_bluenoise_fixture():
    bn = H.bluenoise()
    assert bn.shape == (256, 256, 4) and bn.dtype == np.uint8
    assert len(np.unique(bn[..., 0])) > 200    # blue noise covers the byte range


@pytest.mark.parametrize("name", ["cornell_256", "gltf_bunny_1080p", "gltf_teapot_320x180", "gltf_helmet_320x180", "sky_256"])
def test_stream_frame_semantics(name):
    """3 draws per frame (pathTracing -> screenCopy -> screenOutput); counters follow the loop at
    js/GLTF_Model_Path_Tracing.js:1191-1220."""
    meta = H.stream(name)
    for f in meta["frames"]:
        assert [c["shader"] for c in f] == ["pathTracingFragmentShader", "screenCopyFragmentShader", "screenOutputFragmentShader"]
        assert [c["target"] for c in f] == ["pathTracingRenderTarget", "screenCopyRenderTarget", None]
        pt, cp, out = f
        assert pt["samplers"]["previousBuffer"] == "screenCopyRenderTarget"
        assert cp["samplers"]["pathTracedImageBuffer"] == "pathTracingRenderTarget"
        assert out["samplers"]["accumulationBuffer"] == "pathTracingRenderTarget"
        s = pt["uniforms"]["uSampleCounter"][1][0]
        assert out["uniforms"]["uOneOverSampleCounter"][1][0] == pytest.approx(1.0 / s)
        w, h = pt["uniforms"]["uResolution"][1]
        assert (w, h) == (meta["width"], meta["height"])
        assert pt["uniforms"]["uULen"][1][0] == pytest.approx(pt["uniforms"]["uVLen"][1][0] * w / h)
    first = meta["frames"][0][0]["uniforms"]
    assert first["uCameraIsMoving"][1][0] == 1


def test_cornell_defaults():
    """Config 1 defaults (js/Babylon_Path_Tracing.js:242-272): camera (0,-20,-120), light on the ceiling."""
    u = H.stream("cornell_256")["frames"][0][0]["uniforms"]
    assert u["uCameraMatrix"][1][12:15] == [0, -20, -120]
    assert u["uQuadLightPlaneSelectionNumber"][1][0] == 6
    assert u["uRightSphereMatType"][1][0] == 3
    assert u["uFrameCounter"][1][0] == 1


def test_helmet_maps_are_the_reference_jpegs():
    """tests/golden/helmet_maps holds the four maps the helmet's material binds, byte for byte the
    reference's models/materials/DamagedHelmet/*.jpg (sha256 below, taken from the reference tree),
    and they decode to 2048x2048 RGBA8."""
    import hashlib
    want = {"Default_albedo.jpg": "2dc95e87aeb0cd7c8a65ef0eb8b23212388da0534ca379811427a9a8780511f5",
            "Default_emissive.jpg": "dd0057989f22f93a4ab796d06ebf85a7c12fbfae1d59a86ae8b0c54770dc1159",
            "Default_metalRoughness.jpg": "0f05e7ffbeaa974f7d2c83436b04109969966d64ab188cbc3a19a265a0a69ae0",
            "Default_normal.jpg": "f253ba09a90a86ffd8a807dc45d7953111f8b3421e15d7a21d1e915b01dd33c1"}
    for name, sha in want.items():
        with open(os.path.join(H.GOLD, "helmet_maps", name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == sha, name
    maps = H.helmet_maps()
    assert sorted(maps) == sorted(H.PBR_SAMPLERS)
    assert all(m.shape == (2048, 2048, 4) and m.dtype == np.uint8 for m in maps.values())
