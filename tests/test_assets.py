"""The asset pipeline restatement (python/pt_assets.py) against the reference's
own output: every model in the reference's models/ directory, loaded by the reference's setup script
(Babylon glTF loader -> MergeMeshes -> convertToUnIndexedMesh -> Prepare_Model_For_PathTracing ->
BVH_Build_Iterative under Node, tests/golden/gen/make_fixtures.js), must come out bit-identical:
the triangle texture records, the builder's per-triangle AABB input and the BVH texture.

The model files are read from /root/reference/models (this container only); the synthetic-GLB
tests below need nothing from the reference.
"""
import json
import os
import struct

import numpy as np
import pytest

import helpers as H

import pt_assets as A

MODELS = "/root/reference/models"
CASES = [  # fixture key, model file, modelInitialScale, modelWasDefinedInRHCoordSystem
    ("teapot",) + (A.MODEL_PRESETS["Utah Teapot"][0], A.MODEL_PRESETS["Utah Teapot"][2], A.MODEL_PRESETS["Utah Teapot"][1]),
    ("bunny",) + (A.MODEL_PRESETS["Stanford Bunny"][0], A.MODEL_PRESETS["Stanford Bunny"][2], A.MODEL_PRESETS["Stanford Bunny"][1]),
    ("duck",) + (A.MODEL_PRESETS["glTF Duck"][0], A.MODEL_PRESETS["glTF Duck"][2], A.MODEL_PRESETS["glTF Duck"][1]),
    ("helmet",) + (A.MODEL_PRESETS["Damaged Helmet"][0], A.MODEL_PRESETS["Damaged Helmet"][2], A.MODEL_PRESETS["Damaged Helmet"][1]),
    ("bookcase", "testBookCase.gltf", 8.0, False),   # 150 meshes, mixed attribute sets
    ("twoparts", "twoParts-opaque.gltf", 25.0, False),
]


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("key,file,scale,rh", CASES, ids=[c[0] for c in CASES])
def test_model_pipeline_bitexact(key, file, scale, rh):
    path = os.path.join(MODELS, file)
    if not os.path.exists(path):
        pytest.skip("reference models not present (build container only)")
    gold = np.load(os.path.join(H.GOLD, "mesh_%s.npz" % key))
    m = A.load_model(path, scale, rh, build_bvh=True)
    for k in ("tri", "aabb_in", "bvh"):
        assert m[k].shape == gold[k].shape, k
        bad = _bits(m[k]) != _bits(gold[k])
        assert not bad.any(), "%s: %d of %d words differ, first at %s" % (k, bad.sum(), bad.size, np.argwhere(bad)[0])


def test_model_presets_match_the_menu():
    """MODEL_PRESETS restates the menu handler (js/GLTF_Model_Path_Tracing.js:891-923); the
    fixture streams were recorded through that menu with these scales."""
    for key, name in (("teapot", "gltf_teapot_320x180"), ("bunny", "gltf_bunny_1080p"), ("duck", "gltf_duck_320x180"),
                      ("helmet", "gltf_helmet_320x180")):
        meta = H.stream(name)
        preset = A.MODEL_PRESETS[meta["model"]]
        assert preset[2] == meta["modelScale"], (key, preset, meta["modelScale"])


def test_material_maps():
    path = os.path.join(MODELS, "DamagedHelmet.gltf")
    if not os.path.exists(path):
        pytest.skip("reference models not present (build container only)")
    gj, buffers = A.load_gltf(path)
    maps = A.material_maps(gj)
    assert set(maps) == {"albedo", "bump", "metal", "emissive"}   # uModelUses*Texture all true
    img = A.decode_rgba8(A.image_bytes(gj, buffers, maps["albedo"], MODELS))
    assert img.dtype == np.uint8 and img.ndim == 3 and img.shape[2] == 4
    duck, _ = A.load_gltf(os.path.join(MODELS, "Duck.gltf"))
    assert set(A.material_maps(duck)) == {"albedo"}


# ------------------------------------------------------------------------------ synthetic GLB
def _glb(gj, blob):
    js = json.dumps(gj).encode()
    js += b" " * (-len(js) % 4)
    blob += b"\0" * (-len(blob) % 4)
    body = struct.pack("<II", len(js), 0x4E4F534A) + js + struct.pack("<II", len(blob), 0x004E4942) + blob
    return struct.pack("<III", 0x46546C67, 2, 12 + len(body)) + body


def _two_triangle_glb(tmp_path, node_extra, indices):
    pos = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0], [0, 0, 3]], np.float32)
    nrm = np.array([[0, 0, 2], [0, 0, 1], [0, 0, 1], [1, 1, 1]], np.float32)
    idx = np.array(indices, np.uint16)
    blob = pos.tobytes() + nrm.tobytes() + idx.tobytes()
    gj = {"asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": [0]}],
          "nodes": [dict({"children": [1]}, **node_extra), {"mesh": 0, "translation": [1.0, 2.0, 3.0]}],
          "meshes": [{"primitives": [{"attributes": {"POSITION": 0, "NORMAL": 1}, "indices": 2}]}],
          "buffers": [{"byteLength": len(blob)}],
          "bufferViews": [{"buffer": 0, "byteOffset": 0, "byteLength": 48}, {"buffer": 0, "byteOffset": 48, "byteLength": 48},
                          {"buffer": 0, "byteOffset": 96, "byteLength": 2 * len(indices)}],
          "accessors": [{"bufferView": 0, "componentType": 5126, "count": 4, "type": "VEC3"},
                        {"bufferView": 1, "componentType": 5126, "count": 4, "type": "VEC3"},
                        {"bufferView": 2, "componentType": 5123, "count": len(indices), "type": "SCALAR"}]}
    p = tmp_path / "m.glb"
    p.write_bytes(_glb(gj, blob))
    return str(p), pos, nrm


def test_synthetic_glb_transforms(tmp_path):
    """A two-level hierarchy (scaled parent, translated child): positions = (child x parent x
    __root__) applied in float64 and rounded once, x negated by the root, RH z flip, the model
    scale, normals renormalised, no UVs (2 vertex kinds -> -1)."""
    path, pos, nrm = _two_triangle_glb(tmp_path, {"scale": [2.0, 2.0, 2.0]}, [0, 1, 2, 0, 2, 3])
    m = A.load_model(path, 10.0, True, build_bvh=False)
    tri = m["tri"]
    assert tri.shape == (2, 32)
    # world: scale 2 then translate (2,4,6) (child translation scaled by the parent), x negated
    w = (pos.astype(np.float64) + [1.0, 2.0, 3.0]) * 2.0
    w[:, 0] *= -1
    # 6 indices != 4 vertices -> unindexed; the root's negative determinant flips each face
    order = [0, 2, 1, 0, 3, 2]
    exp = w[order]
    exp[:, 2] *= -1
    exp = (exp * 10.0).astype(np.float32).reshape(2, 9)
    assert np.array_equal(tri[:, 0:9], exp)
    n = nrm.astype(np.float64)[order] * 2.0
    n[:, 0] *= -1
    n[:, 2] *= -1
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    assert np.allclose(tri[:, 9:18].reshape(-1, 3), n, rtol=0, atol=1e-7)
    assert (tri[:, 18:24] == -1).all() and (tri[:, 24:] == 0).all()
    a = m["aabb_in"]
    assert np.array_equal(a[:, 0:3], tri[:, 0:9].reshape(2, 3, 3).min(1))
    assert np.array_equal(a[:, 3:6], tri[:, 0:9].reshape(2, 3, 3).max(1))


def test_synthetic_glb_matrix_node(tmp_path):
    """A node.matrix is decomposed and recomposed (Matrix.decompose + ComposeToRef) before it
    joins the chain; 3 indices over 4 vertices -> unindexed, the face flipped by the root."""
    mat = [0.5, 0, 0, 0, 0, 0.5, 0, 0, 0, 0, 0.5, 0, 7, 0, 0, 1]
    path, pos, _ = _two_triangle_glb(tmp_path, {"matrix": mat}, [2, 1, 0])
    gj, buffers = A.load_gltf(path)
    p, n, uv, kinds = A.merged_vertices(gj, buffers)
    assert kinds == 2 and uv is None
    w = (pos.astype(np.float64) + [1.0, 2.0, 3.0]) * 0.5 + [7.0, 0, 0]
    w[:, 0] *= -1
    assert np.array_equal(p, w.astype(np.float32)[[2, 0, 1]])


def test_texture_arrays_layout():
    gold = np.load(os.path.join(H.GOLD, "mesh_teapot.npz"))
    t = A.texture_arrays({"bvh": gold["bvh"], "tri": gold["tri"]})
    ref = H.texture_payloads({"scene": "gltf"}, {"bvh": gold["bvh"], "tri": gold["tri"]})
    for k in ("bvh", "tri"):
        assert t[k].shape == (4 * 2048 * 2048,) and np.array_equal(_bits(t[k]), _bits(ref[k]))


# ------------------------------------------------------------------------------ HDR environment
@pytest.mark.parametrize("w,h", [(64, 16), (5, 3)])   # RLE scanlines, flat scanlines (w < 8)
def test_decode_hdr_matches_rgbe(tmp_path, w, h):
    rng = np.random.default_rng(w)
    img = rng.exponential(2.0, (h, w, 3)) * (rng.random((h, w, 1)) < 0.8)
    img[0, :4] = 7.0   # runs
    rgbe = H.rgbe_encode(img)
    p = tmp_path / "e.hdr"
    if w >= 8:
        H.write_radiance_hdr(str(p), rgbe)
    else:
        p.write_bytes(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + ("-Y %d +X %d\n" % (h, w)).encode() + rgbe.tobytes())
    got = A.decode_hdr(p.read_bytes())
    assert np.array_equal(_bits(got), _bits(H.rgbe_decode(rgbe)))


def test_hdr_sun_direction_matches_the_script():
    """The HDRI setup script derived uSunDirection from synthetic_hdr() when the fixture streams
    were recorded; the uniform (float32) must be reproduced exactly."""
    d = A.hdr_sun_direction(H.synthetic_hdr())
    for name in ("hdri_teapot_320x180", "hdri_helmet_320x180"):
        u = H.path_call(H.stream(name)["frames"][0])["uniforms"]["uSunDirection"][1]
        assert np.array_equal(np.float32(u), np.float32(d)), (u, d)
