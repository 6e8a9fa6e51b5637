"""The JavaScript host path on the GPU: recorded reference streams replayed through the Babylon
effect-API shim (js/babylon_pt.js) and the N-API addon onto libpt.so, bit-exact vs the oracle."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import helpers as H

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not shutil.which("node"), reason="node not installed")]
REPLAY = os.path.join(H.ROOT, "babylon.js-pathtracing-renderer_amd", "js", "replay_stream.js")


@pytest.mark.parametrize("name", ["cornell_256", "sky_256", "quadric_256", "gltf_teapot_320x180", "hdri_teapot_320x180"])
def test_node_replay_bitexact(tmp_path, name):
    meta = H.stream(name)
    H.bluenoise().tofile(tmp_path / "bluenoise.u8")
    if meta["scene"] in ("gltf", "hdri"):
        for k, v in H.texture_payloads(meta, H.mesh(meta)).items():
            v.tofile(tmp_path / (k + ".f32"))
    out = str(tmp_path / "out")
    subprocess.run(["node", REPLAY, os.path.join(H.GOLD, name + ".json"), str(tmp_path), out],
                   check=True, timeout=300)
    w, h = meta["width"], meta["height"]
    acc = np.fromfile(out + ".acc.f32", np.float32).reshape(h, w, 4)
    can = np.fromfile(out + ".canvas.u8", np.uint8).reshape(h, w, 4)
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True)
    assert np.array_equal(acc.view(np.uint32), ref_acc[-1].view(np.uint32))
    assert np.array_equal(can, ref_can[-1])


def test_node_replay_gltf_pbr_maps_bitexact(tmp_path):
    """The helmet stream through Node with its four PBR maps bound the way Babylon's glTF loader
    leaves them (textures holding JPEG file bytes): the shim decodes and uploads them at
    setTexture, and the frames match the oracle rendering the same decoded maps."""
    import io
    import json
    from PIL import Image
    import pt_assets
    meta = H.stream("gltf_helmet_320x180")
    H.bluenoise().tofile(tmp_path / "bluenoise.u8")
    for k, v in H.texture_payloads(meta, H.mesh(meta)).items():
        v.tofile(tmp_path / (k + ".f32"))
    maps, decoded, spec = H.synthetic_pbr_maps(), {}, {}
    for kind, sampler in H.PBR_SAMPLERS.items():
        buf = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(maps[kind][..., :3])).save(buf, "JPEG", quality=90)
        f = tmp_path / (kind + ".jpg")
        f.write_bytes(buf.getvalue())
        spec[sampler] = str(f)
        decoded[kind] = pt_assets.decode_rgba8(buf.getvalue())
    (tmp_path / "maps.json").write_text(json.dumps(spec))
    out = str(tmp_path / "out")
    subprocess.run(["node", REPLAY, os.path.join(H.GOLD, "gltf_helmet_320x180.json"), str(tmp_path), out],
                   check=True, timeout=300)
    w, h = meta["width"], meta["height"]
    acc = np.fromfile(out + ".acc.f32", np.float32).reshape(h, w, 4)
    can = np.fromfile(out + ".canvas.u8", np.uint8).reshape(h, w, 4)
    ref_acc, ref_can, _ = H.oracle_replay(meta, with_output=True, maps=decoded)
    assert np.array_equal(acc.view(np.uint32), ref_acc[-1].view(np.uint32))
    assert np.array_equal(can, ref_can[-1])
