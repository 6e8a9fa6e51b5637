"""Pack the reference-run fixtures into tests/golden/ (build container only).

Runs ``make_fixtures.js`` (which executes the reference's own babylon.js / glTF loader /
BVH_Fast_Builder.js / setup scripts from /root/reference under Node) and stores the numeric
outputs as small fixtures:

  tests/golden/<name>.json         per-frame render-call stream (uniforms, samplers, targets)
  tests/golden/mesh_<model>.npz    bvh (2N-1, 8) f32 and tri (N, 32) f32: the exact payloads the
                                   setup script hands to RawTexture.CreateRGBATexture
  tests/golden/bluenoise_rgba8.npy 256x256x4 u8: textures/BlueNoise_RGBA256.png (16-bit/channel)
                                   reduced to the 8-bit texels WebGL samples. Pinned convention:
                                   high byte (v16 >> 8), see DESIGN.md.

  The HDRI streams run HDRI_Environment_Path_Tracing.js on the synthetic environment of
  browser_env.js syntheticHDR (== tests/helpers.py synthetic_hdr; the reference's .hdr files are
  not in it); the stream records that texture's sha256, the payload itself is regenerated.

  tests/golden/controls_<scene>.json  the same stream with the render loop's inputs driven

usage: python tests/golden/gen/make_fixtures.py [stream names | mesh_<model fixture> ...]   (default: all)
"""
import sys
import hashlib
import json
import os
import struct
import subprocess
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.dirname(HERE)
REF = os.environ.get("PT_REFERENCE", "/root/reference")

STREAMS = [
    # name, scene, width, height, frames, seed, model
    ("cornell_256", "cornell", 256, 256, 4, 1, None),
    ("sky_256", "sky", 256, 256, 3, 3, None),
    ("gltf_teapot_320x180", "gltf", 320, 180, 3, 5, "Utah Teapot"),
    ("gltf_bunny_1080p", "gltf", 1920, 1080, 4, 1, "Stanford Bunny"),
    ("gltf_duck_320x180", "gltf", 320, 180, 3, 7, "glTF Duck"),
    ("gltf_helmet_320x180", "gltf", 320, 180, 3, 9, "Damaged Helmet"),
    ("hdri_teapot_320x180", "hdri", 320, 180, 3, 11, "Utah Teapot"),
    ("hdri_helmet_320x180", "hdri", 320, 180, 3, 13, "Damaged Helmet"),
    ("quadric_256", "quadric", 256, 256, 3, 17, None),
]
# the Cornell render loop driven through its own input state (make_fixtures.js PT_CONTROLS): WASD/QE
# flight, opposing keys, mouse-wheel FOV, a pointer-lock camera rotation, focus distance and
# aperture keys (aperture clamped at 0), then still frames. Pins python/pt_controls.py.
def _controls_script():
    c = [dict() for _ in range(40)]
    c[2] = {"down": ["w"]}
    c[5] = {"up": ["w"]}
    c[6] = {"down": ["d"]}
    c[7] = {"down": ["e"]}
    c[9] = {"up": ["d", "e"]}
    c[10] = {"down": ["a", "d"]}
    c[11] = {"up": ["a", "d"]}
    c[12] = {"wheel": 1}
    c[13] = {"wheel": 1}
    c[14] = {"wheel": -1}
    c[15] = {"rot": [0.1, 0.3]}
    c[16] = {"down": ["w"]}
    c[18] = {"up": ["w"]}
    c[19] = {"down": ["s", "q"]}
    c[21] = {"up": ["s", "q"]}
    c[22] = {"down": ["equals"]}
    c[24] = {"up": ["equals"]}
    c[25] = {"down": ["dash"]}
    c[26] = {"up": ["dash"]}
    c[27] = {"down": ["rightbracket"]}
    c[29] = {"up": ["rightbracket"], "rot": [-0.25, -0.7]}
    c[30] = {"down": ["leftbracket", "a"]}
    c[33] = {"up": ["leftbracket", "a"]}
    return c


CONTROL_STREAMS = [
    ("controls_cornell", "cornell", 96, 64, 40, 19, None, _controls_script()),
]

# models of the reference's models/ outside the setup script's menu, loaded through the script's
# own loadModel(): only their mesh payloads are kept (they pin the asset-pipeline restatement,
# python/pt_assets.py, on multi-mesh merges and mixed vertex-attribute sets)
MODEL_FIXTURES = [
    ("bookcase", "file:testBookCase.gltf:8:0"),
    ("twoparts", "file:twoParts-opaque.gltf:25:0"),
]


def run_stream(name, scene, w, h, frames, seed, model, tmp, controls=None):
    out = os.path.join(tmp, name)
    cmd = ["node", os.path.join(HERE, "make_fixtures.js"), scene, out, str(w), str(h), str(frames), str(seed)]
    if model:
        cmd.append(model)
    env = dict(os.environ)
    if controls is not None:
        env["PT_CONTROLS"] = json.dumps(controls)
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, env=env)
    with open(os.path.join(out, "frames.json")) as f:
        meta = json.load(f)
    mesh = None
    if scene in ("gltf", "hdri"):
        n = meta["triangles"]
        bvh = np.fromfile(os.path.join(out, "bvh.f32"), dtype="<f4").reshape(2 * n - 1, 8)
        tri = np.fromfile(os.path.join(out, "tri.f32"), dtype="<f4").reshape(n, 32)
        aabb_in = np.fromfile(os.path.join(out, "aabb_in.f32"), dtype="<f4").reshape(n, 9)
        mesh = (bvh, tri, aabb_in)
    return meta, mesh


def tree_depth(bvh):
    """Max root-to-leaf depth of the packed layout (left child = n+1, right = bvh[n,4])."""
    depth = 0
    stack = [(0, 1)]
    while stack:
        n, d = stack.pop()
        depth = max(depth, d)
        if bvh[n, 0] < 0:
            stack.append((n + 1, d + 1))
            stack.append((int(bvh[n, 4]), d + 1))
    return depth


def png_rgba16(path):
    """Minimal PNG decoder for the 16-bit RGBA, non-interlaced blue-noise image."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", None
    while pos < len(data):
        ln, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + ln]
        if typ == b"IHDR":
            w, h, bd, ct, _, _, il = struct.unpack(">IIBBBBB", body)
            assert (bd, ct, il) == (16, 6, 0)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + ln
    raw = zlib.decompress(idat)
    bpp, stride = 8, w * 8
    out = np.zeros((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int32)
    p = 0
    for y in range(h):
        ft = raw[p]
        line = np.frombuffer(raw[p + 1:p + 1 + stride], dtype=np.uint8).astype(np.int32)
        p += 1 + stride
        cur = np.zeros(stride, dtype=np.int32)
        for x in range(stride):
            a = cur[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if ft == 0:
                v = line[x]
            elif ft == 1:
                v = line[x] + a
            elif ft == 2:
                v = line[x] + b
            elif ft == 3:
                v = line[x] + ((a + b) >> 1)
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                v = line[x] + pr
            cur[x] = v & 255
        out[y] = cur
        prev = cur
    v16 = out.reshape(h, w, 4, 2)
    return (v16[..., 0].astype(np.uint16) << 8) | v16[..., 1]


def main():
    only = set(sys.argv[1:])
    mpath = os.path.join(GOLD, "MANIFEST.json")
    manifest = json.load(open(mpath)) if only and os.path.exists(mpath) else {}
    with tempfile.TemporaryDirectory() as tmp:
        meshes = {}
        for name, scene, w, h, frames, seed, model in STREAMS:
            if only and name not in only:
                continue
            meta, mesh = run_stream(name, scene, w, h, frames, seed, model, tmp)
            if mesh is not None:
                key = model.split()[-1].lower()
                # the HDRI scene builds its own BVH (its own model scales); share the file when equal
                shared = manifest.get("mesh_" + key, {})
                if scene == "hdri" and shared.get("sha256_bvh") != hashlib.sha256(mesh[0].tobytes()).hexdigest():
                    key = "hdri_" + key
                meta["mesh"] = "mesh_%s.npz" % key
                meshes[key] = mesh
            with open(os.path.join(GOLD, name + ".json"), "w") as f:
                json.dump(meta, f, indent=0)
            manifest[name] = {"scene": scene, "width": w, "height": h, "frames": frames, "seed": seed, "model": model}
        for name, scene, w, h, frames, seed, model, controls in CONTROL_STREAMS:
            if only and name not in only:
                continue
            meta, _ = run_stream(name, scene, w, h, frames, seed, model, tmp, controls)
            with open(os.path.join(GOLD, name + ".json"), "w") as f:
                json.dump(meta, f, indent=0)
            manifest[name] = {"scene": scene, "width": w, "height": h, "frames": frames, "seed": seed, "controls": True}
        for key, model in MODEL_FIXTURES:
            if only and "mesh_" + key not in only:
                continue
            meta, mesh = run_stream("model_" + key, "gltf", 64, 64, 1, 1, model, tmp)
            meshes[key] = mesh
        for key, (bvh, tri, aabb_in) in meshes.items():
            # aabb_in: BVH_Build_Iterative's input (js/BVH_Fast_Builder.js:320), work list = 0..N-1
            np.savez_compressed(os.path.join(GOLD, "mesh_%s.npz" % key), bvh=bvh, tri=tri, aabb_in=aabb_in)
            manifest["mesh_" + key] = {
                "triangles": int(tri.shape[0]), "nodes": int(bvh.shape[0]), "depth": tree_depth(bvh),
                "sha256_bvh": hashlib.sha256(bvh.tobytes()).hexdigest(),
                "sha256_tri": hashlib.sha256(tri.tobytes()).hexdigest(),
            }
            src = dict(MODEL_FIXTURES).get(key)
            if src:
                manifest["mesh_" + key]["model"] = src
    v16 = png_rgba16(os.path.join(REF, "textures/BlueNoise_RGBA256.png"))
    np.save(os.path.join(GOLD, "bluenoise_rgba8.npy"), (v16 >> 8).astype(np.uint8))
    manifest["bluenoise"] = {"sha256_rgba16": hashlib.sha256(v16.astype("<u2").tobytes()).hexdigest(),
                             "convention": "u8 = v16 >> 8"}
    with open(os.path.join(GOLD, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
