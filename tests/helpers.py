"""Shared loaders for the golden fixtures and oracle replays (test infrastructure)."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def stream(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def bluenoise():
    return np.load(os.path.join(GOLD, "bluenoise_rgba8.npy"))


def mesh(meta_or_key):
    key = meta_or_key if isinstance(meta_or_key, str) else meta_or_key["mesh"][len("mesh_"):-len(".npz")]
    m = np.load(os.path.join(GOLD, "mesh_%s.npz" % key))
    return {"bvh": m["bvh"], "tri": m["tri"]}


def texture_payloads(meta, m):
    """The RGBA32F arrays exactly as the setup script uploads them: the two 2048x2048 mesh textures
    (zero tail) and, for the HDRI scene, the environment (synthetic_hdr)."""
    out = {}
    for kind in ("bvh", "tri"):
        full = np.zeros(2048 * 2048 * 4, np.float32)
        flat = m[kind].reshape(-1)
        full[:flat.size] = flat
        out[kind] = full
    if meta["scene"] == "hdri":
        out["hdr"] = synthetic_hdr()
    return out


def path_call(frame):
    return next(c for c in frame if c["shader"] == "pathTracingFragmentShader")


def output_call(frame):
    return next(c for c in frame if c["shader"] == "screenOutputFragmentShader")


def oracle_scene(meta, width=None, height=None, mesh_arrays=None, maps=None):
    import ptoracle as po
    w, h = width or meta["width"], height or meta["height"]
    if meta["scene"] in ("gltf", "hdri", "skymesh"):
        m = mesh_arrays if mesh_arrays is not None else mesh(meta)
        hdr = synthetic_hdr() if meta["scene"] == "hdri" else None
        return po.Scene(meta["scene"], w, h, bluenoise(), m["bvh"], m["tri"], hdr, maps)
    return po.Scene(meta["scene"], w, h, bluenoise())


def with_resolution(uniforms, w, h):
    """The uniforms a setup script pushes after resizing to w x h (handleWindowResize +
    onApply, js/GLTF_Model_Path_Tracing.js:521-537, 815-816): uResolution and uULen = uVLen*w/h."""
    u = dict(uniforms)
    if [float(w), float(h)] != [float(v) for v in u["uResolution"][1]]:
        u["uResolution"] = ["f", [float(w), float(h)]]
        u["uULen"] = ["f", [u["uVLen"][1][0] * (w / h)]]
    return u


def oracle_replay(meta, frames=None, width=None, height=None, nthreads=0, with_output=False, mesh=None, maps=None):
    """Run the oracle over the recorded stream: returns accumulation after each frame (+ canvas)."""
    import ptoracle as po
    w, h = width or meta["width"], height or meta["height"]
    sc = oracle_scene(meta, w, h, mesh, maps)
    acc = np.zeros((h, w, 4), np.float32)
    accs, canvases, counters = [], [], []
    for f in meta["frames"][:frames]:
        u = with_resolution(path_call(f)["uniforms"], w, h)
        acc, cnt = sc.path_trace(u, acc, nthreads=nthreads)
        accs.append(acc.copy())
        counters.append(cnt)
        if with_output:
            ou = output_call(f)["uniforms"]
            exp = ou.get("uToneMappingExposure", ["f", [0.0]])[1][0]
            canvases.append(po.screen_output(acc, ou["uOneOverSampleCounter"][1][0], exp))
    return accs, canvases, counters


HDR_W, HDR_H, SUN_X, SUN_Y = 2048, 1024, 1536, 300


def synthetic_hdr():
    """The synthetic equirect environment the fixture generator hands to the HDRI setup script in
    place of its missing .hdr files (tests/golden/gen/browser_env.js syntheticHDR): (1024, 2048, 4)
    float32 in the order the script passes it to RawTexture.CreateRGBATexture (invertY = true).
    Every value is a short dyadic rational, so both generators produce the same bits."""
    i = np.arange(HDR_W * HDR_H, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x85EBCA77)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    n = (h & np.uint64(255)).astype(np.float64).reshape(HDR_H, HDR_W) / 4096.0
    y = np.arange(HDR_H, dtype=np.float64)[:, None]
    t = (HDR_H / 2 - y) / 2048.0
    sky = y < HDR_H / 2
    out = np.ones((HDR_H, HDR_W, 4), np.float64)
    out[..., 0] = np.where(sky, 0.25 + t + n, 0.125 + n)
    out[..., 1] = np.where(sky, 0.375 + t + n, 0.1875 + n)
    out[..., 2] = np.where(sky, 0.75 + 2 * t + n, 0.0625 + n)
    out[SUN_Y - 2:SUN_Y + 3, SUN_X - 2:SUN_X + 3, :3] = 512.0
    out[SUN_Y, SUN_X, :3] = 4096.0
    return out.astype(np.float32)


def rgbe_encode(img):
    """float RGB(A) (H, W, >=3) -> RGBE bytes (H, W, 4), Ward's float2rgbe: shared exponent of the
    largest channel, mantissas truncated to 8 bits."""
    rgb = np.asarray(img, np.float64)[..., :3]
    m = rgb.max(axis=-1)
    mant, e = np.frexp(m)
    ok = m >= 1e-32
    scale = np.where(ok, mant * 256.0 / np.where(ok, m, 1.0), 0.0)
    out = np.zeros(rgb.shape[:2] + (4,), np.uint8)
    out[..., :3] = np.floor(rgb * scale[..., None]).astype(np.uint8)
    out[..., 3] = np.where(ok, e + 128, 0).astype(np.uint8)
    return out


def rgbe_decode(rgbe):
    """RGBE bytes -> float32 RGBA, value = mantissa * 2^(e - 136) (Babylon HDRTools), alpha 1."""
    rgbe = np.asarray(rgbe)
    e = rgbe[..., 3].astype(np.int32)
    f = np.where(e > 0, np.ldexp(1.0, e - 136), 0.0)
    out = np.ones(rgbe.shape[:2] + (4,), np.float64)
    out[..., :3] = rgbe[..., :3] * f[..., None]
    return out.astype(np.float32)


def write_radiance_hdr(path, rgbe):
    """A Radiance .hdr file with adaptive run-length scanlines (what HDR tools write)."""
    h, w = rgbe.shape[:2]
    parts = [b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n", ("-Y %d +X %d\n" % (h, w)).encode()]
    for y in range(h):
        parts.append(bytes([2, 2, w >> 8, w & 255]))
        for c in range(4):
            ch = rgbe[y, :, c]
            x = 0
            while x < w:                       # runs of >= 3 equal bytes, else literal dumps
                run = 1
                while x + run < w and run < 127 and ch[x + run] == ch[x]:
                    run += 1
                if run >= 3:
                    parts.append(bytes([128 + run, int(ch[x])]))
                    x += run
                    continue
                start = x
                while x < w and x - start < 128:
                    if x + 2 < w and ch[x] == ch[x + 1] == ch[x + 2]:
                        break
                    x += 1
                parts.append(bytes([x - start]) + ch[start:x].tobytes())
    with open(path, "wb") as f:
        f.write(b"".join(parts))


def synthetic_dragon(nu=512, nv=512, knot=(1, 1), tube=9.0):
    """A deterministic stand-in for StanfordDragon.glb (not in the reference, SURVEY.md §8d config
    4): a bumpy (p, q) torus-knot tube (default (1, 1): a bumpy torus, BVH depth 29, no stack
    overflow; (2, 3) nests deeper than stackLevels[28]) of nu x nv x 2 triangles (524,288 at the default, the most the
    2048x2048 triangle texture holds), packed exactly as Prepare_Model_For_PathTracing packs a
    model (js/GLTF_Model_Path_Tracing.js:296-454: float64 vertex math, float32 storage, UVs -1,
    per-triangle AABBs) and built by the native builder (bit-identical to BVH_Fast_Builder.js).
    Returns {"bvh": (2N-1, 8), "tri": (N, 32), "aabb_in": (N, 9)}."""
    import babylon_pt as bp
    t = np.arange(nu) * (2 * np.pi / nu)
    v = np.arange(nv) * (2 * np.pi / nv)

    p, q = knot

    def curve(tt):
        r = 2.0 + np.cos(q * tt)
        return np.stack([r * np.cos(p * tt), r * np.sin(q * tt) * 0.6, r * np.sin(p * tt)], -1) * 9.0 + [0, -10, 0]

    c = curve(t)
    tan = curve(t + 1e-4) - curve(t - 1e-4)
    tan /= np.linalg.norm(tan, axis=1, keepdims=True)
    # rotation-minimising frame by parallel transport from an arbitrary start
    nrm = np.zeros_like(c)
    n0 = np.cross(tan[0], [0.0, 0.0, 1.0])
    nrm[0] = n0 / np.linalg.norm(n0)
    for i in range(1, nu):
        n1 = nrm[i - 1] - tan[i] * np.dot(nrm[i - 1], tan[i])
        nrm[i] = n1 / np.linalg.norm(n1)
    bin_ = np.cross(tan, nrm)
    rad = tube * (1.0 + 0.18 * np.sin(17 * t)[:, None] * np.sin(5 * v)[None, :] + 0.07 * np.sin(41 * t)[:, None])
    ring = np.cos(v)[None, :, None] * nrm[:, None, :] + np.sin(v)[None, :, None] * bin_[:, None, :]
    P = c[:, None, :] + rad[..., None] * ring                               # (nu, nv, 3) float64
    du = np.roll(P, -1, 0) - np.roll(P, 1, 0)
    dv = np.roll(P, -1, 1) - np.roll(P, 1, 1)
    N = np.cross(du, dv)
    N *= np.sign(np.sum(N * ring, -1))[..., None]                           # outward
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    i0, j0 = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    i1, j1 = (i0 + 1) % nu, (j0 + 1) % nv
    a = np.stack([i0, j0], -1).reshape(-1, 2)
    b = np.stack([i1, j0], -1).reshape(-1, 2)
    cc = np.stack([i1, j1], -1).reshape(-1, 2)
    d = np.stack([i0, j1], -1).reshape(-1, 2)
    tris = np.stack([np.stack([a, b, cc], 1), np.stack([a, cc, d], 1)], 1).reshape(-1, 3, 2)
    pos = P[tris[..., 0], tris[..., 1]]                                     # (N, 3, 3)
    nor = N[tris[..., 0], tris[..., 1]]
    # front faces outward: cross(e1, e2) along the outward normal (single-sided BVH test)
    face = np.cross(pos[:, 1] - pos[:, 0], pos[:, 2] - pos[:, 0])
    flip = np.sum(face * nor.sum(1), -1) < 0
    pos[flip] = pos[flip][:, ::-1]
    nor[flip] = nor[flip][:, ::-1]
    n = pos.shape[0]
    tri = np.zeros((n, 32), np.float32)
    tri[:, 0:9] = pos.reshape(n, 9)
    tri[:, 9:18] = nor.reshape(n, 9)
    tri[:, 18:24] = -1.0
    lo, hi = pos.min(1), pos.max(1)
    aabb_in = np.concatenate([lo, hi, (lo + hi) * 0.5], 1).astype(np.float32)
    return {"bvh": bp.bvh_build(aabb_in), "tri": tri, "aabb_in": aabb_in}


def subdivided_mesh(m, levels=2):
    """A model's triangle records split `levels` times at their edge midpoints (x4 per level: the
    StanfordBunny's 30,338 triangles -> 485,408 at 2 levels, near the 524,288 the 2048^2 triangle
    texture holds): the same surface - every new vertex lies on its triangle's plane, normals and UVs
    are the vertices' linear interpolants, windings are kept - with a scan's triangle density, so a
    BVH over real scanned geometry (depth, overlap) of the dragon's size. Float64 midpoints, float32
    storage, per-triangle AABBs, native builder (bit-identical to BVH_Fast_Builder.js); the scale-
    free scan-like counterpart of synthetic_dragon for the bench."""
    import babylon_pt as bp
    t = m["tri"].astype(np.float64)
    n = t.shape[0]
    pos, nor, uv = t[:, 0:9].reshape(n, 3, 3), t[:, 9:18].reshape(n, 3, 3), t[:, 18:24].reshape(n, 3, 2)
    for _ in range(levels):
        def mid(a, i, j):
            return (a[:, i] + a[:, j]) * 0.5
        def split(a):
            ab, bc, ca = mid(a, 0, 1), mid(a, 1, 2), mid(a, 2, 0)
            return np.stack([np.stack([a[:, 0], ab, ca], 1), np.stack([ab, a[:, 1], bc], 1),
                             np.stack([ca, bc, a[:, 2]], 1), np.stack([ab, bc, ca], 1)], 1).reshape(-1, 3, a.shape[2])
        pos, nor, uv = split(pos), split(nor), split(uv)
    n = pos.shape[0]
    tri = np.zeros((n, 32), np.float32)
    tri[:, 0:9] = pos.reshape(n, 9)
    tri[:, 9:18] = nor.reshape(n, 9)
    tri[:, 18:24] = uv.reshape(n, 6)
    p32 = tri[:, 0:9].reshape(n, 3, 3)
    lo, hi = p32.min(1), p32.max(1)
    aabb_in = np.concatenate([lo, hi, (lo + hi) * 0.5], 1).astype(np.float32)
    return {"bvh": bp.bvh_build(aabb_in), "tri": tri, "aabb_in": aabb_in}


# BASELINE configs[4]: the physical-sky page's recorded stream (sky_256) with the glTF page's model
# uniforms and samplers added, i.e. the effect the sky shader + glTF model block composite declares
# (DESIGN.md §1). Model transform: a 180-degree turn about y (exact +-1 entries), as the glTF page
# turns the dragon (js/GLTF_Model_Path_Tracing.js:905-910); material: the page's default, Metal
# (js/GLTF_Model_Path_Tracing.js:720).
SKY_MESH_MODEL_INV = [-1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, -1.0, 0.0, 0.0, 0.0, 0.0, 1.0]


def sky_mesh_stream(material=3, model_inv=None):
    meta = stream("sky_256")
    meta = dict(meta, scene="skymesh", textures={"raw2": "bvh", "raw3": "tri"}, model="StanfordDragon stand-in")
    frames = []
    for f in meta["frames"]:
        fr = []
        for c in f:
            c = dict(c, uniforms=dict(c["uniforms"]), samplers=dict(c["samplers"]))
            if c["shader"] == "pathTracingFragmentShader":
                c["uniforms"].update({
                    "uGLTF_Model_InvMatrix": ["f", list(model_inv or SKY_MESH_MODEL_INV)],
                    "uModelMaterialType": ["i", [material]],
                    "uModelUsesAlbedoTexture": ["i", [0]], "uModelUsesBumpTexture": ["i", [0]],
                    "uModelUsesMetallicTexture": ["i", [0]], "uModelUsesEmissiveTexture": ["i", [0]]})
                c["samplers"].update({"tAABBTexture": "raw2", "tTriangleTexture": "raw3"})
            fr.append(c)
        frames.append(fr)
    meta["frames"] = frames
    return meta


def po_screen_output(acc, one_over_n, exposure=1.0):
    """The oracle's screenOutput (js/PathTracingCommon.js:19-309) of an RGBA32F frame -> RGBA8."""
    import ptoracle as po
    return po.screen_output(acc, one_over_n, exposure)


# the DamagedHelmet's four PBR samplers, by the names its stream binds (js/GLTF_Model_Path_Tracing.js:
# 749-758 loads them through the glTF loader; the JPEGs stay in the reference tree)
PBR_SAMPLERS = {"albedo": "Material_MR (Base Color)", "bump": "Material_MR (Normal)",
                "metallic": "Material_MR (Metallic Roughness)", "emissive": "Material_MR (Emissive)"}


HELMET_MAP_FILES = {"albedo": "Default_albedo.jpg", "bump": "Default_normal.jpg",
                    "metallic": "Default_metalRoughness.jpg", "emissive": "Default_emissive.jpg"}


def helmet_maps():
    """The DamagedHelmet's four bound PBR maps (tests/golden/helmet_maps/, the reference's own
    models/materials/DamagedHelmet/*.jpg, bound at js/GLTF_Model_Path_Tracing.js:252-274), decoded
    as both hosts decode them (pt_assets.decode_rgba8: Pillow / libjpeg-turbo, rows top first,
    invertY false): {kind: (2048, 2048, 4) uint8}."""
    import pt_assets
    out = {}
    for kind, name in HELMET_MAP_FILES.items():
        with open(os.path.join(GOLD, "helmet_maps", name), "rb") as f:
            out[kind] = pt_assets.decode_rgba8(f.read())
    return out


# the bench workloads (bench.py --workload; tools/prof_frames.py): recorded stream, mesh arrays,
# PBR maps, default frame size
WORKLOADS = {
    "dragon": ("gltf_bunny_1080p", "dragon", None, (1920, 1080)),       # BASELINE.json metric
    "bunny": ("gltf_bunny_1080p", None, None, (1920, 1080)),           # configs[1]
    "helmet": ("hdri_helmet_320x180", None, "helmet", (1920, 1080)),   # configs[2]
    "sky_dragon": ("skymesh", "dragon", None, (3840, 2160)),           # configs[4]
    "bunny16": ("gltf_bunny_1080p", "bunny16", None, (1920, 1080)),    # scan-like dragon-sized stand-in
}


def workload(name):
    """(meta, mesh arrays, maps or None, (W, H)) of a bench workload."""
    key, mesh_kind, maps_kind, size = WORKLOADS[name]
    meta = sky_mesh_stream() if key == "skymesh" else stream(key)
    m = synthetic_dragon() if mesh_kind == "dragon" else subdivided_mesh(mesh(meta)) if mesh_kind == "bunny16" else mesh(meta)
    return meta, m, (helmet_maps() if maps_kind == "helmet" else None), size


def synthetic_pbr_maps(n=256, seed=7):
    """Seeded stand-ins for the helmet's PBR maps (RGBA8 n x n): smooth albedo, a normal map around
    +z, metallic-roughness regions below and above the shader's 0.01 thresholds (diffuse, clear
    coat, metal: .g roughness, .b metal) and a few emissive spots - every material branch of
    CalculateRadiance's PBR decode is taken."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:n, 0:n].astype(np.float64) / n
    def u8(a):
        return np.clip(np.rint(a * 255.0), 0, 255).astype(np.uint8)
    alb = np.stack([0.5 + 0.4 * np.sin(6.3 * x), 0.5 + 0.4 * np.cos(4.1 * y), 0.3 + 0.3 * x * y,
                    np.ones_like(x)], -1)
    nx, ny = 0.3 * np.sin(9.0 * x + 2.0 * y), 0.3 * np.cos(7.0 * y)
    nrm = np.stack([nx * 0.5 + 0.5, ny * 0.5 + 0.5, np.sqrt(np.clip(1.0 - nx * nx - ny * ny, 0, 1)) * 0.5 + 0.5,
                    np.ones_like(x)], -1)
    zone = (np.floor(x * 4) + np.floor(y * 4)) % 3            # 0 diffuse, 1 clear coat, 2 metal
    rough = np.where(zone >= 1, 0.2 + 0.6 * y, 0.0)
    metal = np.where(zone == 2, 0.9, 0.0)
    mr = np.stack([np.zeros_like(x), rough, metal, np.ones_like(x)], -1)
    spots = (rng.random((n, n)) < 0.01).astype(np.float64)
    emi = np.stack([spots, spots * 0.5, spots * 0.2, np.ones_like(x)], -1)
    return {"albedo": u8(alb), "bump": u8(nrm), "metallic": u8(mr), "emissive": u8(emi)}
