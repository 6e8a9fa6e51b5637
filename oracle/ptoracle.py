"""ctypes front-end of the CPU oracle (oracle/libptoracle.so) — TEST INFRASTRUCTURE.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this module.
It maps a recorded uniform stream (tests/golden/*.json, the exact effect.set* calls the reference
setup scripts make) onto the oracle's frame struct and runs the restated fragment programs.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libptoracle.so")

SCENES = {"cornell": 0, "gltf": 1, "sky": 2, "hdri": 3, "quadric": 4, "skymesh": 5}
SHAPES = ("uSphereInvMatrix", "uCylinderInvMatrix", "uConeInvMatrix", "uParaboloidInvMatrix", "uHyperboloidInvMatrix",
          "uCapsuleInvMatrix", "uFlattenedRingInvMatrix", "uBoxInvMatrix", "uPyramidFrustumInvMatrix", "uDiskInvMatrix",
          "uRectangleInvMatrix", "uTorusInvMatrix")

c_f = ctypes.c_float
c_i = ctypes.c_int32
F16 = c_f * 16


class Frame(ctypes.Structure):
    _fields_ = [
        ("scene", c_i), ("width", c_i), ("height", c_i),
        ("uResolution", c_f * 2), ("uRandomVec2", c_f * 2),
        ("uULen", c_f), ("uVLen", c_f), ("uTime", c_f),
        ("uFrameCounter", c_f), ("uSampleCounter", c_f),
        ("uEPS_intersect", c_f), ("uApertureSize", c_f), ("uFocusDistance", c_f),
        ("uCameraIsMoving", c_i),
        ("uCameraMatrix", F16), ("uLeftSphereInvMatrix", F16), ("uRightSphereInvMatrix", F16),
        ("uGLTF_Model_InvMatrix", F16),
        ("uQuadLightPlaneSelectionNumber", c_f), ("uQuadLightRadius", c_f),
        ("uRightSphereMatType", c_i), ("uModelMaterialType", c_i),
        ("uModelUsesAlbedoTexture", c_i), ("uModelUsesBumpTexture", c_i),
        ("uModelUsesMetallicTexture", c_i), ("uModelUsesEmissiveTexture", c_i),
        ("blueNoise", ctypes.c_void_p),
        ("aabb", ctypes.c_void_p), ("aabbTexels", ctypes.c_int64),
        ("tri", ctypes.c_void_p), ("triTexels", ctypes.c_int64),
        ("albedo", ctypes.c_void_p), ("albedoW", c_i), ("albedoH", c_i),
        ("bump", ctypes.c_void_p), ("bumpW", c_i), ("bumpH", c_i),
        ("metallic", ctypes.c_void_p), ("metallicW", c_i), ("metallicH", c_i),
        ("emissive", ctypes.c_void_p), ("emissiveW", c_i), ("emissiveH", c_i),
        ("uSunDirection", c_f * 3),
        ("uHDRExposure", c_f), ("uSunPower", c_f),
        ("hdr", ctypes.c_void_p), ("hdrW", c_i), ("hdrH", c_i),
        ("uShapeInvMatrix", (c_f * 16) * 12), ("uShapeK", c_f), ("uAllShapesMatType", c_i),
    ]


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("paths", "segments", "node_fetches", "leaf_tests", "hit_lookups", "rgba8_taps", "stack_overflow",
                 "hdr_taps")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_libs = {}
# the tolerance study's other built-in sets (oracle/Makefile; tools/tolerance.py): "" = the pinned build
VARIANTS = ("", "fma", "libm", "gpu")


def lib(variant=""):
    if variant not in _libs:
        path = LIB_PATH if not variant else os.path.join(HERE, "libptoracle_%s.so" % variant)
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.pto_path_trace.argtypes = [P(Frame), ctypes.c_void_p, ctypes.c_void_p, c_i, c_i, c_i, P(Counters)]
        L.pto_gbuffer.argtypes = [P(Frame), ctypes.c_void_p, c_i, c_i, c_i]
        L.pto_screen_output.argtypes = [c_i, c_i, ctypes.c_void_p, c_f, c_f, ctypes.c_void_p, c_i]
        L.pto_screen_output_f32.argtypes = [c_i, c_i, ctypes.c_void_p, c_f, c_f, ctypes.c_void_p]
        L.pto_math_probe.argtypes = [c_i, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_i]
        L.pto_sky_color.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_i]
        L.pto_quadric_probe.argtypes = [c_i, c_f, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_i]
        _libs[variant] = L
    return _libs[variant]


class Scene:
    """Keeps the sampler arrays alive and builds Frame structs from recorded uniforms."""

    def __init__(self, scene, width, height, bluenoise, bvh=None, tri=None, hdr=None, maps=None, variant=""):
        """hdr: the tHDRTexture payload as the setup script uploads it (rows top-first, invertY).
        maps: {"albedo"|"bump"|"metallic"|"emissive": RGBA8 (h, w, 4)} in upload row order.
        variant: the built-in set (VARIANTS; "" = pinned, the only one the parity tests use)."""
        self.variant = variant
        self.maps = {k: np.ascontiguousarray(v, dtype=np.uint8) for k, v in (maps or {}).items()}
        self.scene = scene
        self.hdr = None if hdr is None else np.ascontiguousarray(np.asarray(hdr, dtype=np.float32)[::-1])
        self.width, self.height = width, height
        self.bluenoise = np.ascontiguousarray(bluenoise, dtype=np.uint8)
        self.bvh = None if bvh is None else np.ascontiguousarray(bvh, dtype=np.float32)
        self.tri = None if tri is None else np.ascontiguousarray(tri, dtype=np.float32)

    def frame(self, uniforms):
        f = Frame()
        f.scene = SCENES[self.scene]
        f.width, f.height = self.width, self.height
        for name, (kind, vals) in uniforms.items():
            if name in SHAPES:
                for i, v in enumerate(vals):
                    f.uShapeInvMatrix[SHAPES.index(name)][i] = v
                continue
            if not hasattr(f, name):
                continue
            cur = getattr(f, name)
            if isinstance(cur, ctypes.Array):
                for i, v in enumerate(vals):
                    cur[i] = v
            else:
                setattr(f, name, int(vals[0]) if kind == "i" else float(vals[0]))
        f.blueNoise = self.bluenoise.ctypes.data
        if self.hdr is not None:
            f.hdr = self.hdr.ctypes.data
            f.hdrH, f.hdrW = self.hdr.shape[:2]
        for k, m in self.maps.items():
            setattr(f, k, m.ctypes.data)
            setattr(f, k + "H", m.shape[0])
            setattr(f, k + "W", m.shape[1])
        if self.bvh is not None:
            f.aabb = self.bvh.ctypes.data
            f.aabbTexels = self.bvh.size // 4
            f.tri = self.tri.ctypes.data
            f.triTexels = self.tri.size // 4
        return f

    def path_trace(self, uniforms, prev, row0=0, row1=None, nthreads=0):
        row1 = self.height if row1 is None else row1
        f = self.frame(uniforms)
        prev = np.ascontiguousarray(prev, dtype=np.float32)
        out = prev.copy()
        cnt = Counters()
        rc = lib(self.variant).pto_path_trace(ctypes.byref(f), prev.ctypes.data, out.ctypes.data, row0, row1, nthreads, ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError("pto_path_trace failed: %d" % rc)
        return out, cnt.as_dict()

    def gbuffer(self, uniforms, row0=0, row1=None, nthreads=0):
        row1 = self.height if row1 is None else row1
        f = self.frame(uniforms)
        g = np.zeros((row1 - row0, self.width, 11), dtype=np.float32)
        rc = lib(self.variant).pto_gbuffer(ctypes.byref(f), g.ctypes.data, row0, row1, nthreads)
        if rc != 0:
            raise RuntimeError("pto_gbuffer failed: %d" % rc)
        return g


def screen_output(acc, one_over_n, exposure=1.0):
    acc = np.ascontiguousarray(acc, dtype=np.float32)
    h, w = acc.shape[:2]
    out = np.zeros((h, w, 4), dtype=np.uint8)
    rc = lib().pto_screen_output(w, h, acc.ctypes.data, one_over_n, exposure, out.ctypes.data, 0)
    if rc != 0:
        raise RuntimeError("pto_screen_output failed")
    return out


def screen_output_f32(acc, one_over_n, exposure=1.0):
    """screenOutput into an RGBA32F target: the tone-mapped floats before the canvas's unorm8."""
    acc = np.ascontiguousarray(acc, dtype=np.float32)
    h, w = acc.shape[:2]
    out = np.zeros((h, w, 4), dtype=np.float32)
    rc = lib().pto_screen_output_f32(w, h, acc.ctypes.data, one_over_n, exposure, out.ctypes.data)
    if rc != 0:
        raise RuntimeError("pto_screen_output_f32 failed")
    return out


def math_probe(op, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = None if y is None else np.ascontiguousarray(y, dtype=np.float32)
    out = np.zeros_like(x)
    rc = lib().pto_math_probe(op, x.ctypes.data, None if y is None else y.ctypes.data, out.ctypes.data, x.size)
    if rc != 0:
        raise RuntimeError("bad op")
    return out


def sky_color(sun, dirs):
    """Get_Sky_Color of the oracle for an (n, 3) array of ray directions."""
    sun = np.ascontiguousarray(sun, dtype=np.float32)
    dirs = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    out = np.zeros_like(dirs)
    lib().pto_sky_color(sun.ctypes.data, dirs.ctypes.data, out.ctypes.data, dirs.shape[0])
    return out


def quadric_probe(shape, k, ro, rd):
    """The oracle's unit-shape intersector `shape` (0..11, SceneIntersect order) on object-space rays."""
    ro = np.ascontiguousarray(ro, dtype=np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(rd, dtype=np.float32).reshape(-1, 3)
    t = np.zeros(ro.shape[0], np.float32)
    n = np.zeros_like(ro)
    if lib().pto_quadric_probe(shape, k, ro.ctypes.data, rd.ctypes.data, t.ctypes.data, n.ctypes.data, ro.shape[0]) != 0:
        raise ValueError("bad shape")
    return t, n
