"""Python binding of libpt.so (include/pt.h), shaped like the Babylon effect API the reference's
setup scripts use, plus a replayer for recorded per-frame render-call streams.

The reference host is JavaScript; its drop-in binding is the Node N-API addon + JS shim in
../napi and ../js. This module is the same boundary seen from Python, for the parity tests and
bench.py: the classes mirror

  new BABYLON.Engine(canvas)                       -> Engine(device)
  BABYLON.RawTexture.CreateRGBATexture(...)        -> RawTexture.CreateRGBATexture(...)
  new BABYLON.Texture(url, ...) (decoded RGBA8)    -> Texture(engine, rgba8, ...)
  new BABYLON.RenderTargetTexture(name, {w,h}, ..) -> RenderTargetTexture(name, (w, h), engine)
  new BABYLON.EffectWrapper({...})                 -> EffectWrapper(engine, program, uniformNames, samplerNames)
  wrapper.effect.setFloat/setFloat2/.../setTexture -> the same method names
  new BABYLON.EffectRenderer(engine).render(w, t)  -> EffectRenderer(engine).render(w, t)

(js/GLTF_Model_Path_Tracing.js:189, 466-487, 749-768, 770-848, 1230-1235). There is no CPU
fallback: if libpt.so or a gfx950 device is missing, construction raises.
"""
import ctypes
import struct
import json
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("PT_LIBPT") or os.path.join(PKG, "libpt.so")

PROG = {"screenCopy": 1, "screenOutput": 2, "cornell": 3, "gltf": 4, "hdri": 5, "sky": 6, "quadric": 7, "skymesh": 8}
ERRORS = {0: "PT_OK", -1: "PT_ERR_ARG", -2: "PT_ERR_HIP", -3: "PT_ERR_SHADER", -4: "PT_ERR_STATE",
          -5: "PT_ERR_OOM", -6: "PT_ERR_DEVICE", -7: "PT_ERR_UNSUPPORTED", -8: "PT_ERR_DATA"}
NEAREST, BILINEAR, TRILINEAR = 1, 2, 3

# every symbol include/pt.h declares (checked by tests/test_capi_symbols.py)
SYMBOLS = [
    "pt_ctx_create", "pt_ctx_create_mask", "pt_ctx_create_devices", "pt_ctx_parts", "pt_ctx_peer_copies", "pt_ctx_destroy", "pt_last_error", "pt_sync", "pt_canvas_resize",
    "pt_effect_create", "pt_effect_create_program", "pt_effect_destroy", "pt_effect_program",
    "pt_set_float", "pt_set_int", "pt_set_texture",
    "pt_texture_create_rgba32f", "pt_texture_create_rgba8", "pt_render_target_create", "pt_render_target_wrap",
    "pt_render_target_resize", "pt_texture_size", "pt_texture_destroy",
    "pt_render", "pt_read_pixels", "pt_write_pixels",
    "pt_set_row_partition", "pt_set_output_partition", "pt_canvas_wrap", "pt_set_backend", "pt_set_bvh_layout", "pt_bvh_layout_used", "pt_set_stream", "pt_texture_device_ptr", "pt_last_render_ms", "pt_timing_begin", "pt_timing_end", "pt_timing_latency",
    "pt_set_counting", "pt_read_counters", "pt_reset_counters", "pt_queue_stats", "pt_math_probe", "pt_math_exhaustive", "pt_bvh_build", "pt_bvh_build_gpu", "pt_jpeg_size", "pt_jpeg_decode_rgba8", "pt_version",
]

_lib = None


def lib():
    """Load libpt.so and declare the C signatures (no device call happens here)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libpt.so not built: run __graft_entry__.build() (%s)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, i32, f32p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_float)
    cpp = ctypes.POINTER(ctypes.c_char_p)
    sig = {
        "pt_ctx_create": ([i32, ip], vp), "pt_ctx_create_mask": ([ctypes.c_uint32, ip], vp),
        "pt_ctx_create_devices": ([ctypes.POINTER(ctypes.c_int), i32, ip], vp), "pt_ctx_parts": ([vp], i32), "pt_ctx_peer_copies": ([vp], i32),
        "pt_ctx_destroy": ([vp], None), "pt_last_error": ([vp], ctypes.c_char_p),
        "pt_sync": ([vp], i32), "pt_canvas_resize": ([vp, i32, i32], i32),
        "pt_effect_create": ([vp, ctypes.c_char_p, cpp, i32, cpp, i32, ip], vp),
        "pt_effect_create_program": ([vp, i32, cpp, i32, cpp, i32, ip], vp),
        "pt_effect_destroy": ([vp], None), "pt_effect_program": ([vp], i32),
        "pt_set_float": ([vp, ctypes.c_char_p, f32p, i32], i32), "pt_set_int": ([vp, ctypes.c_char_p, i32], i32),
        "pt_set_texture": ([vp, ctypes.c_char_p, vp], i32),
        "pt_texture_create_rgba32f": ([vp, i32, i32, vp, i32, i32, ip], vp),
        "pt_texture_create_rgba8": ([vp, i32, i32, vp, i32, i32, ip], vp),
        "pt_render_target_create": ([vp, i32, i32, ip], vp),
        "pt_render_target_wrap": ([vp, i32, i32, vp, ip], vp),
        "pt_render_target_resize": ([vp, i32, i32], i32),
        "pt_texture_size": ([vp, ip, ip], i32), "pt_texture_destroy": ([vp], None),
        "pt_render": ([vp, vp], i32), "pt_read_pixels": ([vp, vp, vp, ctypes.c_size_t], i32),
        "pt_write_pixels": ([vp, vp, vp, ctypes.c_size_t], i32),
        "pt_set_row_partition": ([vp, i32, i32], i32), "pt_texture_device_ptr": ([vp], vp),
        "pt_set_backend": ([vp, i32], i32), "pt_set_output_partition": ([vp, i32], i32),
        "pt_canvas_wrap": ([vp, i32, i32, vp], i32), "pt_set_stream": ([vp, vp], i32),
        "pt_set_bvh_layout": ([vp, i32], i32), "pt_bvh_layout_used": ([vp], i32),
        "pt_bvh_build": ([vp, vp, i32, vp, i32], i32),
        "pt_bvh_build_gpu": ([i32, vp, vp, i32, vp, i32, f32p], i32),
        "pt_jpeg_size": ([ctypes.c_char_p, ctypes.c_size_t, ip, ip], i32),
        "pt_jpeg_decode_rgba8": ([ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.c_size_t], i32),
        "pt_last_render_ms": ([vp, i32, f32p], i32), "pt_set_counting": ([vp, i32], i32),
        "pt_timing_begin": ([vp], i32),
        "pt_timing_end": ([vp, i32, ctypes.POINTER(ctypes.c_double), ip], i32),
        "pt_timing_latency": ([vp, i32, ctypes.POINTER(ctypes.c_float), i32, ip], i32),
        "pt_read_counters": ([vp, ctypes.POINTER(ctypes.c_uint64)], i32), "pt_reset_counters": ([vp], i32),
        "pt_math_probe": ([vp, i32, vp, vp, vp, i32], i32),
        "pt_math_exhaustive": ([vp, i32, vp], i32),
        "pt_queue_stats": ([vp, ctypes.POINTER(ctypes.c_uint32)], i32), "pt_version": ([], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


class PtError(RuntimeError):
    pass


def _names(seq):
    arr = (ctypes.c_char_p * max(1, len(seq)))()
    for i, s in enumerate(seq):
        arr[i] = s.encode()
    return arr


class Engine:
    """`new BABYLON.Engine(canvas)` -> a pt context: one part (one HIP stream) on `device`, or one
    part per entry of `devices` (a device may repeat); with several parts libpt splits every frame
    over them into 16-row bands and gathers the canvas (include/pt.h)."""

    def __init__(self, device=0, devices=None):
        err = ctypes.c_int(0)
        if devices is None:
            self.ctx = lib().pt_ctx_create(device, ctypes.byref(err))
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            self.ctx = lib().pt_ctx_create_devices(arr, len(devices), ctypes.byref(err))
        if not self.ctx:
            raise PtError("pt_ctx_create(%s) failed: %s" % (devices if devices is not None else device,
                                                             ERRORS.get(err.value, err.value)))
        self.device = device if devices is None else devices[0]
        self.parts = lib().pt_ctx_parts(self.ctx)
        self.peer_copies = lib().pt_ctx_peer_copies(self.ctx) == 1
        self._objs = []

    def check(self, rc, what=""):
        if rc != 0:
            raise PtError("%s: %s (%s)" % (what, ERRORS.get(rc, rc), lib().pt_last_error(self.ctx).decode()))
        return rc

    def sync(self):
        self.check(lib().pt_sync(self.ctx), "pt_sync")

    def resize_canvas(self, w, h):
        self.check(lib().pt_canvas_resize(self.ctx, w, h), "pt_canvas_resize")

    def read_canvas(self, w, h):
        out = np.zeros((h, w, 4), dtype=np.uint8)
        self.check(lib().pt_read_pixels(self.ctx, None, out.ctypes.data, out.nbytes), "pt_read_pixels")
        return out

    def set_row_partition(self, parts, part):
        self.check(lib().pt_set_row_partition(self.ctx, parts, part), "pt_set_row_partition")

    def set_output_partition(self, on):
        """screenOutput shades only this context's row bands (halo rows must be exchanged first)."""
        self.check(lib().pt_set_output_partition(self.ctx, 1 if on else 0), "pt_set_output_partition")

    def canvas_wrap(self, w, h, device_ptr):
        """The RGBA8 canvas over caller-owned device memory (e.g. a torch uint8 tensor)."""
        self.check(lib().pt_canvas_wrap(self.ctx, w, h, ctypes.c_void_p(device_ptr)), "pt_canvas_wrap")

    def set_stream(self, hip_stream):
        """Enqueue on a caller-owned stream (an int handle, e.g. a dedicated torch.cuda.Stream's
        .cuda_stream); None restores the context's own stream. A 0 handle is refused: it is HIP's
        legacy default stream (what torch.cuda.current_stream() is unless a stream was made
        current), which the context's non-blocking stream would not be ordered with."""
        if hip_stream is not None and not hip_stream:
            raise PtError("set_stream(0): pass a dedicated stream's handle (or None for the context's own stream)")
        self.check(lib().pt_set_stream(self.ctx, ctypes.c_void_p(hip_stream) if hip_stream else None), "pt_set_stream")

    def set_backend(self, backend):
        """'megakernel' (default), 'wavefront' or 'persistent': same bits, different schedule."""
        self.check(lib().pt_set_backend(self.ctx, {"megakernel": 0, "wavefront": 1, "persistent": 2}[backend]),
                   "pt_set_backend")

    BVH_LAYOUTS = {"reference": 0, "pairs": 1, "trail": 2}

    def set_bvh_layout(self, layout):
        """'pairs' (default: child-pair records with the short stack, falls back to the reference
        walk for malformed trees), 'trail' (the same records walked stacklessly with the restart
        trail; trees it cannot walk keep 'pairs') or 'reference' (walk the reference texel pairs):
        same bits, different memory path."""
        self.check(lib().pt_set_bvh_layout(self.ctx, self.BVH_LAYOUTS[layout]), "pt_set_bvh_layout")

    def bvh_layout_used(self):
        """Layout walked by the last glTF draw: 'trail', 'pairs', 'reference' or None."""
        v = lib().pt_bvh_layout_used(self.ctx)
        return {0: "reference", 1: "pairs", 2: "trail"}.get(v)

    def last_render_ms(self, program):
        ms = ctypes.c_float(0)
        self.check(lib().pt_last_render_ms(self.ctx, PROG.get(program, program), ctypes.byref(ms)), "pt_last_render_ms")
        return ms.value

    def timing_begin(self):
        self.check(lib().pt_timing_begin(self.ctx), "pt_timing_begin")

    def timing_end(self, program):
        """(total device ms, launches) of `program` draws since timing_begin (synchronises)."""
        t, n = ctypes.c_double(0), ctypes.c_int(0)
        self.check(lib().pt_timing_end(self.ctx, PROG.get(program, program), ctypes.byref(t), ctypes.byref(n)), "pt_timing_end")
        return t.value, n.value

    def timing_latency(self, program, cap=4096):
        """Per-frame ms from each bracketed `program` draw's begin (its path tracing may start) to the
        next bracketed screenOutput's end (its canvas complete), since timing_begin (synchronises)."""
        buf = (ctypes.c_float * cap)()
        n = ctypes.c_int(0)
        self.check(lib().pt_timing_latency(self.ctx, PROG.get(program, program), buf, cap, ctypes.byref(n)),
                   "pt_timing_latency")
        return list(buf[:n.value])

    def set_counting(self, on):
        self.check(lib().pt_set_counting(self.ctx, 1 if on else 0))

    def reset_counters(self):
        self.check(lib().pt_reset_counters(self.ctx))

    def counters(self):
        keys = ("paths", "segments", "node_fetches", "leaf_tests", "hit_lookups", "rgba8_taps", "stack_overflow",
                "hdr_taps")
        buf = (ctypes.c_uint64 * len(keys))()
        self.check(lib().pt_read_counters(self.ctx, buf), "pt_read_counters")
        return {k: int(v) for k, v in zip(keys, buf)}

    def queue_stats(self):
        """Wavefront queue sizes of the last draw (paths per bounce, BVH rays per bounce) and the
        tiles the next megakernel draw of the same grid splits into 16-lane waves."""
        buf = (ctypes.c_uint32 * 16)()
        self.check(lib().pt_queue_stats(self.ctx, buf), "pt_queue_stats")
        return {"paths": list(buf[0:7]), "bvh": list(buf[8:14]), "split_tiles": int(buf[7]),
                "late_bounce_compaction": {0: "off", 1: "auto: off", 2: "auto: on", 3: "on", 4: "auto: trial",
                                           5: "auto: default on", 6: "auto: default off"}[int(buf[14]) & 0xFF],
                "frames_in_flight": (int(buf[14]) >> 8) & 0xFF,
                "compacting_draws": int(buf[14]) >> 16,
                "compaction_trial_ratio": buf[15] / 1000.0 if buf[15] else None}

    def math_probe(self, op, x, y=None):
        x = np.ascontiguousarray(x, dtype=np.float32)
        y = None if y is None else np.ascontiguousarray(y, dtype=np.float32)
        out = np.zeros_like(x)
        self.check(lib().pt_math_probe(self.ctx, op, x.ctypes.data, None if y is None else y.ctypes.data,
                                       out.ctypes.data, x.size), "pt_math_probe")
        return out

    def math_exhaustive(self, op):
        """Mismatches of device fast sequence `op` vs its IEEE operation over all 2^32 inputs."""
        n = ctypes.c_uint64(0)
        self.check(lib().pt_math_exhaustive(self.ctx, op, ctypes.byref(n)), "pt_math_exhaustive")
        return n.value

    def dispose(self):
        if self.ctx:
            lib().pt_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.dispose()
        except Exception:
            pass


class _Tex:
    def __init__(self, engine, handle, name):
        self.engine, self.handle, self.name = engine, handle, name

    def getSize(self):
        w, h = ctypes.c_int(0), ctypes.c_int(0)
        lib().pt_texture_size(self.handle, ctypes.byref(w), ctypes.byref(h))
        return {"width": w.value, "height": h.value}

    def dispose(self):
        if self.handle and self.engine.ctx:
            lib().pt_texture_destroy(self.handle)
        self.handle = None


class RenderTargetTexture(_Tex):
    """RGBA32F render target, zero-filled (js/GLTF_Model_Path_Tracing.js:762-768)."""

    def __init__(self, name, size, engine, device_ptr=None):
        w, h = (size["width"], size["height"]) if isinstance(size, dict) else size
        err = ctypes.c_int(0)
        if device_ptr is None:
            hnd = lib().pt_render_target_create(engine.ctx, w, h, ctypes.byref(err))
        else:   # caller-owned device memory (e.g. a torch tensor shared with RCCL)
            hnd = lib().pt_render_target_wrap(engine.ctx, w, h, ctypes.c_void_p(device_ptr), ctypes.byref(err))
        if not hnd:
            raise PtError("pt_render_target_create: %s" % ERRORS.get(err.value, err.value))
        super().__init__(engine, hnd, name)

    def resize(self, size):
        w, h = (size["width"], size["height"]) if isinstance(size, dict) else size
        self.engine.check(lib().pt_render_target_resize(self.handle, w, h), "resize")

    def read(self):
        s = self.getSize()
        out = np.zeros((s["height"], s["width"], 4), dtype=np.float32)
        self.engine.check(lib().pt_read_pixels(self.engine.ctx, self.handle, out.ctypes.data, out.nbytes), "read")
        return out

    def write(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float32)
        self.engine.check(lib().pt_write_pixels(self.engine.ctx, self.handle, arr.ctypes.data, arr.nbytes), "write")

    def device_ptr(self):
        return lib().pt_texture_device_ptr(self.handle)


class RawTexture(_Tex):
    @staticmethod
    def CreateRGBATexture(data, w, h, engine, generateMipMaps=False, invertY=False, samplingMode=NEAREST, name=None):
        """RGBA32F data texture (js/GLTF_Model_Path_Tracing.js:466-487); data is copied."""
        arr = np.ascontiguousarray(np.asarray(data, dtype=np.float32).reshape(-1))
        if arr.size < 4 * w * h:
            arr = np.concatenate([arr, np.zeros(4 * w * h - arr.size, np.float32)])
        err = ctypes.c_int(0)
        hnd = lib().pt_texture_create_rgba32f(engine.ctx, w, h, arr.ctypes.data, samplingMode, 1 if invertY else 0, ctypes.byref(err))
        if not hnd:
            raise PtError("pt_texture_create_rgba32f: %s" % ERRORS.get(err.value, err.value))
        return RawTexture(engine, hnd, name or "raw")


class Texture(_Tex):
    """An 8-bit image texture (the blue-noise PNG, PBR maps), decoded by the host to RGBA8."""

    def __init__(self, engine, rgba8, invertY=False, samplingMode=NEAREST, name="texture"):
        arr = np.ascontiguousarray(rgba8, dtype=np.uint8)
        h, w = arr.shape[:2]
        err = ctypes.c_int(0)
        hnd = lib().pt_texture_create_rgba8(engine.ctx, w, h, arr.ctypes.data, samplingMode, 1 if invertY else 0, ctypes.byref(err))
        if not hnd:
            raise PtError("pt_texture_create_rgba8: %s" % ERRORS.get(err.value, err.value))
        super().__init__(engine, hnd, name)


class Effect:
    """wrapper.effect: the uniform/sampler setters of js/GLTF_Model_Path_Tracing.js:818-847."""

    def __init__(self, engine, handle):
        self.engine, self.handle = engine, handle
        # the last value each uniform was given, as its float32 / int bits: a set that repeats it is
        # skipped (Babylon's Effect keeps the same value cache for setFloat*/setInt/setMatrix, and
        # skips rebinding the texture a sampler already has), so a still camera's frame crosses the C
        # ABI only for the counters and the random vector
        self._cache = {}
        self._entry = {}   # the recorded-stream entry (StreamPlayer) each uniform was last set from
        self._tex = {}

    def _set_entry(self, name, ent):
        """A recorded uniform entry [kind, values]: nothing to do when this very entry object was
        the last one set (recorded entries are never mutated)."""
        if self._entry.get(name) is ent:
            return
        kind, vals = ent
        if kind == "i":
            self.setInt(name, vals[0])
        else:
            self._f(name, vals)
        self._entry[name] = ent

    def _f(self, name, vals):
        self._entry.pop(name, None)
        try:   # (the C cast ctypes makes; a finite double beyond float range packs as ctypes's inf)
            bits = struct.pack("%df" % len(vals), *vals)
        except (OverflowError, struct.error):
            bits = bytes((ctypes.c_float * len(vals))(*vals))
        if self._cache.get(name) == bits:
            return
        arr = (ctypes.c_float * len(vals)).from_buffer_copy(bits)
        self.engine.check(lib().pt_set_float(self.handle, name.encode(), arr, len(vals)), "setFloat " + name)
        self._cache[name] = bits

    def setFloat(self, name, v):
        self._f(name, [v])

    def setFloat2(self, name, a, b):
        self._f(name, [a, b])

    def setFloat3(self, name, a, b, c):
        self._f(name, [a, b, c])

    def setMatrix(self, name, m):
        self._f(name, list(m))

    def setInt(self, name, v):
        self._entry.pop(name, None)
        v = int(v)
        if self._cache.get(name) == v:
            return
        self.engine.check(lib().pt_set_int(self.handle, name.encode(), v), "setInt " + name)
        self._cache[name] = v

    def setBool(self, name, v):
        self.setInt(name, 1 if v else 0)

    def setTexture(self, name, tex):
        h = tex.handle if tex is not None else None
        last = self._tex.get(name)
        if last is not None and last[0] is tex and last[1] == h:
            return
        self.engine.check(lib().pt_set_texture(self.handle, name.encode(), h), "setTexture")
        self._tex[name] = (tex, h)


class EffectWrapper:
    """EffectWrapper({engine, fragmentShader, uniformNames, samplerNames, name}).

    `program` is either the GLSL text registered in Effect.ShadersStore (as the JS shim passes it)
    or a program key from PROG (hosts that do not carry the reference's shader text)."""

    def __init__(self, engine, program, uniformNames=(), samplerNames=(), name="effect"):
        err = ctypes.c_int(0)
        un, sn = _names(list(uniformNames)), _names(list(samplerNames))
        if isinstance(program, str) and program in PROG:
            hnd = lib().pt_effect_create_program(engine.ctx, PROG[program], un, len(uniformNames), sn, len(samplerNames), ctypes.byref(err))
        else:
            src = program.encode() if isinstance(program, str) else program
            hnd = lib().pt_effect_create(engine.ctx, src, un, len(uniformNames), sn, len(samplerNames), ctypes.byref(err))
        if not hnd:
            raise PtError("EffectWrapper(%s): %s (%s)" % (name, ERRORS.get(err.value, err.value), lib().pt_last_error(engine.ctx).decode()))
        self.engine, self.name = engine, name
        self.effect = Effect(engine, hnd)
        self._observers = []
        self.onApplyObservable = self

    def add(self, fn):                      # onApplyObservable.add(cb)
        self._observers.append(fn)

    def program(self):
        return lib().pt_effect_program(self.effect.handle)


class EffectRenderer:
    """eRenderer.render(wrapper, target): fire onApply observers, then draw (target None = canvas)."""

    def __init__(self, engine):
        self.engine = engine

    def render(self, wrapper, target=None):
        for fn in wrapper._observers:
            fn()
        rc = lib().pt_render(wrapper.effect.handle, target.handle if target is not None else None)
        self.engine.check(rc, "render(%s)" % wrapper.name)


# ------------------------------------------------------------------------------------------------
# Replaying recorded render-call streams (tests/golden/*.json): the same effect.set* calls, sampler
# bindings and draw order the reference's setup scripts issued, through this boundary.

SHADER_PROG = {"pathTracingFragmentShader": None, "screenCopyFragmentShader": "screenCopy",
               "screenOutputFragmentShader": "screenOutput"}


def bvh_build(aabb_in, work=None):
    """BVH_Build_Iterative (js/BVH_Fast_Builder.js) in libpt: (n, 9) per-triangle AABBs ->
    (2n-1, 8) float32 nodes in the tAABBTexture layout."""
    aabb_in = np.ascontiguousarray(aabb_in, dtype=np.float32).reshape(-1, 9)
    n = aabb_in.shape[0]
    work = np.arange(n, dtype=np.uint32) if work is None else np.ascontiguousarray(work, dtype=np.uint32)
    out = np.zeros((2 * len(work), 8), np.float32)
    rc = lib().pt_bvh_build(aabb_in.ctypes.data, work.ctypes.data, len(work), out.ctypes.data, out.shape[0])
    if rc < 0:
        raise PtError("pt_bvh_build: %s" % ERRORS.get(rc, rc))
    return out[:rc]


def bvh_build_gpu(aabb_in, work=None, device=0):
    """The same build on the device (pt_bvh_build_gpu, csrc/pt_bvh_gpu.hip): returns (nodes, ms of
    device time)."""
    aabb_in = np.ascontiguousarray(aabb_in, dtype=np.float32).reshape(-1, 9)
    n = aabb_in.shape[0]
    work = np.arange(n, dtype=np.uint32) if work is None else np.ascontiguousarray(work, dtype=np.uint32)
    if len(work) and int(work.max()) >= n:
        raise PtError("pt_bvh_build_gpu: work names a triangle beyond aabb_in")
    out = np.zeros((max(1, 2 * len(work) - 1), 8), np.float32)
    ms = ctypes.c_float(0.0)
    rc = lib().pt_bvh_build_gpu(device, aabb_in.ctypes.data, work.ctypes.data, len(work), out.ctypes.data,
                                out.shape[0], ctypes.byref(ms))
    if rc < 0:
        raise PtError("pt_bvh_build_gpu: %s" % ERRORS.get(rc, rc))
    return out[:rc], ms.value


def decode_jpeg(data):
    """JPEG bytes -> (h, w, 4) uint8 RGBA rows top first (pt_jpeg_decode_rgba8: libjpeg-turbo's
    default decompression, bit for bit)."""
    data = bytes(data)
    w, h = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().pt_jpeg_size(data, len(data), ctypes.byref(w), ctypes.byref(h))
    if rc < 0:
        raise PtError("pt_jpeg_size: %s" % ERRORS.get(rc, rc))
    out = np.zeros((h.value, w.value, 4), np.uint8)
    rc = lib().pt_jpeg_decode_rgba8(data, len(data), out.ctypes.data, out.size)
    if rc < 0:
        raise PtError("pt_jpeg_decode_rgba8: %s" % ERRORS.get(rc, rc))
    return out


def splitmix64_uniforms(seed, n):
    """n floats in [0,1) with 24-bit resolution (exact in fp32): the Math.random stand-in the
    fixture generator installs (tests/golden/gen/make_fixtures.js)."""
    M = (1 << 64) - 1
    st, out = seed & M, []
    for _ in range(n):
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out.append((z >> 40) / 16777216.0)
    return out


class StreamPlayer:
    """Drives the boundary with a recorded per-frame call stream, the way the setup script's
    render loop does (js/GLTF_Model_Path_Tracing.js:1087-1235): per frame set uniforms + samplers
    on each wrapper and render pathTracing -> screenCopy -> screenOutput."""

    def __init__(self, engine, meta, bluenoise, mesh=None, width=None, height=None, rt_ptrs=None):
        self.engine = engine
        self.meta = meta
        w = width or meta["width"]
        h = height or meta["height"]
        self.width, self.height = w, h
        scene = meta["scene"]
        rt_ptrs = rt_ptrs or {}
        self.textures = {
            n: RenderTargetTexture(n, (w, h), engine, rt_ptrs.get(n))
            for n in ("pathTracingRenderTarget", "screenCopyRenderTarget")
        }
        self.textures["file:BlueNoise_RGBA256.png"] = Texture(engine, bluenoise, name="blueNoise")
        if mesh is not None:
            for raw, kind in meta["textures"].items():
                if kind == "hdr":   # the environment: its own size, uploaded with invertY as the script does
                    hd = meta["hdr"]
                    self.textures[raw] = RawTexture.CreateRGBATexture(mesh[kind], hd["width"], hd["height"], engine,
                                                                      invertY=hd["invertY"], samplingMode=TRILINEAR,
                                                                      name=kind)
                else:
                    self.textures[raw] = RawTexture.CreateRGBATexture(mesh[kind], 2048, 2048, engine, name=kind)
        self.renderer = EffectRenderer(engine)
        self.wrappers = {}
        for call in meta["frames"][0]:
            key = SHADER_PROG[call["shader"]] or scene
            self.wrappers[call["effect"]] = EffectWrapper(engine, key, list(call["uniforms"].keys()),
                                                          list(call["samplers"].keys()), call["effect"])
        self.override = {}
        if w != meta["width"] or h != meta["height"]:
            # what handleWindowResize() + onApply recompute for a new canvas size (:521-537, :815-816)
            vlen = path_uniform(meta["frames"][0], "uVLen")
            self.override = {"uResolution": ["f", [float(w), float(h)]], "uULen": ["f", [vlen * (w / h)]]}

    def play_call(self, call, uniform_override=None):
        wr = self.wrappers[call["effect"]]
        fx = wr.effect
        uniforms = dict(call["uniforms"])
        uniforms.update({k: v for k, v in self.override.items() if k in uniforms})
        if uniform_override:
            uniforms.update({k: v for k, v in uniform_override.items() if k in uniforms})
        for name, ent in uniforms.items():
            fx._set_entry(name, ent)
        for name, tex in call["samplers"].items():
            fx.setTexture(name, self.textures.get(tex) if tex else None)
        target = self.textures[call["target"]] if call["target"] else None
        self.renderer.render(wr, target)

    def play_frame(self, i, uniform_override=None):
        for call in self.meta["frames"][i]:
            self.play_call(call, uniform_override)

    def synth_frame(self, k, seed=12345):
        """Frame k after the recording ends, camera still: what the render loop pushes next
        (uFrameCounter/uSampleCounter += 1, uCameraIsMoving false, a fresh uRandomVec2)."""
        last = self.meta["frames"][-1]
        fc = path_uniform(last, "uFrameCounter") + 1 + k
        sc = path_uniform(last, "uSampleCounter") + 1 + k
        r = splitmix64_uniforms(seed * 1000003 + k, 2)
        frame = []
        for call in last:
            c = dict(call)
            u = dict(call["uniforms"])
            if "uFrameCounter" in u:
                u["uFrameCounter"] = ["f", [float(fc)]]
                u["uSampleCounter"] = ["f", [float(sc)]]
                u["uCameraIsMoving"] = ["i", [0]]
                u["uRandomVec2"] = ["f", r]
                u["uTime"] = ["f", [u["uTime"][1][0] + (k + 1) / 60.0]]
            if "uOneOverSampleCounter" in u:
                u["uOneOverSampleCounter"] = ["f", [1.0 / sc]]
            c["uniforms"] = u
            frame.append(c)
        return frame


def path_uniform(frame, name):
    for c in frame:
        if c["shader"] == "pathTracingFragmentShader":
            return c["uniforms"][name][1][0]
    raise KeyError(name)


# ------------------------------------------------------------------------------------------------
# Multi-GPU framebuffer bands (pt_set_row_partition): 16-row bands dealt round-robin to ranks.
# The helpers work on torch tensors on any device, so the same code runs on RCCL (GPU) and gloo (CPU).

BAND = 16


def padded_bands(height, world):
    """Band count padded to a multiple of `world`, so every rank owns the same number of bands."""
    nb = (height + BAND - 1) // BAND
    return ((nb + world - 1) // world) * world


def bands_owned(height, world, rank):
    """How many 16-row bands rank `rank` shades (pt_set_row_partition: bands b with b % world == rank)."""
    nb = (height + BAND - 1) // BAND
    return (nb - rank + world - 1) // world if rank < nb else 0


def owned_rows(height, world, rank):
    """Rows of the frame this rank shades (bands b with b % world == rank)."""
    rows = []
    for b in range(rank, (height + BAND - 1) // BAND, world):
        rows.extend(range(b * BAND, min(height, (b + 1) * BAND)))
    return rows


def band_view(acc_padded, world):
    """View a band-padded (padded_bands*16, W, 4) accumulation as (bands/world, world, 16, W, 4):
    [:, r] is rank r's share, strided in memory (no repacking of the frame)."""
    rows, w, c = acc_padded.shape
    return acc_padded.view(rows // (BAND * world), world, BAND, w, c)


def gather_bands(dist, acc_padded, world, rank, send_buf, gather_list, full_padded=None):
    """Gather every rank's bands of `acc_padded` into rank 0's `full_padded` (RCCL or gloo)."""
    send_buf.copy_(band_view(acc_padded, world)[:, rank])
    dist.gather(send_buf, gather_list if rank == 0 else None, dst=0)
    if rank == 0:
        fv = band_view(full_padded, world)
        for r in range(world):
            fv[:, r].copy_(gather_list[r])


def exchange_halos(dist, acc_padded, world, rank, bufs):
    """Before a partitioned screenOutput: fill the 2 rows above and below each of this rank's bands
    with the neighbouring bands' rows. Band b = g*world + r; its lower neighbour b-1 belongs to rank
    r-1 (mod world) and its upper neighbour b+1 to rank r+1, so every rank sends its bands' two top
    rows to rank r-1 and its two bottom rows to rank r+1 (one batched P2P round over RCCL or gloo),
    and lands what it receives at those rows' own places in the frame. `bufs` = halo_buffers(...)."""
    if world == 1:
        return
    bv = band_view(acc_padded, world)
    lo, hi = (rank - 1) % world, (rank + 1) % world
    bufs["send_top"].copy_(bv[:, rank, 0:2])
    bufs["send_bot"].copy_(bv[:, rank, BAND - 2:BAND])
    # the same posting order on every rank (tops first, then bottoms), so that at world 2, where both
    # neighbours are one rank, the two messages of a pair still match in order
    ops = [dist.P2POp(dist.isend, bufs["send_top"], lo), dist.P2POp(dist.isend, bufs["send_bot"], hi),
           dist.P2POp(dist.irecv, bufs["recv_top"], hi), dist.P2POp(dist.irecv, bufs["recv_bot"], lo)]
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    bv[:, lo, BAND - 2:BAND].copy_(bufs["recv_bot"])   # rank r-1's bottom rows, under our bands
    bv[:, hi, 0:2].copy_(bufs["recv_top"])              # rank r+1's top rows, over our bands


class PipelinedBandGather:
    """Per-frame gather of the ranks' RGBA8 bands to rank 0, overlapped with the next frame: two
    band-padded canvases alternate; frame k renders into target(), submit() starts its gather
    (async), and the gather that last used a buffer is waited for (and, on rank 0, assembled into
    a full frame) only when that buffer comes round again, two frames later, or at drain().
    On rank 0 `frames` collects (frame index, assembled canvas) in order when keep=True."""

    def __init__(self, dist, world, rank, rows, width, device, keep=False):
        import torch
        self.dist, self.world, self.rank, self.keep = dist, world, rank, keep
        self.canvas = [torch.zeros((rows, width, 4), dtype=torch.uint8, device=device) for _ in range(2)]
        self.send = [torch.zeros((rows // (BAND * world), BAND, width, 4), dtype=torch.uint8, device=device)
                     for _ in range(2)]
        self.glist = [[torch.empty_like(self.send[b]) for _ in range(world)] if rank == 0 else None for b in range(2)]
        self.full = [torch.zeros_like(self.canvas[0]) if rank == 0 else None for _ in range(2)]
        self.work = [None, None]
        self.frame_of = [None, None]
        self.k = 0
        self.frames = []

    def target(self):
        """The canvas tensor to render frame k into (its previous gather, two frames ago, is done)."""
        b = self.k % 2
        self._finish(b)
        return self.canvas[b]

    def submit(self):
        """Start gathering frame k's bands (after its screenOutput was enqueued on this stream)."""
        b = self.k % 2
        self.send[b].copy_(band_view(self.canvas[b], self.world)[:, self.rank])
        self.work[b] = self.dist.gather(self.send[b], self.glist[b], dst=0, async_op=True)
        self.frame_of[b] = self.k
        self.k += 1

    def _finish(self, b):
        if self.work[b] is None:
            return
        self.work[b].wait()
        self.work[b] = None
        if self.rank == 0:
            fv = band_view(self.full[b], self.world)
            for r in range(self.world):
                fv[:, r].copy_(self.glist[b][r])
            if self.keep:
                self.frames.append((self.frame_of[b], self.full[b].clone()))

    def drain(self):
        """Complete every outstanding gather, oldest first."""
        for b in sorted((b for b in range(2) if self.work[b] is not None), key=lambda b: self.frame_of[b]):
            self._finish(b)

    def last_frame(self):
        """Rank 0: the assembled canvas of the newest submitted frame (drains first)."""
        self.drain()
        done = [b for b in range(2) if self.frame_of[b] is not None]
        return self.full[max(done, key=lambda b: self.frame_of[b])] if done and self.rank == 0 else None


def halo_buffers(acc_padded, world):
    """Send/receive buffers for exchange_halos (same device and dtype as the accumulation)."""
    import torch
    rows, w, c = acc_padded.shape
    shape = (rows // (BAND * world), 2, w, c)
    return {k: torch.empty(shape, dtype=acc_padded.dtype, device=acc_padded.device)
            for k in ("send_top", "send_bot", "recv_top", "recv_bot")}


def load_stream(path):
    with open(path) as f:
        return json.load(f)
