/* pt_napi.c — Node N-API addon over libpt.so (include/pt.h).
 *
 * The reference's host is JavaScript (js/*_Path_Tracing.js driving Babylon's effect API). This
 * addon is the thin native layer that lets that JavaScript reach the gfx950 kernels: every C-ABI
 * entry point is exported one-to-one (handles are N-API externals, typed arrays are passed
 * zero-copy), and ../js/babylon_pt.js builds the Babylon-shaped classes on top.
 *
 * Error convention: functions return the pt_status code (0 = PT_OK) or a handle / null; they
 * never throw for a pt_status, mirroring Babylon's silent render of a non-ready effect. They do
 * throw a TypeError for malformed JavaScript arguments.
 */
#include <node_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pt.h"

#define MAXARGS 8
#define CHECK(call) do { if ((call) != napi_ok) { napi_throw_error(env, NULL, #call " failed"); return NULL; } } while (0)

static napi_value num(napi_env env, double v) { napi_value r; napi_create_double(env, v, &r); return r; }
static napi_value nul(napi_env env) { napi_value r; napi_get_null(env, &r); return r; }

static int args(napi_env env, napi_callback_info info, napi_value* argv, size_t want)
{
    size_t argc = MAXARGS;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return -1;
    for (size_t i = argc; i < MAXARGS; i++) argv[i] = NULL;
    if (argc < want) { napi_throw_type_error(env, NULL, "too few arguments"); return -1; }
    return (int)argc;
}
static void* handle(napi_env env, napi_value v)
{
    napi_valuetype t;
    if (!v || napi_typeof(env, v, &t) != napi_ok || t == napi_null || t == napi_undefined) return NULL;
    void* p = NULL;
    if (t == napi_external) napi_get_value_external(env, v, &p);
    return p;
}
static napi_value ext(napi_env env, void* p)
{
    if (!p) return nul(env);
    napi_value r;
    napi_create_external(env, p, NULL, NULL, &r);
    return r;
}
static int i32(napi_env env, napi_value v) { int32_t x = 0; napi_get_value_int32(env, v, &x); return x; }
static double f64(napi_env env, napi_value v) { double x = 0; napi_get_value_double(env, v, &x); return x; }
static char* str(napi_env env, napi_value v)
{
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) return NULL;
    char* s = (char*)malloc(n + 1);
    napi_get_value_string_utf8(env, v, s, n + 1, &n);
    return s;
}
/* typed array or ArrayBuffer -> data pointer + byte length */
static void* bytes_of(napi_env env, napi_value v, size_t* len)
{
    bool is;
    void* data = NULL;
    *len = 0;
    if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
        napi_typedarray_type tt; size_t n; napi_value ab; size_t off;
        napi_get_typedarray_info(env, v, &tt, &n, &data, &ab, &off);
        size_t el = (tt == napi_float32_array || tt == napi_int32_array || tt == napi_uint32_array) ? 4 :
                    (tt == napi_float64_array || tt == napi_bigint64_array || tt == napi_biguint64_array) ? 8 :
                    (tt == napi_int16_array || tt == napi_uint16_array) ? 2 : 1;
        *len = n * el;
        return data;
    }
    if (napi_is_arraybuffer(env, v, &is) == napi_ok && is) {
        napi_get_arraybuffer_info(env, v, &data, len);
        return data;
    }
    return NULL;
}
/* JS string[] -> char*[] */
static char** strings(napi_env env, napi_value arr, uint32_t* n)
{
    *n = 0;
    bool is = false;
    if (!arr || napi_is_array(env, arr, &is) != napi_ok || !is) return NULL;
    napi_get_array_length(env, arr, n);
    char** out = (char**)calloc(*n ? *n : 1, sizeof(char*));
    for (uint32_t i = 0; i < *n; i++) { napi_value e; napi_get_element(env, arr, i, &e); out[i] = str(env, e); }
    return out;
}
static void free_strings(char** s, uint32_t n) { for (uint32_t i = 0; i < n; i++) free(s[i]); free(s); }

/* ---------------------------------------------------------------- context */
static napi_value CtxCreate(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL;
    int err = 0;
    pt_ctx* c = pt_ctx_create(i32(env, a[0]), &err);
    return c ? ext(env, c) : num(env, err);
}
/* pt_ctx_create_devices(devices[]): a JS array of HIP device ids, one part each */
static napi_value CtxCreateDevices(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL;
    uint32_t n = 0;
    bool isarr = false;
    if (napi_is_array(env, a[0], &isarr) != napi_ok || !isarr || napi_get_array_length(env, a[0], &n) != napi_ok || n == 0 || n > 64) {
        napi_throw_type_error(env, NULL, "pt_ctx_create_devices: expected a non-empty array of device ids");
        return NULL;
    }
    int devs[64];
    for (uint32_t i = 0; i < n; i++) { napi_value v; CHECK(napi_get_element(env, a[0], i, &v)); devs[i] = i32(env, v); }
    int err = 0;
    pt_ctx* c = pt_ctx_create_devices(devs, (int)n, &err);
    return c ? ext(env, c) : num(env, err);
}
static napi_value CtxCreateMask(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL;
    uint32_t m = 0; napi_get_value_uint32(env, a[0], &m);
    int err = 0;
    pt_ctx* c = pt_ctx_create_mask(m, &err);
    return c ? ext(env, c) : num(env, err);
}
static napi_value CtxParts(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_ctx_parts((pt_ctx*)handle(env, a[0]))); }
static napi_value CtxPeerCopies(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_ctx_peer_copies((pt_ctx*)handle(env, a[0]))); }
static napi_value CtxDestroy(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; pt_ctx_destroy((pt_ctx*)handle(env, a[0])); return nul(env); }
static napi_value LastError(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    CHECK(napi_create_string_utf8(env, pt_last_error((pt_ctx*)handle(env, a[0])), NAPI_AUTO_LENGTH, &r));
    return r;
}
static napi_value Sync(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_sync((pt_ctx*)handle(env, a[0]))); }
static napi_value CanvasResize(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL; return num(env, pt_canvas_resize((pt_ctx*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]))); }

/* ---------------------------------------------------------------- effects */
static napi_value EffectCreate(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    uint32_t nu = 0, ns = 0;
    char* src = str(env, a[1]);
    char** un = strings(env, a[2], &nu);
    char** sn = strings(env, a[3], &ns);
    int err = 0;
    pt_effect* fx = pt_effect_create((pt_ctx*)handle(env, a[0]), src, (const char* const*)un, (int)nu, (const char* const*)sn, (int)ns, &err);
    free(src); free_strings(un, nu); free_strings(sn, ns);
    return fx ? ext(env, fx) : num(env, err);
}
static napi_value EffectCreateProgram(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    uint32_t nu = 0, ns = 0;
    char** un = strings(env, a[2], &nu);
    char** sn = strings(env, a[3], &ns);
    int err = 0;
    pt_effect* fx = pt_effect_create_program((pt_ctx*)handle(env, a[0]), i32(env, a[1]), (const char* const*)un, (int)nu, (const char* const*)sn, (int)ns, &err);
    free_strings(un, nu); free_strings(sn, ns);
    return fx ? ext(env, fx) : num(env, err);
}
static napi_value EffectDestroy(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; pt_effect_destroy((pt_effect*)handle(env, a[0])); return nul(env); }
static napi_value EffectProgram(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_effect_program((pt_effect*)handle(env, a[0]))); }

static napi_value SetFloat(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    float v[16];
    int n = 0;
    bool is = false;
    napi_valuetype t;
    napi_typeof(env, a[2], &t);
    if (t == napi_number) { v[0] = (float)f64(env, a[2]); n = 1; }
    else if (napi_is_array(env, a[2], &is) == napi_ok && is) {
        uint32_t len; napi_get_array_length(env, a[2], &len);
        for (uint32_t i = 0; i < len && i < 16; i++) { napi_value e; napi_get_element(env, a[2], i, &e); v[n++] = (float)f64(env, e); }
    } else {
        size_t len; float* p = (float*)bytes_of(env, a[2], &len);
        if (!p) { napi_throw_type_error(env, NULL, "setFloat expects a number, array or Float32Array"); return NULL; }
        for (size_t i = 0; i < len / 4 && i < 16; i++) v[n++] = p[i];
    }
    char* name = str(env, a[1]);
    int rc = pt_set_float((pt_effect*)handle(env, a[0]), name, v, n);
    free(name);
    return num(env, rc);
}
static napi_value SetInt(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    char* name = str(env, a[1]);
    napi_valuetype t; napi_typeof(env, a[2], &t);
    int v = 0;
    if (t == napi_boolean) { bool b; napi_get_value_bool(env, a[2], &b); v = b ? 1 : 0; } else v = i32(env, a[2]);
    int rc = pt_set_int((pt_effect*)handle(env, a[0]), name, v);
    free(name);
    return num(env, rc);
}
static napi_value SetTexture(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    char* name = str(env, a[1]);
    int rc = pt_set_texture((pt_effect*)handle(env, a[0]), name, (pt_texture*)handle(env, a[2]));
    free(name);
    return num(env, rc);
}

/* ---------------------------------------------------------------- textures */
static napi_value TexF32(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    size_t len; const float* p = (const float*)bytes_of(env, a[3], &len);
    int w = i32(env, a[1]), h = i32(env, a[2]), err = 0;
    if (!p || len < (size_t)w * h * 16) { napi_throw_type_error(env, NULL, "Float32Array of w*h*4 expected"); return NULL; }
    pt_texture* t = pt_texture_create_rgba32f((pt_ctx*)handle(env, a[0]), w, h, p, a[4] ? i32(env, a[4]) : 1, a[5] ? i32(env, a[5]) : 0, &err);
    return t ? ext(env, t) : num(env, err);
}
static napi_value TexU8(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    size_t len; const uint8_t* p = (const uint8_t*)bytes_of(env, a[3], &len);
    int w = i32(env, a[1]), h = i32(env, a[2]), err = 0;
    if (!p || len < (size_t)w * h * 4) { napi_throw_type_error(env, NULL, "Uint8Array of w*h*4 expected"); return NULL; }
    pt_texture* t = pt_texture_create_rgba8((pt_ctx*)handle(env, a[0]), w, h, p, a[4] ? i32(env, a[4]) : 1, a[5] ? i32(env, a[5]) : 0, &err);
    return t ? ext(env, t) : num(env, err);
}
static napi_value RtCreate(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    int err = 0;
    pt_texture* t = pt_render_target_create((pt_ctx*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]), &err);
    return t ? ext(env, t) : num(env, err);
}
static napi_value RtWrap(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    uint64_t ptr = 0; bool lossless;
    napi_get_value_bigint_uint64(env, a[3], &ptr, &lossless);
    int err = 0;
    pt_texture* t = pt_render_target_wrap((pt_ctx*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]), (void*)(uintptr_t)ptr, &err);
    return t ? ext(env, t) : num(env, err);
}
static napi_value RtResize(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL; return num(env, pt_render_target_resize((pt_texture*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]))); }
static napi_value TexSize(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    int w = 0, h = 0;
    pt_texture_size((pt_texture*)handle(env, a[0]), &w, &h);
    CHECK(napi_create_array_with_length(env, 2, &r));
    napi_set_element(env, r, 0, num(env, w));
    napi_set_element(env, r, 1, num(env, h));
    return r;
}
static napi_value TexDestroy(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; pt_texture_destroy((pt_texture*)handle(env, a[0])); return nul(env); }
static napi_value TexDevicePtr(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    CHECK(napi_create_bigint_uint64(env, (uint64_t)(uintptr_t)pt_texture_device_ptr((pt_texture*)handle(env, a[0])), &r));
    return r;
}

/* ---------------------------------------------------------------- draw / readback */
static napi_value Render(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_render((pt_effect*)handle(env, a[0]), (pt_texture*)handle(env, a[1]))); }
static napi_value ReadPixels(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    size_t len; void* p = bytes_of(env, a[2], &len);
    if (!p) { napi_throw_type_error(env, NULL, "typed array expected"); return NULL; }
    return num(env, pt_read_pixels((pt_ctx*)handle(env, a[0]), (const pt_texture*)handle(env, a[1]), p, len));
}
static napi_value WritePixels(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    size_t len; void* p = bytes_of(env, a[2], &len);
    if (!p) { napi_throw_type_error(env, NULL, "typed array expected"); return NULL; }
    return num(env, pt_write_pixels((pt_ctx*)handle(env, a[0]), (pt_texture*)handle(env, a[1]), p, len));
}

/* ---------------------------------------------------------------- MI355X extensions */
static napi_value RowPartition(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL; return num(env, pt_set_row_partition((pt_ctx*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]))); }
static napi_value SetBackend(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL; return num(env, pt_set_backend((pt_ctx*)handle(env, a[0]), i32(env, a[1]))); }
static napi_value SetOutputPartition(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL; return num(env, pt_set_output_partition((pt_ctx*)handle(env, a[0]), i32(env, a[1]))); }
static napi_value CanvasWrap(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    uint64_t ptr = 0; bool lossless;
    napi_valuetype t; napi_typeof(env, a[3], &t);
    if (t == napi_bigint) napi_get_value_bigint_uint64(env, a[3], &ptr, &lossless);
    return num(env, pt_canvas_wrap((pt_ctx*)handle(env, a[0]), i32(env, a[1]), i32(env, a[2]), (void*)(uintptr_t)ptr));
}
static napi_value SetBvhLayout(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL; return num(env, pt_set_bvh_layout((pt_ctx*)handle(env, a[0]), i32(env, a[1]))); }
static napi_value BvhLayoutUsed(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_bvh_layout_used((pt_ctx*)handle(env, a[0]))); }
static napi_value SetStream(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL;
    uint64_t ptr = 0; bool lossless;
    napi_valuetype t; napi_typeof(env, a[1], &t);
    if (t == napi_bigint) napi_get_value_bigint_uint64(env, a[1], &ptr, &lossless);
    return num(env, pt_set_stream((pt_ctx*)handle(env, a[0]), (void*)(uintptr_t)ptr));
}
static napi_value LastRenderMs(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL;
    float ms = -1.0f;
    int rc = pt_last_render_ms((pt_ctx*)handle(env, a[0]), i32(env, a[1]), &ms);
    return num(env, rc == PT_OK ? ms : -1.0);
}
static napi_value TimingBegin(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_timing_begin((pt_ctx*)handle(env, a[0]))); }
static napi_value TimingEnd(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 2) < 0) return NULL;
    double ms = 0; int n = 0;
    int rc = pt_timing_end((pt_ctx*)handle(env, a[0]), i32(env, a[1]), &ms, &n);
    CHECK(napi_create_array_with_length(env, 3, &r));
    napi_set_element(env, r, 0, num(env, rc));
    napi_set_element(env, r, 1, num(env, ms));
    napi_set_element(env, r, 2, num(env, n));
    return r;
}
static napi_value TimingLatency(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 2) < 0) return NULL;
    float ms[1024]; int n = 0;
    int rc = pt_timing_latency((pt_ctx*)handle(env, a[0]), i32(env, a[1]), ms, 1024, &n);
    if (rc != PT_OK) n = 0;
    CHECK(napi_create_array_with_length(env, (size_t)n + 1, &r));
    napi_set_element(env, r, 0, num(env, rc));
    for (int i = 0; i < n; i++) napi_set_element(env, r, (uint32_t)i + 1, num(env, ms[i]));
    return r;
}
static napi_value SetCounting(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL; return num(env, pt_set_counting((pt_ctx*)handle(env, a[0]), i32(env, a[1]))); }
static napi_value ReadCounters(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    uint64_t c[PT_NUM_COUNTERS] = { 0 };
    pt_read_counters((pt_ctx*)handle(env, a[0]), c);
    CHECK(napi_create_array_with_length(env, PT_NUM_COUNTERS, &r));
    for (uint32_t i = 0; i < PT_NUM_COUNTERS; i++) napi_set_element(env, r, i, num(env, (double)c[i]));
    return r;
}
static napi_value ResetCounters(napi_env env, napi_callback_info info)
{ napi_value a[MAXARGS]; if (args(env, info, a, 1) < 0) return NULL; return num(env, pt_reset_counters((pt_ctx*)handle(env, a[0]))); }
static napi_value QueueStats(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    uint32_t q[16] = { 0 };
    pt_queue_stats((pt_ctx*)handle(env, a[0]), q);
    CHECK(napi_create_array_with_length(env, 16, &r));
    for (uint32_t i = 0; i < 16; i++) napi_set_element(env, r, i, num(env, q[i]));
    return r;
}
/* pt_bvh_build(aabbIn: Float32Array (9 per triangle), work: Uint32Array, out: Float32Array) -> node count */
static napi_value BvhBuild(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 3) < 0) return NULL;
    size_t la, lw, lo;
    const float* aabb = (const float*)bytes_of(env, a[0], &la);
    const uint32_t* work = (const uint32_t*)bytes_of(env, a[1], &lw);
    float* out = (float*)bytes_of(env, a[2], &lo);
    int n = (int)(lw / 4);
    if (!aabb || !work || !out || la < (size_t)n * 36) return num(env, PT_ERR_ARG);
    return num(env, pt_bvh_build(aabb, work, n, out, (int)(lo / 32)));
}
/* pt_bvh_build_gpu(device, aabbIn, work, out) -> node count (the device build, same bits) */
static napi_value BvhBuildGpu(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 4) < 0) return NULL;
    int32_t dev = 0;
    CHECK(napi_get_value_int32(env, a[0], &dev));
    size_t la, lw, lo;
    const float* aabb = (const float*)bytes_of(env, a[1], &la);
    const uint32_t* work = (const uint32_t*)bytes_of(env, a[2], &lw);
    float* out = (float*)bytes_of(env, a[3], &lo);
    int n = (int)(lw / 4);
    if (!aabb || !work || !out) return num(env, PT_ERR_ARG);
    for (int i = 0; i < n; i++)
        if ((size_t)work[i] * 36 + 36 > la) return num(env, PT_ERR_ARG);
    return num(env, pt_bvh_build_gpu(dev, aabb, work, n, out, (int)(lo / 32), NULL));
}
/* pt_jpeg_size(bytes: Uint8Array) -> [width, height] or a negative pt_status */
static napi_value JpegSize(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS], r; if (args(env, info, a, 1) < 0) return NULL;
    size_t n; const uint8_t* d = (const uint8_t*)bytes_of(env, a[0], &n);
    int w = 0, h = 0;
    const int rc = d ? pt_jpeg_size(d, n, &w, &h) : PT_ERR_ARG;
    if (rc != PT_OK) return num(env, rc);
    CHECK(napi_create_array_with_length(env, 2, &r));
    napi_set_element(env, r, 0, num(env, w));
    napi_set_element(env, r, 1, num(env, h));
    return r;
}
/* pt_jpeg_decode_rgba8(bytes: Uint8Array, out: Uint8Array (4 * w * h)) -> status */
static napi_value JpegDecode(napi_env env, napi_callback_info info)
{
    napi_value a[MAXARGS]; if (args(env, info, a, 2) < 0) return NULL;
    size_t n, cap;
    const uint8_t* d = (const uint8_t*)bytes_of(env, a[0], &n);
    uint8_t* out = (uint8_t*)bytes_of(env, a[1], &cap);
    if (!d || !out) return num(env, PT_ERR_ARG);
    return num(env, pt_jpeg_decode_rgba8(d, n, out, cap));
}
static napi_value Version(napi_env env, napi_callback_info info)
{
    napi_value r; (void)info;
    CHECK(napi_create_string_utf8(env, pt_version(), NAPI_AUTO_LENGTH, &r));
    return r;
}

static napi_value Init(napi_env env, napi_value exports)
{
    static const struct { const char* name; napi_callback fn; } F[] = {
        { "pt_ctx_create", CtxCreate }, { "pt_ctx_create_devices", CtxCreateDevices }, { "pt_ctx_create_mask", CtxCreateMask },
        { "pt_ctx_peer_copies", CtxPeerCopies }, { "pt_ctx_parts", CtxParts }, { "pt_ctx_destroy", CtxDestroy }, { "pt_last_error", LastError },
        { "pt_sync", Sync }, { "pt_canvas_resize", CanvasResize },
        { "pt_effect_create", EffectCreate }, { "pt_effect_create_program", EffectCreateProgram },
        { "pt_effect_destroy", EffectDestroy }, { "pt_effect_program", EffectProgram },
        { "pt_set_float", SetFloat }, { "pt_set_int", SetInt }, { "pt_set_texture", SetTexture },
        { "pt_texture_create_rgba32f", TexF32 }, { "pt_texture_create_rgba8", TexU8 },
        { "pt_render_target_create", RtCreate }, { "pt_render_target_wrap", RtWrap },
        { "pt_render_target_resize", RtResize }, { "pt_texture_size", TexSize }, { "pt_texture_destroy", TexDestroy },
        { "pt_render", Render }, { "pt_read_pixels", ReadPixels }, { "pt_write_pixels", WritePixels },
        { "pt_set_row_partition", RowPartition }, { "pt_set_backend", SetBackend }, { "pt_set_output_partition", SetOutputPartition }, { "pt_canvas_wrap", CanvasWrap }, { "pt_set_bvh_layout", SetBvhLayout },
        { "pt_bvh_layout_used", BvhLayoutUsed }, { "pt_set_stream", SetStream }, { "pt_texture_device_ptr", TexDevicePtr },
        { "pt_last_render_ms", LastRenderMs }, { "pt_timing_begin", TimingBegin }, { "pt_timing_end", TimingEnd },
        { "pt_timing_latency", TimingLatency },
        { "pt_set_counting", SetCounting }, { "pt_read_counters", ReadCounters }, { "pt_reset_counters", ResetCounters }, { "pt_queue_stats", QueueStats },
        { "pt_bvh_build", BvhBuild }, { "pt_bvh_build_gpu", BvhBuildGpu },
        { "pt_jpeg_size", JpegSize }, { "pt_jpeg_decode_rgba8", JpegDecode }, { "pt_version", Version },
    };
    for (size_t i = 0; i < sizeof(F) / sizeof(F[0]); i++) {
        napi_value fn;
        if (napi_create_function(env, F[i].name, NAPI_AUTO_LENGTH, F[i].fn, NULL, &fn) != napi_ok) return NULL;
        if (napi_set_named_property(env, exports, F[i].name, fn) != napi_ok) return NULL;
    }
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
