// pt_group.cpp — the exported C ABI of libpt.so (include/pt.h). A context is one or more parts,
// each a Dev (pt_dev.h: one HIP stream on one gfx950 device); every texture, render target and
// effect exists once per part, and every call is forwarded to each part. This is where the
// multi-GPU fan-out the reference's render loop never sees happens (the unmodified
// js/GLTF_Model_Path_Tracing.js:1230-1235 issues eRenderer.render(...) three times per frame):
//
//   * the frame is cut into 16-row bands dealt round-robin: part k shades bands b % N == k
//     (path tracing and screenCopy touch only those texels, so render targets stay distributed:
//     every texel is valid on the part that owns its band);
//   * screenOutput reads +-2 rows around each band, so before it each part pulls the 2 rows below
//     and above its bands from its band neighbours (parts k-1 and k+1) - device-to-device 2D
//     copies over xGMI (peer access), one per neighbour, strided by N bands;
//   * screenOutput writes each part's bands of its own canvas, and part 0 gathers the other parts'
//     bands into its canvas (the one pt_read_pixels(ctx, NULL) returns): RGBA8, 4 B per pixel;
//   * cross-part ordering is by HIP events only, no host sync inside a frame: a part's path
//     tracing waits for its neighbours' last output (which pulled halo rows from its accumulation
//     target), a part's output waits for its neighbours' last path tracing and for the previous
//     gather (which read its canvas), the gather waits for every part's output.
//
// With one part (pt_ctx_create) every call is a plain forward to that part.
#include "../../include/pt.h"
#include "pt_dev.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace {
constexpr int kBand = 16;   // row-band height (pt_args.h kTile)
enum Kind { K_F32 = 0, K_U8 = 1, K_RT = 2 };
}  // namespace

struct pt_texture;

struct pt_ctx {
    std::vector<Dev*> parts;
    std::vector<hipEvent_t> ev_draw, ev_out;   // per part: after its last path-tracing draw / output
    std::vector<bool> has_draw, has_out;
    hipEvent_t ev_gather = nullptr;            // part 0: after the last canvas gather
    bool has_gather = false;
    // peer access between every two distinct devices of the context: the halo pulls and the gather are
    // strided 2D copies over xGMI. Without it (hipDeviceCanAccessPeer false, hipDeviceEnablePeerAccess
    // failing, or PT_PEER=0) they go band by band through hipMemcpyPeerAsync, which the runtime stages
    std::vector<int> devs;
    bool peer = true;
    int cw = 0, ch = 0;
    std::string err;
    std::set<pt_texture*> textures;
    std::set<pt_effect*> effects;
    int n() const { return (int)parts.size(); }
};

struct pt_texture {
    pt_ctx* ctx = nullptr;
    std::vector<DevTex*> sub;
    int kind = K_F32;
    int w = 0, h = 0;
};

struct pt_effect {
    pt_ctx* ctx = nullptr;
    std::vector<DevFx*> sub;
    int prog = PT_PROG_UNKNOWN;
    std::unordered_map<std::string, pt_texture*> bound;   // sampler -> texture (for the halo source)
};

namespace {

int fail(pt_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

// a part's error -> the context's message
int take(pt_ctx* c, int k, int rc)
{
    if (rc != PT_OK) c->err = "part " + std::to_string(k) + ": " + dev_last_error(c->parts[k]);
    return rc;
}

int hipfail(pt_ctx* c, hipError_t e, const char* what)
{
    return fail(c, PT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define GHIP(c, call)                                      \
    do {                                                   \
        hipError_t e_ = (call);                            \
        if (e_ != hipSuccess) return hipfail(c, e_, #call); \
    } while (0)

bool is_trace(int prog)
{
    return prog == PT_PROG_CORNELL || prog == PT_PROG_GLTF || prog == PT_PROG_HDRI || prog == PT_PROG_SKY ||
           prog == PT_PROG_QUADRIC || prog == PT_PROG_SKY_MESH;
}

// Rows [b*16 + off, b*16 + off + nrows) of the bands b = b0, b0 + N, b0 + 2N, ... (count of them),
// clipped to [0, H), from src to dst (same row layout, `rowbytes` per row): one strided 2D copy for
// the bands whose rows all lie inside the image, single copies for the (at most two) clipped ones.
//
// Peer fallback (dst_dev >= 0): one hipMemcpyPeerAsync per band (its rows are contiguous), from src_dev.
hipError_t copy_band_rows(char* dst, const char* src, size_t rowbytes, int N, int b0, int count, int off, int nrows,
                          int H, hipMemcpyKind kind, hipStream_t s, int dst_dev = -1, int src_dev = -1)
{
    if (count <= 0) return hipSuccess;
    auto row0 = [&](int m) { return (long)(b0 + (long)m * N) * kBand + off; };
    if (dst_dev >= 0) {
        hipError_t e = hipSuccess;
        for (int m = 0; m < count && e == hipSuccess; m++) {
            const long r0 = std::max(0L, row0(m)), r1 = std::min((long)H, row0(m) + nrows);
            if (r1 > r0)
                e = hipMemcpyPeerAsync(dst + r0 * rowbytes, dst_dev, src + r0 * rowbytes, src_dev,
                                       (size_t)(r1 - r0) * rowbytes, s);
        }
        return e;
    }
    int lo = 0, hi = count - 1;
    while (lo <= hi && row0(lo) < 0) lo++;
    while (hi >= lo && row0(hi) + nrows > H) hi--;
    hipError_t e = hipSuccess;
    if (lo <= hi) {
        const size_t pitch = (size_t)N * kBand * rowbytes;
        const size_t at = (size_t)row0(lo) * rowbytes;
        e = hipMemcpy2DAsync(dst + at, pitch, src + at, pitch, nrows * rowbytes, (size_t)(hi - lo + 1), kind, s);
    }
    for (int m = 0; m < count && e == hipSuccess; m++) {
        if (m >= lo && m <= hi) continue;
        const long r0 = std::max(0L, row0(m)), r1 = std::min((long)H, row0(m) + nrows);
        if (r1 > r0)
            e = hipMemcpyAsync(dst + r0 * rowbytes, src + r0 * rowbytes, (size_t)(r1 - r0) * rowbytes, kind, s);
    }
    return e;
}

int bands_of(int nb, int N, int k) { return k < nb ? (nb - k + N - 1) / N : 0; }

int wait(pt_ctx* c, int k, hipEvent_t e, bool recorded)
{
    if (recorded) GHIP(c, hipStreamWaitEvent(dev_stream(c->parts[k]), e, 0));
    return PT_OK;
}

int record(pt_ctx* c, int k, hipEvent_t e)
{
    GHIP(c, hipSetDevice(dev_device(c->parts[k])));
    GHIP(c, hipEventRecord(e, dev_stream(c->parts[k])));
    return PT_OK;
}

// screenOutput over N parts: halo rows, each part's bands, gather to part 0's canvas
int render_output_parts(pt_effect* fx, pt_texture* target)
{
    pt_ctx* c = fx->ctx;
    const int N = c->n();
    auto it = fx->bound.find("accumulationBuffer");
    pt_texture* acc = it == fx->bound.end() ? nullptr : it->second;
    for (int j = 0; j < N; j++) {
        Dev* d = c->parts[j];
        GHIP(c, hipSetDevice(dev_device(d)));
        const int lo = (j + N - 1) % N, hi = (j + 1) % N;
        if (int rc = wait(c, j, c->ev_draw[lo], c->has_draw[lo])) return rc;
        if (int rc = wait(c, j, c->ev_draw[hi], c->has_draw[hi])) return rc;
        if (!target)   // the previous gather read this part's canvas
            if (int rc = wait(c, j, c->ev_gather, c->has_gather)) return rc;
        if (acc && acc->kind != K_U8) {
            // rows 2 below / 2 above each owned band, from the parts that own those bands
            const int nb = (acc->h + kBand - 1) / kBand;
            const size_t rb = (size_t)acc->w * 16;
            char* dst = (char*)dev_texture_device_ptr(acc->sub[j]);
            const int cnt = bands_of(nb, N, j);
            const int dd = c->peer ? -1 : c->devs[j];
            GHIP(c, copy_band_rows(dst, (const char*)dev_texture_device_ptr(acc->sub[lo]), rb, N, j, cnt, -2, 2, acc->h,
                                   hipMemcpyDefault, dev_stream(d), dd, c->devs[lo]));
            GHIP(c, copy_band_rows(dst, (const char*)dev_texture_device_ptr(acc->sub[hi]), rb, N, j, cnt, kBand, 2, acc->h,
                                   hipMemcpyDefault, dev_stream(d), dd, c->devs[hi]));
        }
        if (int rc = take(c, j, dev_render(fx->sub[j], target ? target->sub[j] : nullptr))) return rc;
        if (int rc = record(c, j, c->ev_out[j])) return rc;
        c->has_out[j] = true;
    }
    if (target) return PT_OK;
    // gather every part's bands of the RGBA8 canvas into part 0's
    Dev* d0 = c->parts[0];
    GHIP(c, hipSetDevice(dev_device(d0)));
    char* dst = (char*)dev_canvas_ptr(d0);
    int cw = c->cw, ch = c->ch;
    if (cw == 0 && ch == 0 && acc) { cw = acc->w; ch = acc->h; }
    const int nb = (ch + kBand - 1) / kBand;
    for (int k = 1; k < N; k++) {
        if (int rc = wait(c, 0, c->ev_out[k], true)) return rc;
        GHIP(c, copy_band_rows(dst, (const char*)dev_canvas_ptr(c->parts[k]), (size_t)cw * 4, N, k, bands_of(nb, N, k), 0,
                               kBand, ch, hipMemcpyDefault, dev_stream(d0), c->peer ? -1 : c->devs[0], c->devs[k]));
    }
    if (int rc = record(c, 0, c->ev_gather)) return rc;
    c->has_gather = true;
    return PT_OK;
}

template <class F>
pt_texture* make_tex(pt_ctx* c, int kind, int w, int h, int* err, F create)
{
    if (err) *err = PT_OK;
    if (!c) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* t = new pt_texture();
    t->ctx = c; t->kind = kind; t->w = w; t->h = h;
    for (int k = 0; k < c->n(); k++) {
        int rc = PT_OK;
        DevTex* d = create(c->parts[k], &rc);
        if (!d) {
            take(c, k, rc);
            for (auto* s : t->sub) dev_texture_destroy(s);
            delete t;
            if (err) *err = rc ? rc : PT_ERR_HIP;
            return nullptr;
        }
        t->sub.push_back(d);
    }
    c->textures.insert(t);
    return t;
}
}  // namespace

extern "C" {

const char* pt_version(void) { return "libpt 0.2.0 gfx950"; }

pt_ctx* pt_ctx_create_devices(const int* devices, int n, int* err)
{
    if (err) *err = PT_OK;
    if (!devices || n < 1 || n > 64) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* c = new pt_ctx();
    int rc = PT_OK;
    for (int k = 0; k < n && rc == PT_OK; k++) {
        Dev* d = dev_ctx_create(devices[k], &rc);
        if (!d) break;
        c->parts.push_back(d);
        if (n > 1) {
            rc = dev_set_row_partition(d, n, k);
            if (rc == PT_OK) rc = dev_set_output_partition(d, 1);
        }
    }
    // peer access between the distinct devices of the context (halo pulls, the gather); where a pair has
    // none, every copy of the context takes the per-band hipMemcpyPeerAsync path instead (pt_ctx::peer)
    c->devs.assign(devices, devices + n);
    if (const char* v = std::getenv("PT_PEER")) c->peer = std::atoi(v) != 0;
    std::vector<int> uniq(devices, devices + n);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    for (size_t a = 0; a < uniq.size() && rc == PT_OK && c->peer; a++)
        for (size_t b = 0; b < uniq.size() && c->peer; b++) {
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, uniq[a], uniq[b]) != hipSuccess || !can) { c->peer = false; break; }
            hipSetDevice(uniq[a]);
            hipError_t e = hipDeviceEnablePeerAccess(uniq[b], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) c->peer = false;
            (void)hipGetLastError();
        }
    for (int k = 0; k < (int)c->parts.size() && rc == PT_OK && n > 1; k++) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipSetDevice(devices[k]) != hipSuccess || hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) { rc = PT_ERR_HIP; break; }
        c->ev_draw.push_back(a); c->ev_out.push_back(b);
        if (k == 0 && hipEventCreateWithFlags(&c->ev_gather, hipEventDisableTiming) != hipSuccess) rc = PT_ERR_HIP;
    }
    c->has_draw.assign(n, false);
    c->has_out.assign(n, false);
    if (rc != PT_OK || (int)c->parts.size() != n) {
        if (err) *err = rc != PT_OK ? rc : PT_ERR_DEVICE;
        pt_ctx_destroy(c);
        return nullptr;
    }
    return c;
}

pt_ctx* pt_ctx_create(int device, int* err) { return pt_ctx_create_devices(&device, 1, err); }

pt_ctx* pt_ctx_create_mask(uint32_t device_mask, int* err)
{
    int devs[32], n = 0;
    for (int d = 0; d < 32; d++)
        if (device_mask & (1u << d)) devs[n++] = d;
    if (n == 0) { if (err) *err = PT_ERR_ARG; return nullptr; }
    return pt_ctx_create_devices(devs, n, err);
}

int pt_ctx_parts(const pt_ctx* c) { return c ? c->n() : PT_ERR_ARG; }

int pt_ctx_peer_copies(const pt_ctx* c) { return c ? (c->peer ? 1 : 0) : PT_ERR_ARG; }

void pt_ctx_destroy(pt_ctx* c)
{
    if (!c) return;
    // every part first: with distinct devices a part's queued halo pull or the gather may still read
    // another part's buffers over the peer link, and hipFree waits only for its own device's streams
    for (int k = 0; k < c->n(); k++) dev_sync(c->parts[k]);
    std::vector<pt_effect*> fx(c->effects.begin(), c->effects.end());
    for (auto* f : fx) pt_effect_destroy(f);
    std::vector<pt_texture*> tx(c->textures.begin(), c->textures.end());
    for (auto* t : tx) pt_texture_destroy(t);
    for (int k = 0; k < c->n(); k++) dev_sync(c->parts[k]);
    for (size_t k = 0; k < c->ev_draw.size(); k++) {
        hipSetDevice(dev_device(c->parts[k]));
        hipEventDestroy(c->ev_draw[k]);
        hipEventDestroy(c->ev_out[k]);
        if (k == 0 && c->ev_gather) hipEventDestroy(c->ev_gather);
    }
    for (auto* d : c->parts) dev_ctx_destroy(d);
    delete c;
}

const char* pt_last_error(pt_ctx* c) { return c ? c->err.c_str() : "no context"; }

int pt_sync(pt_ctx* c)
{
    if (!c) return PT_ERR_ARG;
    int first = PT_OK;
    for (int k = 0; k < c->n(); k++) {
        int rc = take(c, k, dev_sync(c->parts[k]));
        if (rc && !first) first = rc;
    }
    return first;
}

int pt_canvas_resize(pt_ctx* c, int w, int h)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_canvas_resize(c->parts[k], w, h))) return rc;
    c->cw = w; c->ch = h;
    return PT_OK;
}

int pt_canvas_wrap(pt_ctx* c, int w, int h, void* ptr)
{
    if (!c) return PT_ERR_ARG;
    // with several parts, the caller's memory receives the gathered frame (part 0's canvas); the
    // other parts keep canvases of their own of the same size
    for (int k = 1; k < c->n(); k++)
        if (int rc = take(c, k, dev_canvas_resize(c->parts[k], w, h))) return rc;
    if (int rc = take(c, 0, dev_canvas_wrap(c->parts[0], w, h, ptr))) return rc;
    c->cw = w; c->ch = h;
    return PT_OK;
}

int pt_set_output_partition(pt_ctx* c, int enable)
{
    if (!c) return PT_ERR_ARG;
    if (c->n() > 1) return fail(c, PT_ERR_ARG, "a multi-part context partitions its output itself");
    return take(c, 0, dev_set_output_partition(c->parts[0], enable));
}

int pt_set_row_partition(pt_ctx* c, int num_parts, int part)
{
    if (!c) return PT_ERR_ARG;
    if (c->n() > 1) return fail(c, PT_ERR_ARG, "a multi-part context partitions its rows itself");
    return take(c, 0, dev_set_row_partition(c->parts[0], num_parts, part));
}

int pt_set_stream(pt_ctx* c, void* stream)
{
    if (!c) return PT_ERR_ARG;
    if (c->n() > 1) return fail(c, PT_ERR_ARG, "pt_set_stream needs a one-part context");
    return take(c, 0, dev_set_stream(c->parts[0], stream));
}

pt_effect* pt_effect_create(pt_ctx* c, const char* src, const char* const* un, int nu, const char* const* sn, int ns,
                            int* err)
{
    if (err) *err = PT_OK;
    if (!c) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* fx = new pt_effect();
    fx->ctx = c;
    for (int k = 0; k < c->n(); k++) {
        int rc = PT_OK;
        DevFx* f = dev_effect_create(c->parts[k], src, un, nu, sn, ns, &rc);
        if (!f) {
            take(c, k, rc);
            for (auto* g : fx->sub) dev_effect_destroy(g);
            delete fx;
            if (err) *err = rc;
            return nullptr;
        }
        fx->sub.push_back(f);
    }
    fx->prog = dev_effect_program(fx->sub[0]);
    c->effects.insert(fx);
    return fx;
}

pt_effect* pt_effect_create_program(pt_ctx* c, int prog, const char* const* un, int nu, const char* const* sn, int ns,
                                    int* err)
{
    if (err) *err = PT_OK;
    if (!c) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* fx = new pt_effect();
    fx->ctx = c;
    for (int k = 0; k < c->n(); k++) {
        int rc = PT_OK;
        DevFx* f = dev_effect_create_program(c->parts[k], prog, un, nu, sn, ns, &rc);
        if (!f) {
            take(c, k, rc);
            for (auto* g : fx->sub) dev_effect_destroy(g);
            delete fx;
            if (err) *err = rc;
            return nullptr;
        }
        fx->sub.push_back(f);
    }
    fx->prog = prog;
    c->effects.insert(fx);
    return fx;
}

void pt_effect_destroy(pt_effect* fx)
{
    if (!fx) return;
    for (auto* f : fx->sub) dev_effect_destroy(f);
    fx->ctx->effects.erase(fx);
    delete fx;
}

int pt_effect_program(const pt_effect* fx) { return fx ? fx->prog : PT_PROG_UNKNOWN; }

int pt_set_float(pt_effect* fx, const char* name, const float* v, int n)
{
    if (!fx) return PT_ERR_ARG;
    for (size_t k = 0; k < fx->sub.size(); k++)
        if (int rc = take(fx->ctx, (int)k, dev_set_float(fx->sub[k], name, v, n))) return rc;
    return PT_OK;
}

int pt_set_int(pt_effect* fx, const char* name, int v)
{
    if (!fx) return PT_ERR_ARG;
    for (size_t k = 0; k < fx->sub.size(); k++)
        if (int rc = take(fx->ctx, (int)k, dev_set_int(fx->sub[k], name, v))) return rc;
    return PT_OK;
}

int pt_set_texture(pt_effect* fx, const char* name, pt_texture* t)
{
    if (!fx || !name) return PT_ERR_ARG;
    if (t && t->ctx != fx->ctx) return fail(fx->ctx, PT_ERR_ARG, "texture belongs to another context");
    for (size_t k = 0; k < fx->sub.size(); k++)
        if (int rc = take(fx->ctx, (int)k, dev_set_texture(fx->sub[k], name, t ? t->sub[k] : nullptr))) return rc;
    fx->bound[name] = t;
    return PT_OK;
}


pt_texture* pt_texture_create_rgba32f(pt_ctx* c, int w, int h, const float* data, int sampling, int invert_y, int* err)
{
    return make_tex(c, K_F32, w, h, err, [&](Dev* d, int* e) {
        return dev_texture_create_rgba32f(d, w, h, data, sampling, invert_y, e);
    });
}

pt_texture* pt_texture_create_rgba8(pt_ctx* c, int w, int h, const uint8_t* data, int sampling, int invert_y, int* err)
{
    return make_tex(c, K_U8, w, h, err, [&](Dev* d, int* e) {
        return dev_texture_create_rgba8(d, w, h, data, sampling, invert_y, e);
    });
}

pt_texture* pt_render_target_create(pt_ctx* c, int w, int h, int* err)
{
    return make_tex(c, K_RT, w, h, err, [&](Dev* d, int* e) { return dev_render_target_create(d, w, h, e); });
}

pt_texture* pt_render_target_wrap(pt_ctx* c, int w, int h, void* dptr, int* err)
{
    if (c && c->n() > 1) {
        fail(c, PT_ERR_ARG, "caller-owned render targets need a one-part context");
        if (err) *err = PT_ERR_ARG;
        return nullptr;
    }
    return make_tex(c, K_RT, w, h, err, [&](Dev* d, int* e) { return dev_render_target_wrap(d, w, h, dptr, e); });
}

int pt_render_target_resize(pt_texture* t, int w, int h)
{
    if (!t) return PT_ERR_ARG;
    if (t->ctx->n() > 1)   // neighbours' queued halo pulls / the gather may read this target's parts
        if (int rc = pt_sync(t->ctx)) return rc;
    for (size_t k = 0; k < t->sub.size(); k++)
        if (int rc = take(t->ctx, (int)k, dev_render_target_resize(t->sub[k], w, h))) return rc;
    t->w = w; t->h = h;
    return PT_OK;
}

int pt_texture_size(const pt_texture* t, int* w, int* h)
{
    if (!t) return PT_ERR_ARG;
    if (w) *w = t->w;
    if (h) *h = t->h;
    return PT_OK;
}

void pt_texture_destroy(pt_texture* t)
{
    if (!t) return;
    pt_ctx* c = t->ctx;
    if (c->n() > 1) pt_sync(c);   // as pt_render_target_resize: no queued peer read of it outlives it
    for (auto* fx : c->effects)
        for (auto& kv : fx->bound)
            if (kv.second == t) kv.second = nullptr;
    for (auto* s : t->sub) dev_texture_destroy(s);
    c->textures.erase(t);
    delete t;
}

int pt_render(pt_effect* fx, pt_texture* target)
{
    if (!fx) return PT_ERR_ARG;
    pt_ctx* c = fx->ctx;
    if (target && target->ctx != c) return fail(c, PT_ERR_ARG, "target belongs to another context");
    const int N = c->n();
    if (N == 1) return take(c, 0, dev_render(fx->sub[0], target ? target->sub[0] : nullptr));
    if (fx->prog == PT_PROG_SCREEN_OUTPUT) return render_output_parts(fx, target);
    const bool trace = is_trace(fx->prog);
    for (int k = 0; k < N; k++) {
        if (trace) {   // the neighbours' last output pulled halo rows from this part's targets
            GHIP(c, hipSetDevice(dev_device(c->parts[k])));
            const int lo = (k + N - 1) % N, hi = (k + 1) % N;
            if (int rc = wait(c, k, c->ev_out[lo], c->has_out[lo])) return rc;
            if (int rc = wait(c, k, c->ev_out[hi], c->has_out[hi])) return rc;
        }
        if (int rc = take(c, k, dev_render(fx->sub[k], target ? target->sub[k] : nullptr))) return rc;
        if (trace) {
            if (int rc = record(c, k, c->ev_draw[k])) return rc;
            c->has_draw[k] = true;
        }
    }
    return PT_OK;
}

int pt_read_pixels(pt_ctx* c, const pt_texture* t, void* dst, size_t bytes)
{
    if (!c || !dst) return PT_ERR_ARG;
    const int N = c->n();
    if (N == 1 || !t || t->kind != K_RT) {
        if (N > 1 && !t)   // the gathered canvas: every part's output first
            if (int rc = pt_sync(c)) return rc;
        return take(c, 0, dev_read_pixels(c->parts[0], t ? t->sub[0] : nullptr, dst, bytes));
    }
    // a render target is distributed by bands: each part's own bands
    const size_t need = (size_t)t->w * t->h * 16;
    if (bytes < need) return fail(c, PT_ERR_ARG, "destination too small");
    const int nb = (t->h + kBand - 1) / kBand;
    for (int k = 0; k < N; k++) {
        Dev* d = c->parts[k];
        if (int rc = take(c, k, dev_flush(d))) return rc;
        GHIP(c, copy_band_rows((char*)dst, (const char*)dev_texture_device_ptr(t->sub[k]), (size_t)t->w * 16, N, k,
                               bands_of(nb, N, k), 0, kBand, t->h, hipMemcpyDeviceToHost, dev_stream(d)));
    }
    return pt_sync(c);
}

int pt_write_pixels(pt_ctx* c, pt_texture* t, const void* src, size_t bytes)
{
    if (!c || !t) return PT_ERR_ARG;
    const int N = c->n();
    for (int k = 0; k < N; k++) {
        if (N > 1) {   // after the neighbours' last output, whose halo pulls read this part's texels
            GHIP(c, hipSetDevice(dev_device(c->parts[k])));
            const int lo = (k + N - 1) % N, hi = (k + 1) % N;
            if (int rc = wait(c, k, c->ev_out[lo], c->has_out[lo])) return rc;
            if (int rc = wait(c, k, c->ev_out[hi], c->has_out[hi])) return rc;
        }
        if (int rc = take(c, k, dev_write_pixels(c->parts[k], t->sub[k], src, bytes))) return rc;
    }
    return PT_OK;
}

int pt_set_backend(pt_ctx* c, int backend)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_set_backend(c->parts[k], backend))) return rc;
    return PT_OK;
}

int pt_set_bvh_layout(pt_ctx* c, int layout)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_set_bvh_layout(c->parts[k], layout))) return rc;
    return PT_OK;
}

int pt_bvh_layout_used(pt_ctx* c) { return c ? dev_bvh_layout_used(c->parts[0]) : PT_ERR_ARG; }

void* pt_texture_device_ptr(pt_texture* t) { return t ? dev_texture_device_ptr(t->sub[0]) : nullptr; }

int pt_last_render_ms(pt_ctx* c, int prog, float* ms)
{
    if (!c || !ms) return PT_ERR_ARG;
    // every part is asked (the first call turns each part's per-draw events on), then the first
    // failure is reported
    float best = 0.0f;
    int first = PT_OK;
    std::string msg;
    for (int k = 0; k < c->n(); k++) {
        float v = 0.0f;
        const int rc = take(c, k, dev_last_render_ms(c->parts[k], prog, &v));
        if (rc && !first) { first = rc; msg = c->err; }
        best = std::max(best, v);
    }
    if (first) { c->err = msg; return first; }
    *ms = best;
    return PT_OK;
}

int pt_timing_begin(pt_ctx* c)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_timing_begin(c->parts[k]))) return rc;
    return PT_OK;
}

int pt_timing_end(pt_ctx* c, int prog, double* total_ms, int* launches)
{
    if (!c || !total_ms || !launches) return PT_ERR_ARG;
    double best = 0.0;
    int n0 = 0;
    for (int k = 0; k < c->n(); k++) {
        double t = 0.0;
        int n = 0;
        if (int rc = take(c, k, dev_timing_end(c->parts[k], prog, &t, &n))) return rc;
        best = std::max(best, t);   // the slowest part bounds the frame
        if (k == 0) n0 = n;
    }
    *total_ms = best;
    *launches = n0;
    return PT_OK;
}

int pt_timing_latency(pt_ctx* c, int prog, float* ms, int cap, int* n)
{
    if (!c || !n || cap < 0 || (cap && !ms)) return PT_ERR_ARG;
    std::vector<float> part((size_t)cap);
    int n0 = 0;
    for (int k = 0; k < c->n(); k++) {
        int m = 0;
        if (int rc = take(c, k, dev_timing_latency(c->parts[k], prog, part.data(), cap, &m))) return rc;
        if (k == 0) { n0 = m; for (int i = 0; i < m; i++) ms[i] = part[i]; }
        else for (int i = 0; i < std::min(m, n0); i++) ms[i] = std::max(ms[i], part[i]);   // the slowest part's canvas
    }
    *n = n0;
    return PT_OK;
}

int pt_set_counting(pt_ctx* c, int enable)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_set_counting(c->parts[k], enable))) return rc;
    return PT_OK;
}

int pt_read_counters(pt_ctx* c, uint64_t out[PT_NUM_COUNTERS])
{
    if (!c || !out) return PT_ERR_ARG;
    std::memset(out, 0, PT_NUM_COUNTERS * sizeof(uint64_t));
    for (int k = 0; k < c->n(); k++) {
        uint64_t v[PT_NUM_COUNTERS];
        if (int rc = take(c, k, dev_read_counters(c->parts[k], v))) return rc;
        for (int i = 0; i < PT_NUM_COUNTERS; i++) out[i] += v[i];
    }
    return PT_OK;
}

int pt_reset_counters(pt_ctx* c)
{
    if (!c) return PT_ERR_ARG;
    for (int k = 0; k < c->n(); k++)
        if (int rc = take(c, k, dev_reset_counters(c->parts[k]))) return rc;
    return PT_OK;
}

int pt_queue_stats(pt_ctx* c, uint32_t out[16])
{
    if (!c || !out) return PT_ERR_ARG;
    std::memset(out, 0, 16 * sizeof(uint32_t));
    for (int k = 0; k < c->n(); k++) {
        uint32_t v[16];
        if (int rc = take(c, k, dev_queue_stats(c->parts[k], v))) return rc;
        for (int i = 0; i < 16; i++) out[i] += v[i];
    }
    return PT_OK;
}

int pt_math_probe(pt_ctx* c, int op, const float* x, const float* y, float* out, int n)
{
    if (!c) return PT_ERR_ARG;
    return take(c, 0, dev_math_probe(c->parts[0], op, x, y, out, n));
}

int pt_math_exhaustive(pt_ctx* c, int op, uint64_t* mismatches)
{
    if (!c) return PT_ERR_ARG;
    return take(c, 0, dev_math_exhaustive(c->parts[0], op, mismatches));
}

}  // extern "C"
