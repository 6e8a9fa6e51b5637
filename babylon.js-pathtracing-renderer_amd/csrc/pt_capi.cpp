// pt_capi.cpp — one device's part of a libpt context (pt_dev.h): contexts, effects, textures,
// render targets and draws on one HIP stream of one gfx950 device, mirroring the Babylon effect API
// the reference's setup scripts call. The exported C ABI (include/pt.h, pt_group.cpp) drives one
// such part per device of a context and fans every call out over them.
//
// What happens on dev_render(effect, target), per recognised program:
//   CORNELL / GLTF  -> uniforms resolved by name, SetupScene() evaluated once on the host with the
//                      same IEEE ops as the GLSL, one pt_trace launch over the 16-row bands this
//                      context owns (dev_set_row_partition);
//   SCREEN_COPY     -> pt_copy over the owned bands;
//   SCREEN_OUTPUT   -> pt_output into the canvas (RGBA8) or an RGBA32F target.
// Everything is enqueued on the context's stream; HIP events bracket every draw for timing.
#include "../../include/pt.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "pt_args.h"
#include "pt_dev.h"

extern "C" {
hipError_t pt_launch_exhaustive(int op, unsigned long long* bad, hipStream_t s);
hipError_t pt_launch_trace(int prog, int count, const pt::TraceArgs* a, int grid_x, int grid_y, hipStream_t s);
hipError_t pt_launch_order_build(unsigned ntiles, const unsigned* cost, unsigned* order, unsigned* split,
                                 unsigned split_cap, unsigned dominance, int near_buckets, hipStream_t s, int threads);
hipError_t pt_launch_copy(const pt::CopyArgs* a, int grid_x, int grid_y, hipStream_t s);
hipError_t pt_launch_blend(const pt::BlendArgs* a, int bands, hipStream_t s, int waves);
hipError_t pt_launch_cont_sort(const pt::SortArgs* a, size_t cap, hipStream_t s);
hipError_t pt_launch_cont(int prog, const pt::TraceArgs* a, int waves, hipStream_t s);
hipError_t pt_launch_output(const pt::OutputArgs* a, hipStream_t s, int waves);
hipError_t pt_launch_math_probe(int op, const float* x, const float* y, float* out, int n, hipStream_t s);
hipError_t pt_launch_persist(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x,
                             unsigned n_wave_tiles, unsigned per_wave, unsigned refill, hipStream_t s);
hipError_t pt_launch_finish(const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x, int bands, hipStream_t s);
hipError_t pt_launch_pairs_pass(int pass, const float4* aabb, long long texels, const float4* tri, long long tri_texels,
                                unsigned nrec, unsigned char* inner, unsigned char* leafref, unsigned* counts,
                                float* code, float4* inner_rec, float4* leaf_rec, unsigned leaf_base, unsigned* bad,
                                hipStream_t s);
hipError_t pt_launch_wavefront(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x, int bands,
                               int persist_blocks, hipStream_t s);
hipError_t pt_launch_trail_pass(int pass, const float4* aabb, long long texels, unsigned nrec, const unsigned char* inner,
                                unsigned* parent, unsigned* refs, unsigned* flag, const float4* rec, uint32_t root,
                                float4* top, hipStream_t s);
}

#ifdef PT_SECPROF
#define PT_SECPROF_BUILD true
#else
#define PT_SECPROF_BUILD false
#endif

namespace {

enum TexKind { TEX_F32 = 0, TEX_U8 = 1, TEX_RT = 2 };
constexpr int kProgSlots = 9;

struct Uniform {
    int n = 0;
    bool is_int = false;
    bool set = false;
    float f[16] = {};
    int i = 0;
};

}  // namespace

struct DevTex {
    Dev* ctx = nullptr;
    int kind = TEX_F32;
    int w = 0, h = 0;
    void* d = nullptr;
    size_t bytes = 0;
    int sampling = PT_SAMPLING_NEAREST;
    int invert_y = 0;
    bool external = false;   // caller-owned device memory (dev_render_target_wrap)
    unsigned long long gen = 0;   // bumped by every host write of the texels
    // child-pair BVH records derived from this texture and the triangle texture drawn with it
    // (pt_pairs_* passes), valid while both keep the generations they were built from
    void* pairs_mem = nullptr;
    const float4* pairs_inner = nullptr;
    const float4* pairs_leaf = nullptr;
    uint32_t pairs_root = 0;
    float pairs_root_box[6] = {};
    uint32_t pairs_bytes = 0;   // inner records, then leaf records from pairs_leaf on, then the jump table
    uint32_t pairs_top = 0;     // byte offset of the restart-trail jump table; 0: the tree is not walkable by the trail
    const DevTex* pairs_tri = nullptr;
    unsigned long long pairs_gen = ~0ull, pairs_tri_gen = ~0ull;
    bool pairs_ok = false;
};

struct DevFx {
    Dev* ctx = nullptr;
    int prog = PT_PROG_UNKNOWN;
    std::unordered_map<std::string, Uniform> uniforms;
    std::unordered_map<std::string, DevTex*> samplers;
};

struct Dev {
    int device = 0;
    hipStream_t stream = nullptr;      // the stream all work is enqueued on
    hipStream_t own_stream = nullptr;  // the context's own stream (dev_set_stream(NULL) restores it)
    std::string err;
    uchar4* canvas = nullptr;
    int cw = 0, ch = 0;
    unsigned* d_err = nullptr;
    unsigned long long* d_counters = nullptr;
    bool counting = false;
    int num_parts = 1, part = 0;
    bool output_partition = false;
    // screenCopy deferred to ride along with the next screenOutput of the same source (flushed as
    // its own kernel before anything else could observe the target: flush_copy)
    struct { bool on; DevTex* src; DevTex* dst; int num_parts, part; } pending_copy = {};
    bool canvas_external = false;     // dev_canvas_wrap: caller-owned canvas memory
    int backend = PT_BACKEND_MEGAKERNEL;
    int bvh_layout = PT_BVH_PAIRS;
    int bvh_used = -1;
    int cu_count = 256;
    pt::WfBufs wf = {};
    void* wf_mem = nullptr;
    size_t wf_pixels = 0, wf_slots = 0, wf_spill = 0;
    float2* mk_spill = nullptr;   // megakernel BVH stack spill slabs (one per side stream of the overlap depth)
    size_t mk_spill_lanes = 0;
    // Frame overlap (megakernel draws; PT_OVERLAP=0 turns it off). pt_trace never reads the history:
    // it writes radiance + the pre-history flag to its buffer set's rad, and pt_blend folds in the
    // history on the main stream. So draw k's path tracing runs on side stream ts[k % depth] and waits
    // only for the main stream's state when an earlier draw began (with depth 2: draw k - 1's mark, i.e.
    // draw k - 2's blend, its order build, the output that read rad / the order), never for draw k - 1's
    // kernel: consecutive frames' path tracing overlap, and the next frame's waves fill the launch tail
    // of this one. Per buffer set: the radiance buffer, the compaction records and the longest-first
    // cost / order / split (each set is its own longest-first pipeline, draw k ordered by the costs of
    // the set's previous draw); per side stream: the spill slab.
    bool overlap = true;
    // (PT_MOVING_SERIAL) frames drawn with uCameraIsMoving set run alone, one frame in flight: while the
    // camera moves, the user sees each frame as soon as it is done instead of two frames later
    bool moving_serial = true;
    // Depth (PT_OVERLAP_DEPTH, 2-6): side streams; draw k waits for the mark draw k - depth - lag + 1
    // recorded (depth 2, lag 0: the previous draw's), so up to `depth` frames' path tracing are in flight.
    static constexpr int kDepthMax = 6;
    int depth = 3;   // (r05q: three frames in flight, with compaction, won on every workload but the bunny)
    int depth_run = 3;            // the last megakernel draw's depth (<= depth: the auto trial may pick 2)
    bool depth_env = false;       // PT_OVERLAP_DEPTH given: the auto mode's default keeps it
    // Lag (PT_OVERLAP_LAG): buffer sets beyond the streams. Draw k's buffer set is k % (depth + lag)
    // (radiance, compaction records, longest-first cost / order: what the main stream's blend, output
    // and order build read) and its stream / spill slab k % depth (what only its own stream touches),
    // and it waits for the mark of draw k - depth - lag + 1: with lag > 0 a side stream runs its next
    // draw as soon as its previous one ends, not after that draw's blend and output on the main stream.
    // By default (lag -1) the lag is kLagSmall for draws that trace fewer than lag_pixels pixels and
    // 0 above: a small frame (a rank's bands of an N-GPU frame) fills the chip only with more frames
    // in flight, a 1080p one lost 3-4 % to the extra lag (r05an: 260-520 kpx +4-10 %, 1 Mpx and up -3 %).
    static constexpr int kLagMax = 6, kSetsMax = kDepthMax + kLagMax, kLagSmall = 2;
    int lag = -1;
    int lag_run = 0;              // the last megakernel draw's lag
    size_t lag_pixels = 800000;   // (PT_OVERLAP_LAG_PIXELS)
    hipStream_t ts[kDepthMax] = {};
    hipEvent_t ev_mark[kSetsMax] = {}, ev_traced[kDepthMax] = {};
    unsigned mk_seq = 0;          // megakernel draws so far (buffer set mk_seq % (depth + lag), stream mk_seq % depth)
    bool need_fresh = true;       // the next megakernel draw must wait for everything before it (a fresh mark)
    unsigned mark_floor = 0;      // no draw waits for a mark older than draw mark_floor's
    float4* rad_mem = nullptr;    // rad[sets()]: radiance + flag per pixel
    size_t rad_pixels = 0;
    // late-bounce compaction of the megakernel's mesh draws (pt_trace<P,false,true> -> pt_cont; PT_CONT:
    // 0 off, 1 on, 2 auto - the default): per buffer set 64-B path records, their pixels and a counter; the
    // bounce from which, and the live lanes at or below which, a wave hands its paths on; the refill batch
    // and pt_cont's one-wave workgroups
    int cont_mode = 2;
    void* cont_mem = nullptr;
    size_t cont_cap = 0;          // records per buffer set ...
    int cont_sets = 0;            // ... and buffer sets allocated
    unsigned cont_bounce = 2, cont_lanes = 48, cont_refill = 16, cont_waves = 2048;
    // pt_cont's waves for draws that trace at least cont_big_pixels (PT_CONT_WAVES_BIG, PT_CONT_BIG_PIXELS): beside
    // a 4K frame's path tracing fewer of them leave more wave slots to the next frames (dragon stand-in 4K
    // +3.2 to +3.9 %, helmet 4K +0.9 %, a rank's half of the 4K frame +1.5 %, 2560x1440 +1.1 %; 1080p keeps
    // 2048: 1536 there -1.8 %; profiles/r06bc_*, r06bd_*, r06be_*)
    unsigned cont_waves_big = 1024;
    size_t cont_big_pixels = 3000000;
    bool cont_waves_env = false;
    int cont_sort = 1;            // (PT_CONT_SORT) pt_cont takes its records ordered by a ray key (0: as stored)
    unsigned cont_grid_bits = 2, cont_key_mode = 0;   // (PT_CONT_SORT_GRID, PT_CONT_SORT_KEY) the key's cells, field order
    bool cont_grid_env = false;
    unsigned sort_chunk = 512;    // (PT_CONT_SORT_CHUNK) records per pt_cont_scatter workgroup (2048: ±0, 8192: -1 to -5 %)
    // auto mode: compaction pays on the heavy 4K frames (sky + dragon +19 %, dragon stand-in +10 %) and
    // costs elsewhere (bunny 4K -22 %, helmet -9 %, rank-sized frames -29 %: profiles/r05i_*), which
    // the draw's arguments do not tell apart. So the draws of one target / program / partition time it:
    // after kContSkip draws (the last two compacting, to warm it up on the side streams), blocks of
    // kContBlock draws with it on and off, kContMeasured draws inside each timed by events on the main
    // stream; at the trial's end the host waits for it once, and compaction stays on only if its faster
    // block took 2 % less time than the faster block without. Same bits either way.
    // The blocks without compaction also try two frames in flight instead of three (on, off, off at
    // depth 2 twice, off, on): the light frames that do not compact lost 2-5 % to the third frame
    // (r05q: bunny 5365 vs 5228 Mpaths/s, bunny16 -4.5 %), so the faster depth stays with "off".
    struct ContTune {
        const void* target; int prog, part, parts, w, h;
        int seen;                 // megakernel draws of this key so far
        bool decided, choice;
        int depth;                // the frames in flight the decision keeps
        float ms_on, ms_off, ms_off2;
    } tune = {};
    // the trial starts at the 33rd draw of a target: short runs (the driver's 5 + 20 frames) stay in the
    // default, longer ones settle on the measured best
    static constexpr int kContSkip = 32, kContBlock = 10, kContSettle = 3, kContMeasured = 5, kContBlocks = 6;
    size_t cont_auto_pixels = 2000000;   // (PT_CONT_AUTO_PIXELS) the default before the trial: on from 2 MP traced (1080p)
    hipEvent_t tune_ev[2 * kContBlocks] = {};
    int cont_last = 0;   // what the last megakernel draw did (cont_decide)
    unsigned cont_draws = 0;   // megakernel draws that launched pt_cont, since the context was created
    pt::WfBufs gb = {};           // persistent backend: per-pixel G-buffer + radiance
    void* gb_mem = nullptr;
    size_t gb_pixels = 0;
    unsigned persist_tiles = 4;   // 8x8 wave tiles per wave (PT_PERSIST_TILES)
    unsigned persist_refill = 16; // finished lanes that trigger a refill (PT_PERSIST_REFILL)
    // longest-first dispatch of the megakernel (PT_LPT=0 disables): cost[] / order[] of the last
    // path-tracing draw, reused when the next draw has the same grid, target and program
    bool lpt = true;
    bool lpt_zig = false;     // PT_LPT=2: the order taken from both ends alternately (TraceArgs::order_zig)
    bool zig_cont = true;     // (PT_LPT_ZIG_CONT) ... for compacting draws of up to lpt_flat_tiles tiles
    bool xcd_blocked = false; // (experiment, PT_XCD_BLOCKED) without an order: a contiguous eighth of the tiles per XCD
    unsigned prio_tiles = 0;   // longest-first: the first prio_tiles 16x16 tiles run at raised wave priority
    unsigned split_tiles = 32; // longest-first: at most this many of the slowest tiles shaded by 16-lane waves
                               // (pt_trace, pt_order_build; PT_SPLIT_TILES)
    int split_near = 3;             // ... those within this many cost buckets of the slowest (1/8 octave each; PT_SPLIT_NEAR)
    // (PT_LPT_FLAT, -1 = off) frames of more than 8192 tiles: the tiles more than this many buckets (1/8 octave
    // each) below the slowest are dealt as one bucket, in about row-major order, so that the tiles in flight lie
    // in one band of the frame (orderBuild). 6: dragon stand-in 4K +1.6-2.2 %, helmet 4K +8 %, sky + dragon 4K
    // +0.9 %, bunny 4K ±0 (profiles/r06g_frames_lpt_flat_4k.log); 1080p frames keep the whole order
    int lpt_flat = 6;
    unsigned lpt_flat_tiles = 8192;   // (PT_LPT_FLAT_TILES) ... for frames of more than this many tiles
    unsigned split_dominance = 8;   // ... when the slowest wave costs this many times the mean (PT_SPLIT_ALWAYS=1: 0)
    // the order build of the last megakernel draw, deferred to run as an extra block of the next
    // screenOutput pass (pt_output) instead of a kernel of its own; any other draw, stream switch or
    // query launches it alone first (flush_order). PT_FUSE_ORDER=0: always alone, after the draw.
    struct { bool on; unsigned n; const unsigned* cost; unsigned* order; unsigned* split; unsigned cap, dominance; int near; }
        pending_order = {};
    bool fuse_order = true;
    // (PT_MAIN_WAVES) pt_blend / pt_output as up to this many one-wave workgroups (0: 4-wave blocks):
    // beside overlapping path tracing a free wave slot comes one at a time, and a 4-wave workgroup waits
    // for four on one CU (r05bi: dragon stand-in 1080p +2 %, helmet +3 %; at 4K -4 %, so only up to 8192
    // tiles)
    int main_waves = 16384;
    size_t blend_1w_tiles = pt::kOrderHeld * 64u;   // (PT_BLEND_1W_TILES) pt_blend in one-wave form up to this many tiles
    size_t out_1w_tiles = pt::kOrderHeld * 64u;     // (PT_OUT_1W_TILES) pt_output likewise, when no order build rides along
    // (PT_ORDER_SIDE_TILES) frames of more tiles than this, drawn without lag, build their longest-first order
    // as a one-wave block on their own side stream after the traced event, instead of riding along with the
    // next screenOutput (which then needs no 4-wave block)
    size_t order_side_tiles = ~(size_t)0;
    unsigned* lpt_mem = nullptr;            // cost[kSetsMax][4 * cap] | order[kSetsMax][cap] | split[kSetsMax]
    size_t lpt_cap = 0;
    struct LptKey { bool valid; size_t n; const void* target; int prog, part, parts; };
    LptKey lpt_key[kSetsMax] = {};          // what cost[p] / order[p] were last written for
    unsigned* lpt_cost(int p) const { return lpt_mem + 4 * lpt_cap * p; }
    unsigned* lpt_order(int p) const { return lpt_mem + 4 * lpt_cap * kSetsMax + lpt_cap * p; }
    unsigned* lpt_split(int p) const { return lpt_mem + 5 * lpt_cap * kSetsMax + p; }
    int sets() const { return depth + (lag >= 0 ? lag : kLagSmall); }   // buffer sets allocated (rad, compaction records)
    // per-draw events for pt_last_render_ms: off until its first call (or PT_DRAW_EVENTS=1). Each
    // hipEventRecord costs ~5 us of stream time between two kernels on MI355X (r02h: two pairs per
    // frame were +19 us per frame, +1.7 % dragon stand-in, +3.8 % bunny)
    bool draw_events = false;
    hipEvent_t ev0[kProgSlots] = {}, ev1[kProgSlots] = {};
    bool ev_used[kProgSlots] = {};
    // timing window: per draw event pairs, reused across windows; every timing_every-th draw of a
    // program kind is bracketed (PT_TIMING_EVERY, default 1 = every draw)
    bool window = false, window_rec = false;
    int timing_every = 1;
    int window_seen[kProgSlots] = {};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    std::vector<std::pair<int, int>> window_draws;   // (program, pool index)
    int pending = -1;
    std::set<DevTex*> textures;
    std::set<DevFx*> effects;
};

namespace {

int fail(Dev* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

int hipfail(Dev* c, hipError_t e, const char* what)
{
    return fail(c, PT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(c, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hipfail(c, e_, #call); \
    } while (0)

bool contains(const char* s, const char* pat) { return s && std::strstr(s, pat) != nullptr; }

// Recognise the program from the GLSL registered in Effect.ShadersStore (the reference passes
// `BABYLON.Effect.ShadersStore["...FragmentShader"]` as `fragmentShader`).
int classify(const char* src)
{
    if (contains(src, "uniform sampler2D pathTracedImageBuffer")) return PT_PROG_SCREEN_COPY;
    if (contains(src, "uniform sampler2D accumulationBuffer")) return PT_PROG_SCREEN_OUTPUT;
    if (!contains(src, "pathtracing_default_main")) return PT_PROG_UNKNOWN;
    if (contains(src, "uniform sampler2D tHDRTexture")) return PT_PROG_HDRI;
    if (contains(src, "uniform mat4 uTorusInvMatrix")) return PT_PROG_QUADRIC;
    if (contains(src, "pathtracing_physical_sky_functions"))   // the sky scene, or its composite with the
        return contains(src, "uniform sampler2D tAABBTexture") ? PT_PROG_SKY_MESH : PT_PROG_SKY;   // glTF model block
    if (contains(src, "uniform sampler2D tAABBTexture")) return PT_PROG_GLTF;
    if (contains(src, "uniform int uRightSphereMatType")) return PT_PROG_CORNELL;
    return PT_PROG_UNKNOWN;
}

float uf(const DevFx* fx, const char* name, int k = 0)
{
    auto it = fx->uniforms.find(name);
    if (it == fx->uniforms.end() || !it->second.set) return 0.0f;   // GLSL uniforms default to 0
    const Uniform& u = it->second;
    if (u.is_int) return (float)u.i;
    return k < u.n ? u.f[k] : 0.0f;
}
int ui(const DevFx* fx, const char* name)
{
    auto it = fx->uniforms.find(name);
    if (it == fx->uniforms.end() || !it->second.set) return 0;
    const Uniform& u = it->second;
    return u.is_int ? u.i : (int)u.f[0];
}
void um4(const DevFx* fx, const char* name, ptg::m4& m)
{
    for (int k = 0; k < 16; k++) m.m[k] = uf(fx, name, k);
}
DevTex* sampler(const DevFx* fx, const char* name)
{
    auto it = fx->samplers.find(name);
    return it == fx->samplers.end() ? nullptr : it->second;
}

pt::Tex8 tex8(const DevTex* t)
{
    pt::Tex8 r{ nullptr, 0, 0 };
    if (t && t->kind == TEX_U8) { r.p = (const uchar4*)t->d; r.w = t->w; r.h = t->h; }
    return r;
}

ptg::f3 v3(float x, float y, float z) { return ptg::f3{ x, y, z }; }
pt::QuadArg quad(ptg::f3 n, ptg::f3 a, ptg::f3 b, ptg::f3 c, ptg::f3 d, ptg::f3 col, int type)
{
    pt::QuadArg q;
    q.normal = n; q.v0 = a; q.v1 = b; q.v2 = c; q.v3 = d; q.color = col; q.type = type;
    return q;
}
float hdist(ptg::f3 a, ptg::f3 b)
{
    float x = a.x - b.x, y = a.y - b.y, z = a.z - b.z;
    return std::sqrt(x * x + y * y + z * z);
}

// The uniform-only terms of Get_Sky_Color (js/PathTracingCommon.js:373-475) with the pinned
// sequences of pt_glsl.h, once per draw instead of once per sky sample
void sky_setup(const DevFx* fx, pt::SkyArgs& k)
{
    using namespace ptg;
    k.sun = v3(uf(fx, "uSunDirection", 0), uf(fx, "uSunDirection", 1), uf(fx, "uSunDirection", 2));
    const float cosSunUpAngle = dot(mk(0.0f, 1.0f, 0.0f), k.sun);
    const float z = gclamp(cosSunUpAngle, -1.0f, 1.0f);   // SunIntensity
    k.sunE = 200.0f * gmax(0.0f, 1.0f - gpow(2.71828182845904524f, -((1.6110731556870734f - gacos(z)) / 1.5f)));
    k.sunE19000 = k.sunE * 19000.0f;
    k.rayleigh = mk(5.804542996261093E-6f, 1.3562911419845635E-5f, 3.0265902468824876E-5f) * 2.0f;
    const float c = (0.2f * 0.5f) * 10E-18f;               // totalMie
    k.mie = (mk(1.8399918514433978E14f, 2.7798023919660528E14f, 4.0790479543861094E14f) * (0.434f * c)) * 0.03f;
    k.rm = k.rayleigh + k.mie;
    k.fade = gclamp(gpow(1.0f - cosSunUpAngle, 5.0f), 0.0f, 1.0f);
    const float sunfade = 1.0f - gclamp(1.0f - gexp((k.sun.y / 450000.0f)), 0.0f, 1.0f);
    k.retExp = 1.0f / (1.2f + (1.2f * sunfade));
}

// SetupScene() of js/BabylonPathTracing_FragmentShader.js:348-378 and
// js/GLTFModelPathTracing_FragmentShader.js:613-643, evaluated once per draw.
void setup_scene(const DevFx* fx, pt::TraceArgs& a)
{
    const float W = 50.0f;
    const float L = uf(fx, "uQuadLightRadius") * 0.2f;
    const ptg::f3 E = v3(1.0f * 10.0f, 1.0f * 10.0f, 1.0f * 10.0f);
    const ptg::f3 white = v3(1.0f, 1.0f, 1.0f);
    um4(fx, "uLeftSphereInvMatrix", a.sph[0].inv);
    um4(fx, "uRightSphereInvMatrix", a.sph[1].inv);
    a.sph[0].color = v3(1.0f, 1.0f, 0.0f);
    a.sph[0].type = pt::CLEARCOAT_DIFFUSE;
    a.sph[1].color = v3(1.0f, 1.0f, 1.0f);
    const bool gltf = fx->prog == PT_PROG_GLTF || fx->prog == PT_PROG_HDRI;
    a.sph[1].type = gltf ? pt::METAL : ui(fx, "uRightSphereMatType");
    pt::QuadArg q[6];
    q[0] = quad(v3(0, 0, 1), v3(-W, W, W), v3(W, W, W), v3(W, -W, W), v3(-W, -W, W), white, pt::DIFFUSE);
    q[1] = quad(v3(1, 0, 0), v3(-W, -W, W), v3(-W, -W, -W), v3(-W, W, -W), v3(-W, W, W), v3(0.7f, 0.05f, 0.05f), pt::DIFFUSE);
    q[2] = quad(v3(-1, 0, 0), v3(W, -W, -W), v3(W, -W, W), v3(W, W, W), v3(W, W, -W), v3(0.05f, 0.05f, 0.7f), pt::DIFFUSE);
    q[3] = quad(v3(0, -1, 0), v3(-W, W, -W), v3(W, W, -W), v3(W, W, W), v3(-W, W, W), white, pt::DIFFUSE);
    q[4] = quad(v3(0, 1, 0), v3(-W, -W, W), v3(W, -W, W), v3(W, -W, -W), v3(-W, -W, -W), white, pt::DIFFUSE);
    const float sel = uf(fx, "uQuadLightPlaneSelectionNumber");
    const float wm = W - 1.0f, wp = -W + 1.0f;
    std::memset(&q[5], 0, sizeof(q[5]));   // unselected: the GLSL global keeps its zero default
    if (sel == 1.0f) q[5] = quad(v3(-1, 0, 0), v3(wm, -L, L), v3(wm, L, L), v3(wm, L, -L), v3(wm, -L, -L), E, pt::LIGHT);
    else if (sel == 2.0f) q[5] = quad(v3(1, 0, 0), v3(wp, -L, -L), v3(wp, L, -L), v3(wp, L, L), v3(wp, -L, L), E, pt::LIGHT);
    else if (sel == 3.0f) q[5] = quad(v3(0, 0, 1), v3(-L, -L, wp), v3(L, -L, wp), v3(L, L, wp), v3(-L, L, wp), E, pt::LIGHT);
    else if (sel == 4.0f) q[5] = quad(v3(0, 0, -1), v3(-L, -L, wm), v3(-L, L, wm), v3(L, L, wm), v3(L, -L, wm), E, pt::LIGHT);
    else if (sel == 5.0f) q[5] = quad(v3(0, 1, 0), v3(-L, wp, -L), v3(-L, wp, L), v3(L, wp, L), v3(L, wp, -L), E, pt::LIGHT);
    else if (sel == 6.0f) q[5] = quad(v3(0, -1, 0), v3(-L, wm, -L), v3(L, wm, -L), v3(L, wm, L), v3(-L, wm, L), E, pt::LIGHT);
    auto sub = [](ptg::f3 x, ptg::f3 y) { return v3(x.x - y.x, x.y - y.y, x.z - y.z); };
    for (int i = 0; i < 6; i++) {
        a.qtri[2 * i] = pt::TriArg{ q[i].v0, sub(q[i].v1, q[i].v0), sub(q[i].v2, q[i].v0) };
        a.qtri[2 * i + 1] = pt::TriArg{ q[i].v0, sub(q[i].v2, q[i].v0), sub(q[i].v3, q[i].v0) };
        a.qnormal[i] = q[i].normal;
        a.qcolor[i] = q[i].color;
        a.qtype[i] = q[i].type;
    }
    a.light = q[5];
    a.light_r2 = hdist(q[5].v0, q[5].v1) * hdist(q[5].v0, q[5].v3);
    a.nquads = 6;
    const bool sky = fx->prog == PT_PROG_SKY || fx->prog == PT_PROG_SKY_MESH;
    if (sky || fx->prog == PT_PROG_HDRI) {
        // js/PhysicalSkyModel_FragmentShader.js:383-399, js/HDRIEnvironmentPathTracing_FragmentShader.js:529-542:
        // N_QUADS 4 = back, left, right walls and the floor (the Cornell ceiling and quad light are gone)
        const pt::QuadArg floor = q[4];
        a.qtri[6] = pt::TriArg{ floor.v0, sub(floor.v1, floor.v0), sub(floor.v2, floor.v0) };
        a.qtri[7] = pt::TriArg{ floor.v0, sub(floor.v2, floor.v0), sub(floor.v3, floor.v0) };
        a.qnormal[3] = floor.normal;
        a.qcolor[3] = floor.color;
        a.qtype[3] = floor.type;
        a.nquads = 4;
    }
    if (sky) sky_setup(fx, a.sky);
    if (fx->prog == PT_PROG_QUADRIC) {   // js/TransformedQuadricGeometry_FragmentShader.js:9-24
        static const char* const kShapes[12] = {
            "uSphereInvMatrix", "uCylinderInvMatrix", "uConeInvMatrix", "uParaboloidInvMatrix",
            "uHyperboloidInvMatrix", "uCapsuleInvMatrix", "uFlattenedRingInvMatrix", "uBoxInvMatrix",
            "uPyramidFrustumInvMatrix", "uDiskInvMatrix", "uRectangleInvMatrix", "uTorusInvMatrix" };
        for (int k = 0; k < 12; k++) um4(fx, kShapes[k], a.shape_inv[k]);
        a.shape_k = uf(fx, "uShapeK");
        a.shape_mat = ui(fx, "uAllShapesMatType");
    }
    if (fx->prog == PT_PROG_HDRI) {
        a.sky.sun = v3(uf(fx, "uSunDirection", 0), uf(fx, "uSunDirection", 1), uf(fx, "uSunDirection", 2));
        a.hdr_exposure = uf(fx, "uHDRExposure");
        const float p = uf(fx, "uSunPower");
        a.sun_weight = p * p * 0.0000001f;
        const DevTex* h = sampler(fx, "tHDRTexture");
        if (h && h->kind != TEX_U8) { a.hdr.p = (const float4*)h->d; a.hdr.w = h->w; a.hdr.h = h->h; }
    }
}

int bands_owned(const Dev* c, int height)
{
    int nb = (height + pt::kTile - 1) / pt::kTile;
    if (c->part >= nb) return 0;
    return (nb - c->part + c->num_parts - 1) / c->num_parts;
}

int begin_draw(Dev* c, int prog, hipStream_t s = nullptr)
{
    if (!s) s = c->stream;
    if (c->draw_events) {
        if (!c->ev0[prog]) {
            HIPCHK(c, hipEventCreate(&c->ev0[prog]));
            HIPCHK(c, hipEventCreate(&c->ev1[prog]));
        }
        HIPCHK(c, hipEventRecord(c->ev0[prog], s));
    }
    c->window_rec = c->window && c->window_seen[prog]++ % c->timing_every == 0;
    if (c->window_rec) {
        size_t k = c->window_draws.size();
        if (k == c->pool.size()) {
            hipEvent_t a, b;
            HIPCHK(c, hipEventCreate(&a));
            HIPCHK(c, hipEventCreate(&b));
            c->pool.emplace_back(a, b);
        }
        HIPCHK(c, hipEventRecord(c->pool[k].first, s));
        c->window_draws.emplace_back(prog, (int)k);
    }
    return PT_OK;
}
int end_draw(Dev* c, int prog, hipStream_t s = nullptr)
{
    if (!s) s = c->stream;
    if (c->draw_events) {
        HIPCHK(c, hipEventRecord(c->ev1[prog], s));
        c->ev_used[prog] = true;
    }
    if (c->window_rec)
        HIPCHK(c, hipEventRecord(c->pool[c->window_draws.back().second].second, s));
    return PT_OK;
}

// (re)allocate the wavefront buffers for `tiles` 16x16 tiles of a wq x hq quad-rounded frame and
// a persistent grid of `blocks` blocks: one slab, carved into the WfBufs arrays
int wf_reserve(Dev* c, int wq, int hq, int tiles, int blocks)
{
    const unsigned cap = (unsigned)((tiles + pt::kShards - 1) / pt::kShards) * pt::kBlock;
    const size_t slots = (size_t)cap * pt::kShards;
    const size_t pixels = (size_t)wq * hq;
    const size_t spill = (size_t)(pt::kStackLevels - pt::kStackLds) * blocks * pt::kBlock;
    if (c->wf_mem && slots <= c->wf_slots && pixels <= c->wf_pixels && spill <= c->wf_spill) {
        c->wf.shard_cap = cap; c->wf.wq = wq; c->wf.hq = hq;
        return PT_OK;
    }
    if (c->wf_mem) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->wf_mem)); c->wf_mem = nullptr; }
    const size_t f4s = slots * sizeof(float4), f4p = pixels * sizeof(float4);
    const size_t bytes = 4096 + 10 * f4s + 3 * f4p + slots * sizeof(unsigned) + spill * sizeof(float2) + 16 * 256;
    HIPCHK(c, hipMalloc(&c->wf_mem, bytes));
    char* m = (char*)c->wf_mem;
    auto take = [&](size_t n) { char* r = m; m += (n + 255) & ~(size_t)255; return r; };
    c->wf.cnt = (unsigned*)take(4096);
    c->wf.bcnt = c->wf.cnt + 8 * pt::kShards;
    for (int k = 0; k < 2; k++) {
        c->wf.qA[k] = (float4*)take(f4s); c->wf.qB[k] = (float4*)take(f4s);
        c->wf.qC[k] = (float4*)take(f4s); c->wf.qD[k] = (float4*)take(f4s);
    }
    c->wf.hit0 = (float4*)take(f4s); c->wf.hit1 = (float4*)take(f4s);
    c->wf.gb0 = (float4*)take(f4p); c->wf.gb1 = (float4*)take(f4p); c->wf.rad = (float4*)take(f4p);
    c->wf.bvhq = (unsigned*)take(slots * sizeof(unsigned));
    c->wf.spill = (float2*)take(spill * sizeof(float2));
    c->wf_slots = slots; c->wf_pixels = pixels; c->wf_spill = spill;
    c->wf.shard_cap = cap; c->wf.wq = wq; c->wf.hq = hq;
    return PT_OK;
}

constexpr size_t kSpillPerLane = pt::kStackLevels - pt::kStackLdsMin + 4;   // float2 per lane of one slab

// the megakernel's spill slabs, one per side stream (overlapping draws must not share one): stack
// levels kStackLdsMin..27, then up to 8 floats per lane for the G-buffer fields kept out of LDS
// (pt_trace.h); slab p starts at spill_slab(c, p)
int spill_reserve(Dev* c, size_t lanes)
{
    if (lanes <= c->mk_spill_lanes) return PT_OK;
    if (c->mk_spill) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->mk_spill)); c->mk_spill = nullptr; }
    c->mk_spill_lanes = 0;
    HIPCHK(c, hipMalloc(&c->mk_spill, (size_t)c->depth * lanes * kSpillPerLane * sizeof(float2)));
    c->mk_spill_lanes = lanes;
    c->need_fresh = true;   // new memory: the next draw waits for everything before it
    return PT_OK;
}
float2* spill_slab(Dev* c, int p) { return c->mk_spill + (size_t)p * c->mk_spill_lanes * kSpillPerLane; }

// rad[sets()] (pt_trace -> pt_blend) for a frame of `pixels`
int rad_reserve(Dev* c, size_t pixels)
{
    if (pixels <= c->rad_pixels) return PT_OK;
    if (c->rad_mem) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->rad_mem)); c->rad_mem = nullptr; }
    c->rad_pixels = 0;
    HIPCHK(c, hipMalloc(&c->rad_mem, (size_t)c->sets() * pixels * sizeof(float4)));
    c->rad_pixels = pixels;
    c->need_fresh = true;
    return PT_OK;
}

// the overlap lag of a draw that traces `traced` pixels (Dev::lag)
int draw_lag(const Dev* c, size_t traced) { return c->lag >= 0 ? c->lag : traced < c->lag_pixels ? Dev::kLagSmall : 0; }

// the pixels a draw of `target` traces: the owned 16-row bands of the partition (a bound on its records)
size_t traced_pixels(const Dev* c, const DevTex* target)
{
    const int nb = (target->h + pt::kTile - 1) / pt::kTile;
    const int own = c->part < nb ? (nb - c->part + c->num_parts - 1) / c->num_parts : 0;
    return std::min((size_t)target->w * target->h, (size_t)own * pt::kTile * target->w);
}

// pt_cont's records for draws that trace up to `paths` pixels (a record per traced pixel at most), in `sets`
// buffer sets: per set records [cap x 64 B] | pixels [cap x 4 B] | counter; the counters start at zero here,
// afterwards each draw's pt_blend zeroes its own. (Sized by the partition's pixels and the sets its draws
// cycle through, not the whole target times every set: a 4K frame's records are 0.53 GB per set.)
// bytes of one buffer set for `paths` records: records [paths x 64 B] | pixels [x 4 B] | (PT_CONT_SORT: order
// [x 4 B] | ranks [x 4 B] | keys [x 2 B] | the keys' totals) | counter
size_t cont_bytes(const Dev* c, size_t paths)
{
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    size_t per = paths * 64 + al(paths * 4) + 256;
    if (c->cont_sort) per += 2 * al(paths * 4) + al(paths * 2) + pt::kSortBins * 4;
    return per;
}
int cont_reserve(Dev* c, size_t paths, int sets)
{
    if (paths <= c->cont_cap && sets <= c->cont_sets) return PT_OK;
    paths = std::max(paths, c->cont_cap);
    sets = std::max(sets, c->cont_sets);
    if (c->cont_mem) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->cont_mem)); c->cont_mem = nullptr; }
    c->cont_cap = 0;
    c->cont_sets = 0;
    const size_t per = cont_bytes(c, paths);
    HIPCHK(c, hipMalloc(&c->cont_mem, (size_t)sets * per));
    // on the main stream (hipMemset would go to the null stream, which the non-blocking side streams do
    // not wait for: the next draw's atomics raced with it); the next draw's path tracing waits for a mark
    // recorded after it
    HIPCHK(c, hipMemsetAsync(c->cont_mem, 0, (size_t)sets * per, c->stream));
    c->cont_cap = paths;
    c->cont_sets = sets;
    c->need_fresh = true;
    return PT_OK;
}
void cont_args(Dev* c, int p, pt::TraceArgs& a)
{
    const size_t per = cont_bytes(c, c->cont_cap);
    char* m = (char*)c->cont_mem + (size_t)p * per;
    a.cont_rec = (float4*)m;
    a.cont_aux = (unsigned*)(m + c->cont_cap * 64);
    a.cont_count = (unsigned*)(m + per - 256);
    a.cont_perm = nullptr;
    a.cont_rank = nullptr;
    a.cont_key = nullptr;
    a.cont_bins = nullptr;
    a.cont_bounce = std::max(2u, c->cont_bounce);   // the G-buffer's normal / colour / id are final from bounce 2
    a.cont_lanes = c->cont_lanes;
    a.cont_refill = c->cont_refill;
}

// auto mode of late-bounce compaction (Dev::ContTune): whether this draw compacts
int cont_decide_(Dev* c, const DevTex* target, int prog, bool eligible, bool* on, int* depth)
{
    *on = false;
    *depth = c->depth;
    if (!eligible || c->cont_mode == 0) return PT_OK;
    // the records first, so that no trial block pays for their allocation (for every set the draws of this
    // target cycle through: the depth, at most c->depth, plus the lag)
    const size_t traced_approx = (size_t)target->w * target->h / (size_t)std::max(1, c->num_parts);   // (as render_trace's)
    if (int rc = cont_reserve(c, traced_pixels(c, target), c->depth + draw_lag(c, traced_approx))) return rc;
    if (c->cont_mode == 1) { *on = true; return PT_OK; }
    auto& t = c->tune;
    if (t.target != target || t.prog != prog || t.part != c->part || t.parts != c->num_parts || t.w != target->w ||
        t.h != target->h)
        t = Dev::ContTune{ target, prog, c->part, c->num_parts, target->w, target->h, 0, false, false, c->depth,
                           0.0f, 0.0f, 0.0f };
    const int i = t.seen++ - Dev::kContSkip;
    if (t.decided) { *on = t.choice; *depth = t.depth; return PT_OK; }
    // before the trial, the default: on for frames of at least cont_auto_pixels (with three frames in
    // flight it won on every frame of 2 MP and more but the light bunny, and lost on the rank-sized one,
    // profiles/r05q_frames_depth_x_compaction.txt); the two draws before the trial compact, one per side
    // stream of the last two buffer sets, whatever the default: the first launch of a variant that needs
    // more scratch than any before it waits for the device to drain while the runtime grows its scratch
    // (r05k: the first trial block then took 2-8x the others)
    if (i < 0) {
        // (the pixels this partition traces: a rank's bands of an N-GPU frame are a small frame -
        // r05ao: 0.5-1 Mpx frames lost 33-41 % to compaction)
        const size_t traced = (size_t)target->w * target->h / (size_t)std::max(1, c->num_parts);
        *on = traced >= c->cont_auto_pixels || i >= -2;
        // without compaction, frames of lag_pixels and more keep two frames in flight (r05aw: the
        // 4K frame's eighth at N = 8 +5.6 %; r05y: StanfordBunny 1080p +3.5 %), smaller ones three
        // and the lag (a 1920x136 frame: two lost a third, r05aa)
        if (!*on && !c->depth_env && traced >= c->lag_pixels) *depth = std::min(2, c->depth);
        return PT_OK;
    }
    constexpr int B = Dev::kContBlock, S = Dev::kContSettle, M = Dev::kContMeasured, trial = Dev::kContBlocks * B;
    // each block times draws S .. S + M - 1 of its own: an event on the main stream (the work before the
    // draw: the previous draw's blend, which waited for its path tracing) at the block's offsets S and
    // S + M. With up to `depth` frames in flight, S draws settle the switch (buffer sets whose
    // longest-first order came from the other mode's costs) and the block's last B - S - M draws keep the
    // next block's frames out of the timed ones.
    const int b = i / B, o = i % B;
    if (i < trial && (o == S || o == S + M)) {
        hipEvent_t& e = c->tune_ev[2 * b + (o == S ? 0 : 1)];
        if (!e) HIPCHK(c, hipEventCreate(&e));
        HIPCHK(c, hipEventRecord(e, c->stream));
    }
    if (i < trial) {
        *on = b == 0 || b == Dev::kContBlocks - 1;   // on, off, off at depth 2 (twice), off, on
        if (b == 2 || b == 3) *depth = std::min(2, c->depth);
        return PT_OK;
    }
    // the trial's end: the host waits for it once (the draws it has already queued ran without), so that
    // every later draw of this target takes the decision; the faster block of each mode decides (one
    // stray block cannot)
    HIPCHK(c, hipEventSynchronize(c->tune_ev[2 * Dev::kContBlocks - 1]));
    t.ms_on = t.ms_off = t.ms_off2 = 1e30f;
    for (int k = 0; k < Dev::kContBlocks; k++) {
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->tune_ev[2 * k], c->tune_ev[2 * k + 1]));
        float& m = k == 0 || k == Dev::kContBlocks - 1 ? t.ms_on : k == 2 || k == 3 ? t.ms_off2 : t.ms_off;
        m = std::min(m, ms);
    }
    t.decided = true;
    const bool two = t.ms_off2 < t.ms_off;
    t.choice = t.ms_on < 0.98f * std::min(t.ms_off, t.ms_off2);
    t.depth = t.choice || !two ? c->depth : std::min(2, c->depth);
    *on = t.choice;
    *depth = t.depth;
    return PT_OK;
}

int cont_decide(Dev* c, const DevTex* target, int prog, bool eligible, bool* on, int* depth)
{
    int rc = cont_decide_(c, target, prog, eligible, on, depth);
    // what the draw did, for pt_queue_stats: 0 off, 1 auto decided off, 2 auto decided on, 3 forced on,
    // 4 auto trial
    const bool tried = c->cont_mode == 2 && eligible;
    c->cont_last = c->cont_mode == 1 && *on ? 3 : !tried ? 0 : c->tune.decided ? (c->tune.choice ? 2 : 1)
                 : c->tune.seen > Dev::kContSkip ? 4 : (*on ? 5 : 6);
    return rc;
}

// the side streams and events of frame overlap (created at the first overlapped draw)
int overlap_init(Dev* c)
{
    if (c->ts[0]) return PT_OK;
    // (experiment, PT_SIDE_STREAMS=1) CU-masked side streams over every CU, each on a hardware queue of
    // its own: with PT_OVERLAP_DEPTH=6, rank-sized dragon frames +30 %, the bunny's bimodal, 1080p -6 %
    // (profiles/r05ad_*, r05an_*); stream priorities and CUs kept free for the main stream lost
    const char* sk = std::getenv("PT_SIDE_STREAMS");
    const int kind = sk ? std::atoi(sk) : 0;
    for (int p = 0; p < c->sets(); p++) HIPCHK(c, hipEventCreateWithFlags(&c->ev_mark[p], hipEventDisableTiming));
    for (int p = 0; p < c->depth; p++) {
        if (kind == 1) {
            uint32_t mask[16];
            for (auto& m : mask) m = 0xffffffffu;
            HIPCHK(c, hipExtStreamCreateWithCUMask(&c->ts[p], 16, mask));
        } else {
            HIPCHK(c, hipStreamCreateWithFlags(&c->ts[p], hipStreamNonBlocking));
        }
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_traced[p], hipEventDisableTiming));
    }
    return PT_OK;
}

int gb_reserve(Dev* c, int wq, int hq)
{
    const size_t pixels = (size_t)wq * hq;
    if (pixels > c->gb_pixels) {
        if (c->gb_mem) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->gb_mem)); c->gb_mem = nullptr; }
        c->gb_pixels = 0;
        const size_t f4p = ((pixels * sizeof(float4)) + 255) & ~(size_t)255;
        HIPCHK(c, hipMalloc(&c->gb_mem, 3 * f4p));
        c->gb.gb0 = (float4*)c->gb_mem;
        c->gb.gb1 = (float4*)((char*)c->gb_mem + f4p);
        c->gb.rad = (float4*)((char*)c->gb_mem + 2 * f4p);
        c->gb_pixels = pixels;
    }
    c->gb.wq = wq; c->gb.hq = hq;
    return PT_OK;
}

// The child-pair records of a BVH texture (with the triangle texture drawn alongside), rebuilt
// when either texture's texels changed since the last build. Only for data textures (their
// texels change only through this API) of at most 2^24 texels (node ids and ranks exact in
// float). Returns false when the reference walk must be used. One host round trip per build.
#ifdef PT_SECPROF
static unsigned long long* g_wave_log = nullptr;
static size_t g_wave_log_n = 0;
extern "C" __attribute__((visibility("default"))) size_t pt_debug_wave_log(unsigned long long* out, size_t n)
{
    hipDeviceSynchronize();
    n = n < g_wave_log_n ? n : g_wave_log_n;
    if (g_wave_log && n) hipMemcpy(out, g_wave_log, n * 8 * pt::kWaveLogSlots, hipMemcpyDeviceToHost);
    return n;
}
// the child-pair walk's load coherence since the last call (WalkStat, pt_device.h): 8 bounces x 5
// counters (wave iterations, record loads, uniform loads, loading lanes, lanes at the first lane's record)
static unsigned long long* g_walk_stat = nullptr;
extern "C" __attribute__((visibility("default"))) int pt_debug_walk_stats(unsigned long long out[40])
{
    hipDeviceSynchronize();
    if (!g_walk_stat) return -1;
    hipMemcpy(out, g_walk_stat, 40 * 8, hipMemcpyDeviceToHost);
    hipMemset(g_walk_stat, 0, 40 * 8);
    return 0;
}
#endif
bool ensure_pairs(Dev* c, DevTex* t, const DevTex* tri, int* rc)
{
    *rc = PT_OK;
    const long long texels = (long long)t->w * t->h;
    if (c->bvh_layout == PT_BVH_REFERENCE || t->kind != TEX_F32 || tri->kind != TEX_F32 || texels > (1ll << 24)) return false;
    if (t->pairs_gen == t->gen && t->pairs_tri == tri && t->pairs_tri_gen == tri->gen) return t->pairs_ok;
    if (t->pairs_mem) { hipStreamSynchronize(c->stream); hipFree(t->pairs_mem); t->pairs_mem = nullptr; }
    t->pairs_ok = false;
    t->pairs_top = 0;
    t->pairs_gen = t->gen; t->pairs_tri = tri; t->pairs_tri_gen = tri->gen;
    const unsigned nrec = (unsigned)((texels + 1) / 2);
    const unsigned nblk = (nrec + 1023) / 1024;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    unsigned char *inner = nullptr, *leafref = nullptr, *scratch = nullptr;
    unsigned* counts = nullptr;
    float* code = nullptr;
    unsigned *parent = nullptr, *refs = nullptr;   // restart-trail checks (pt_pairs_links / _depth)
    const size_t u4 = al(nrec * sizeof(unsigned));
    hipError_t e = hipMalloc(&scratch, 2 * al(nrec) + al(2 * nblk * sizeof(unsigned)) + al(nrec * sizeof(float)) + 2 * u4);
    std::vector<unsigned> h(2 * nblk);
    unsigned bad = 0, notrail = 0;
    if (e == hipSuccess) {
        inner = scratch; leafref = scratch + al(nrec);
        counts = (unsigned*)(scratch + 2 * al(nrec));
        code = (float*)((char*)counts + al(2 * nblk * sizeof(unsigned)));
        parent = (unsigned*)((char*)code + al(nrec * sizeof(float)));
        refs = (unsigned*)((char*)parent + u4);
        e = hipMemsetAsync(leafref, 0, nrec, c->stream);
    }
    if (e == hipSuccess) e = hipMemsetAsync(refs, 0, nrec * sizeof(unsigned), c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_err + 1, 0, 2 * sizeof(unsigned), c->stream);
    const float4* aabb = (const float4*)t->d;
    const float4* trid = (const float4*)tri->d;
    const long long ttex = (long long)tri->w * tri->h;
    unsigned leaf_base = 0;   // byte offset of the leaf records in the one record array
    auto pass = [&](int k, float4* ir, float4* lr) {
        return pt_launch_pairs_pass(k, aabb, texels, trid, ttex, nrec, inner, leafref, counts, code, ir, lr, leaf_base,
                                    c->d_err + 1, c->stream);
    };
    if (e == hipSuccess) e = pass(1, nullptr, nullptr);
    if (e == hipSuccess) e = pass(2, nullptr, nullptr);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), counts, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, c->d_err + 1, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    size_t n_inner = 0, n_leaf = 0;
    if (e == hipSuccess && !bad) {
        for (unsigned b = 0; b < nblk; b++) {   // exclusive scan of the per-block counts
            unsigned ci = h[2 * b], cl = h[2 * b + 1];
            h[2 * b] = (unsigned)n_inner; h[2 * b + 1] = (unsigned)n_leaf;
            n_inner += ci; n_leaf += cl;
        }
        leaf_base = (unsigned)al(n_inner * 64);
        const size_t top_base = leaf_base + al(n_leaf * 48);
        const size_t rec_bytes = top_base + (size_t)pt::kTopEntries * 64;
        e = hipMalloc(&t->pairs_mem, rec_bytes + 256);
        if (e == hipSuccess) {
            t->pairs_inner = (const float4*)t->pairs_mem;
            t->pairs_leaf = (const float4*)((char*)t->pairs_mem + leaf_base);
            e = hipMemcpyAsync(counts, h.data(), h.size() * sizeof(unsigned), hipMemcpyHostToDevice, c->stream);
        }
        if (e == hipSuccess) e = pass(3, nullptr, nullptr);
        if (e == hipSuccess) e = pass(4, (float4*)t->pairs_inner, (float4*)t->pairs_leaf);
        auto tpass = [&](int k, uint32_t root) {
            return pt_launch_trail_pass(k, aabb, texels, nrec, inner, parent, refs, c->d_err + 2, t->pairs_inner, root,
                                        (float4*)((char*)t->pairs_mem + top_base), c->stream);
        };
        if (e == hipSuccess) e = tpass(1, 0);
        if (e == hipSuccess) e = tpass(2, 0);
        float root = 0.0f, node0[8] = {};
        if (e == hipSuccess) e = hipMemcpyAsync(&root, code, sizeof(float), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(node0, aabb, sizeof(node0), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(&notrail, c->d_err + 2, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        t->pairs_root = pt::pairCode(root, leaf_base);
        const float box6[6] = { node0[1], node0[2], node0[3], node0[5], node0[6], node0[7] };
        std::memcpy(t->pairs_root_box, box6, sizeof(box6));
        t->pairs_bytes = (uint32_t)rec_bytes;
        // the restart trail's jump table, for trees it can walk (one parent per node, depth <= 28)
        if (e == hipSuccess && !notrail) {
            e = tpass(3, t->pairs_root);
            if (e == hipSuccess) t->pairs_top = (uint32_t)top_base;
        }
    }
    if (scratch) { hipStreamSynchronize(c->stream); hipFree(scratch); }
    if (e != hipSuccess) { *rc = hipfail(c, e, "BVH child-pair build"); return false; }
    t->pairs_ok = !bad;
    return t->pairs_ok;
}

// launch a deferred order build now, as its own kernel
int flush_order(Dev* c)
{
    if (!c->pending_order.on) return PT_OK;
    c->pending_order.on = false;
    const auto& po = c->pending_order;
    HIPCHK(c, pt_launch_order_build(po.n, po.cost, po.order, po.split, po.cap, po.dominance, po.near, c->stream,
                                    1024));
    return PT_OK;
}

int render_trace(DevFx* fx, DevTex* target)
{
    Dev* c = fx->ctx;
    if (int rc = flush_order(c)) return rc;   // this draw's order (before lpt_mem could be reallocated)
    if (!target || target->kind != TEX_RT) return fail(c, PT_ERR_ARG, "path tracing draws need a render target");
    DevTex* prev = sampler(fx, "previousBuffer");
    DevTex* bn = sampler(fx, "blueNoiseTexture");
    if (!prev || prev->kind == TEX_U8 || prev->w != target->w || prev->h != target->h)
        return fail(c, PT_ERR_STATE, "previousBuffer must be an RGBA32F texture of the target's size");
    if (!bn || bn->kind != TEX_U8) return fail(c, PT_ERR_STATE, "blueNoiseTexture must be bound (RGBA8)");
    pt::TraceArgs a;
    std::memset(&a, 0, sizeof(a));
    a.width = target->w;
    a.height = target->h;
    a.num_parts = c->num_parts;
    a.part = c->part;
    a.res[0] = uf(fx, "uResolution", 0); a.res[1] = uf(fx, "uResolution", 1);
    a.rnd[0] = uf(fx, "uRandomVec2", 0); a.rnd[1] = uf(fx, "uRandomVec2", 1);
    a.ulen = uf(fx, "uULen"); a.vlen = uf(fx, "uVLen");
    a.frame = uf(fx, "uFrameCounter");
    a.eps = uf(fx, "uEPS_intersect");
    a.aperture = uf(fx, "uApertureSize");
    a.focus = uf(fx, "uFocusDistance");
    a.moving = ui(fx, "uCameraIsMoving");
    um4(fx, "uCameraMatrix", a.cam);
    setup_scene(fx, a);
    a.prev = (const float4*)prev->d;
    a.out = (float4*)target->d;
    a.bluenoise = tex8(bn);
    const bool mesh = fx->prog == PT_PROG_GLTF || fx->prog == PT_PROG_HDRI || fx->prog == PT_PROG_SKY_MESH;
    if (mesh) {
        DevTex* bvh = sampler(fx, "tAABBTexture");
        DevTex* tri = sampler(fx, "tTriangleTexture");
        if (!bvh || !tri || bvh->kind != TEX_F32 || tri->kind != TEX_F32)
            return fail(c, PT_ERR_STATE, "tAABBTexture / tTriangleTexture must be bound RGBA32F data textures");
        um4(fx, "uGLTF_Model_InvMatrix", a.model);
        a.model_mat = ui(fx, "uModelMaterialType");
        a.uses_albedo = ui(fx, "uModelUsesAlbedoTexture");
        a.uses_bump = ui(fx, "uModelUsesBumpTexture");
        a.uses_metal = ui(fx, "uModelUsesMetallicTexture");
        a.uses_emissive = ui(fx, "uModelUsesEmissiveTexture");
        a.aabb = (const float4*)bvh->d;
        a.aabb_texels = (long long)bvh->w * bvh->h;
        a.tri = (const float4*)tri->d;
        a.tri_texels = (long long)tri->w * tri->h;
        int prc = PT_OK;
        if (ensure_pairs(c, bvh, tri, &prc)) {
            a.bvh_pairs = bvh->pairs_inner;
            a.bvh_root_code = bvh->pairs_root;
            std::memcpy(a.bvh_root_box, bvh->pairs_root_box, sizeof(a.bvh_root_box));
            a.bvh_pairs_bytes = bvh->pairs_bytes;
            a.bvh_top_base = c->bvh_layout == PT_BVH_TRAIL ? bvh->pairs_top : 0u;
        }
        if (prc) return prc;
        a.bvh_walk = a.bvh_top_base ? pt::WALK_TRAIL : a.bvh_pairs ? pt::WALK_PAIRS : pt::WALK_REF;
        c->bvh_used = a.bvh_top_base ? PT_BVH_TRAIL : a.bvh_pairs ? PT_BVH_PAIRS : PT_BVH_REFERENCE;
        a.albedo = tex8(sampler(fx, "tAlbedoTexture"));
        a.bump = tex8(sampler(fx, "tBumpTexture"));
        a.metal = tex8(sampler(fx, "tMetallicTexture"));
        a.emissive = tex8(sampler(fx, "tEmissiveTexture"));
    }
    a.counters = c->d_counters;
    a.err = c->d_err;
#ifdef PT_SECPROF
    {   // experiment builds: the wave timeline of the last megakernel draw (pt_debug_wave_log)
        static size_t cap = 0;
        const size_t tx = (size_t)((target->w + pt::kTile - 1) / pt::kTile);   // + split tiles' padding rows
        const size_t need = (tx * bands_owned(c, target->h) * 4 + (4 * pt::kSplitParts - 4) * (size_t)c->split_tiles + 4 * tx) * pt::kWaveLogSlots;
        if (cap < need) { if (g_wave_log) hipFree(g_wave_log); hipMalloc(&g_wave_log, need * 8); cap = need; }
        hipMemsetAsync(g_wave_log, 0, need * 8, c->stream);   // padding workgroups leave zero rows
        g_wave_log_n = need / pt::kWaveLogSlots;
        a.wave_log = g_wave_log;
        // the walk statistics' global atomics (every wave, every bounce) slow the launch ~4x and skew
        // the timeline by XCD: only when asked for (tools/walkstat.py sets PT_WALKSTAT=1)
        static const bool walkstat = std::getenv("PT_WALKSTAT") && std::atoi(std::getenv("PT_WALKSTAT")) != 0;
        if (walkstat && !g_walk_stat && hipMalloc(&g_walk_stat, 40 * 8) == hipSuccess) hipMemset(g_walk_stat, 0, 40 * 8);
        a.walk_stat = walkstat ? g_walk_stat : nullptr;
    }
#endif
    int gx = (target->w + pt::kTile - 1) / pt::kTile;
    int gy = bands_owned(c, target->h);
    const int persist = ((c->cu_count * 4 + pt::kShards - 1) / pt::kShards) * pt::kShards;
    if (c->backend == PT_BACKEND_WAVEFRONT) {
        // the quad-rounded frame is what gets shaded (helpers at odd edges included)
        int rc = wf_reserve(c, (target->w + 1) & ~1, (target->h + 1) & ~1, gx * gy, persist);
        if (rc) return rc;
    }
    const unsigned n_wave_tiles = (unsigned)gx * gy * 4u;
    if (c->backend == PT_BACKEND_PERSISTENT) {
        int rc = gb_reserve(c, (target->w + 1) & ~1, (target->h + 1) & ~1);
        if (rc) return rc;
        const unsigned waves = (n_wave_tiles + c->persist_tiles - 1) / c->persist_tiles;
        const size_t lanes = (size_t)((waves + 3) / 4) * pt::kBlock;
        if (lanes * kSpillPerLane > 0xffffffffull)   // 32-bit slab index
            return fail(c, PT_ERR_ARG, "render target too large for the BVH stack slab");
        if (mesh && (rc = spill_reserve(c, lanes))) return rc;
        a.spill = c->mk_spill;
        a.spill_stride = lanes;
    }
    if (c->backend != PT_BACKEND_MEGAKERNEL || gy <= 0) {
        // the wavefront / persistent schedules: on the main stream, their finish pass accumulating;
        // the next megakernel draw waits for all of it (they share the spill slab)
        if (c->backend != PT_BACKEND_MEGAKERNEL) c->need_fresh = true;
        int rc = begin_draw(c, fx->prog);
        if (rc) return rc;
        if (gy > 0 && c->backend == PT_BACKEND_WAVEFRONT) {
            HIPCHK(c, hipMemsetAsync(c->wf.cnt, 0, 16 * pt::kShards * sizeof(unsigned), c->stream));
            HIPCHK(c, pt_launch_wavefront(fx->prog, c->counting ? 1 : 0, &a, &c->wf, gx, gy, persist, c->stream));
        } else if (gy > 0) {
            HIPCHK(c, pt_launch_persist(fx->prog, c->counting ? 1 : 0, &a, &c->gb, gx, n_wave_tiles, c->persist_tiles,
                                        c->persist_refill, c->stream));
            HIPCHK(c, pt_launch_finish(&a, &c->gb, gx, gy, c->stream));
        }
        return end_draw(c, fx->prog);
    }

    // ---- the megakernel: draw k = mk_seq uses buffer set k % depth
    // late-bounce compaction and the frames in flight (cont_decide): when compaction is on, no split
    // tiles - their 16-lane waves would hand their slowest paths to pt_cont at once (r05j: dragon
    // stand-in 4K with both 2222 Mpaths/s, with compaction alone 2762)
    bool cont = false;
    int depth = c->depth;
    if (int rc = cont_decide(c, target, fx->prog, mesh && !c->counting && !PT_SECPROF_BUILD, &cont, &depth)) return rc;
    // a moving-camera draw that runs alone (PT_MOVING_SERIAL) does not compact: with no next frame beside it,
    // pt_cont's tail (a wave waits for its longest chain of walks) is the frame's (dragon stand-in 1080p
    // 1.19 -> 1.09 ms per frame, profiles/r06af_movpx.log); its slowest tiles are split instead
    if (a.moving && c->moving_serial) cont = false;
    const size_t traced = (size_t)target->w * target->h / (size_t)std::max(1, c->num_parts);   // (about)
    const int lag = draw_lag(c, traced);
    if (depth != c->depth_run || lag != c->lag_run) {   // another buffer-set cycle: the draw waits for everything before it
        c->depth_run = depth;
        c->lag_run = lag;
        c->need_fresh = true;
    }
    const unsigned nsets = (unsigned)(depth + lag);
    const int par = (int)(c->mk_seq % nsets);            // buffer set
    const int str = (int)(c->mk_seq % (unsigned)depth);  // stream and spill slab
    // longest-first: the wave durations of draw k - sets (same buffer set) order this draw's workgroups
    // when it drew the same grid, target and program; split tiles take 12 more workgroups each, in
    // padding rows
    const size_t n = (size_t)gx * gy;   // 16x16 tiles
    const Dev::LptKey& key = c->lpt_key[par];
    const bool lpt = c->lpt && !c->counting;
    const bool same = lpt && key.valid && key.n == n && key.target == target && key.prog == fx->prog &&
                      key.part == c->part && key.parts == c->num_parts && c->lpt_cap >= n;
    const unsigned split = same && !cont ? (unsigned)std::min<size_t>(c->split_tiles, n) & ~7u : 0u;   // the cap
    const unsigned extra = 4u * pt::kSplitParts - 4u;   // more workgroups per split tile
    const int gy_grid = gy + (int)((extra * split + 4u * gx - 1) / (4u * gx));
    if (mesh) {
        const size_t lanes = (size_t)gx * gy_grid * pt::kBlock;
        if (lanes * kSpillPerLane > 0xffffffffull)   // 32-bit slab index
            return fail(c, PT_ERR_ARG, "render target too large for the BVH stack slab");
        int rc = spill_reserve(c, lanes);
        if (rc) return rc;
        a.spill = spill_slab(c, str);
        a.spill_stride = lanes;
    }
    if (int rc = rad_reserve(c, (size_t)target->w * target->h)) return rc;
    a.rad = c->rad_mem + (size_t)par * c->rad_pixels;
    if (cont) {   // (records for this draw's set: allocated by cont_decide already, unless the lag changed)
        if (int rc = cont_reserve(c, traced_pixels(c, target), (int)nsets)) return rc;
        cont_args(c, par, a);
    }
    if (lpt && c->lpt_cap < n) {
        if (c->lpt_mem) {   // (side-stream order builds write it after their traced event: every stream first)
            HIPCHK(c, hipStreamSynchronize(c->stream));
            for (int p = 0; p < Dev::kDepthMax; p++)
                if (c->ts[p]) HIPCHK(c, hipStreamSynchronize(c->ts[p]));
            HIPCHK(c, hipFree(c->lpt_mem));
            c->lpt_mem = nullptr;
        }
        HIPCHK(c, hipMalloc(&c->lpt_mem, (5 * n + 1) * Dev::kSetsMax * sizeof(unsigned)));   // cost | order | split
        c->lpt_cap = n;
        c->need_fresh = true;
        for (auto& k : c->lpt_key) k.valid = false;
    }
    // where the path tracing runs: a side stream gated by the main stream's state when the previous
    // megakernel draw began (or now: the first draw, after another schedule or a stream switch, with
    // counting kernels, or when a sampler is a render target, which draws on the main stream may write)
    bool overlap = c->overlap && !c->counting && !PT_SECPROF_BUILD;   // (experiment builds: one wave log)
    if (a.moving && c->moving_serial) overlap = false;
    for (const auto& kv : fx->samplers)
        if (kv.second && kv.second->kind == TEX_RT && kv.first != "previousBuffer") overlap = false;
    hipStream_t ts = c->stream;
    if (overlap) {
        if (int rc = overlap_init(c)) return rc;
        const unsigned k = c->mk_seq, D = nsets;
        if (c->need_fresh) { c->mark_floor = k; c->need_fresh = false; }
        HIPCHK(c, hipEventRecord(c->ev_mark[par], c->stream));
        ts = c->ts[str];
        // the mark of draw k - sets + 1 (its state: draw k - sets' blend, order build and output), or
        // of the oldest draw after everything this draw must wait for; the draw k - depth before it on
        // this stream is ordered by the stream
        const unsigned w = k + 1 >= D ? std::max(k + 1 - D, c->mark_floor) : c->mark_floor;
        HIPCHK(c, hipStreamWaitEvent(ts, c->ev_mark[w % D], 0));
    } else {
        c->need_fresh = true;
    }
    if (lpt) {
        if (!same) HIPCHK(c, hipMemsetAsync(c->lpt_cost(par), 0, 4 * n * sizeof(unsigned), ts));   // costs start afresh
        a.order = same ? c->lpt_order(par) : nullptr;
        a.cost = c->lpt_cost(par);
        a.prio_tiles = a.order ? c->prio_tiles : 0u;
        // from both ends (runs of 8 tiles: the slowest, the cheapest, ...) also for compacting draws whose order
        // is not flattened: with the slowest tiles' late bounces handed to pt_cont, cheap tiles mixed in early
        // keep the slots full (dragon stand-in 1080p +1.5 %, its 20-frame run +1.7 %, helmet +1.6 %, three
        // rounds, profiles/r06bo_*; uncompacted the bunny lost 1.4 %, and at 4K the flattened order 1.9 %)
        a.order_zig = c->lpt_zig || (cont && c->zig_cont && n <= c->lpt_flat_tiles) ? 1u : 0u;
        a.split = (a.order && split) ? c->lpt_split(par) : nullptr;
    }
    a.ntiles = (unsigned)n;
    if (!a.order && c->xcd_blocked) a.order_zig = 2u;
    if (int rc = begin_draw(c, fx->prog, ts)) return rc;
    if (cont && c->cont_sort && a.bvh_walk != pt::WALK_REF) {   // (the model's root box: child-pair walks only)
        const size_t cap = c->cont_cap;
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        char* m = (char*)a.cont_rec + cap * 64 + al(cap * 4);
        a.cont_perm = (unsigned*)m;
        a.cont_rank = (unsigned*)(m + al(cap * 4));
        a.cont_key = (unsigned short*)(m + 2 * al(cap * 4));
        a.cont_bins = (unsigned*)(m + 2 * al(cap * 4) + al(cap * 2));
        // 8x8x8 cells for draws that trace 3 Mpx or more (4K: dragon stand-in +0.4 %, helmet +1.1 %, sky +
        // dragon +0.6 %, three rounds, profiles/r06bj_*; at 1080p the helmet lost 5.5 % with them, r06ao_*)
        const unsigned gb = c->cont_grid_env || c->cont_key_mode >= 3u || traced < c->cont_big_pixels ? c->cont_grid_bits : 3u;
        for (int k = 0; k < 3; k++) {
            const float ext = a.bvh_root_box[3 + k] - a.bvh_root_box[k];
            a.cont_cell[k] = ext > 0.0f ? (float)(1u << gb) / ext : 0.0f;
        }
        a.cont_grid_bits = gb;
        a.cont_key_mode = c->cont_key_mode;
    }
    HIPCHK(c, pt_launch_trace(fx->prog, c->counting ? 1 : 0, &a, gx, a.split ? gy_grid : gy, ts));
    if (a.cont_bins) {   // (PT_CONT_SORT) the records' order, from the keys' totals and ranks pt_trace took
        pt::SortArgs so;
        std::memset(&so, 0, sizeof(so));
        so.count = a.cont_count;
        so.key = a.cont_key;
        so.rank = a.cont_rank;
        so.bins = a.cont_bins;
        so.perm = (unsigned*)a.cont_perm;
        so.chunk = c->sort_chunk;
        so.nbins = (c->cont_key_mode == 3u ? 64u : c->cont_key_mode == 4u ? 32u : 16u) << (3u * a.cont_grid_bits);
        HIPCHK(c, pt_launch_cont_sort(&so, c->cont_cap, ts));
    }
    if (cont) {   // (its one-wave workgroups index the spill slab below the trace grid's lanes)
        // (the sky composite keeps 2048: its sky pixels store few records, and 1024 waves cost it 0.5 %)
        const bool big = !c->cont_waves_env && traced >= c->cont_big_pixels && fx->prog != PT_PROG_SKY_MESH;
        HIPCHK(c, pt_launch_cont(fx->prog, &a, (int)std::min<size_t>(big ? c->cont_waves_big : c->cont_waves, (size_t)gx * gy * 4), ts));
        c->cont_draws++;
    }
    // the draw's timing events bracket all of its path tracing on the side stream: pt_trace and, when the
    // draw compacts, pt_cont (the blend below is the main stream's)
    if (int rc = end_draw(c, fx->prog, ts)) return rc;
    const int near_arg = c->split_near | ((c->lpt_flat + 1) << 8) | (int)((c->lpt_flat_tiles / 64u) << 16);
    const unsigned split_cap = (unsigned)std::min<size_t>(c->split_tiles, n) & ~7u;
    bool side_order = false;
    if (overlap) {
        HIPCHK(c, hipEventRecord(c->ev_traced[str], ts));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_traced[str], 0));
        // the set's next draw runs on this stream (no lag), so the order it reads is built by then
        side_order = a.cost && lag == 0 && n > c->order_side_tiles;
        if (side_order)
            HIPCHK(c, pt_launch_order_build((unsigned)n, a.cost, c->lpt_order(par), c->lpt_split(par), split_cap,
                                            c->split_dominance, near_arg, ts, 64));
    }
    // the history half of main() on the main stream, where the copy / output draws that read the
    // accumulation follow
    pt::BlendArgs b{ a.width, a.height, a.num_parts, a.part, a.frame, a.moving, a.rad, a.prev, a.out, a.cont_count, a.cont_bins };
    // (one-wave workgroups up to 8192 tiles, as the output pass below)
    HIPCHK(c, pt_launch_blend(&b, gy, c->stream, n <= c->blend_1w_tiles ? c->main_waves : 0));
    if (a.cost) {   // this draw's costs order draw k + 2: the build rides along with the next screenOutput
        if (!side_order) {
            c->pending_order = { true, (unsigned)n, a.cost, c->lpt_order(par), c->lpt_split(par), split_cap,
                                 c->split_dominance, near_arg };
            if (!c->fuse_order) { if (int rc = flush_order(c)) return rc; }
        }
        c->lpt_key[par] = { true, n, target, fx->prog, c->part, c->num_parts };
    }
    c->mk_seq++;
    return PT_OK;
}

int launch_copy(Dev* c, DevTex* src, DevTex* dst, int num_parts, int part)
{
    pt::CopyArgs a{ dst->w, dst->h, num_parts, part, (const float4*)src->d, (float4*)dst->d };
    const int nb = (dst->h + pt::kTile - 1) / pt::kTile;
    int gx = (dst->w + 255) / 256, gy = part < nb ? (nb - part + num_parts - 1) / num_parts : 0;
    if (gy > 0) HIPCHK(c, pt_launch_copy(&a, gx, gy, c->stream));
    return PT_OK;
}

// run a deferred screenCopy now, as its own kernel (timed as a screenCopy draw)
int flush_copy(Dev* c)
{
    if (!c->pending_copy.on) return PT_OK;
    c->pending_copy.on = false;
    int rc = begin_draw(c, PT_PROG_SCREEN_COPY);
    if (rc) return rc;
    rc = launch_copy(c, c->pending_copy.src, c->pending_copy.dst, c->pending_copy.num_parts, c->pending_copy.part);
    if (rc) return rc;
    return end_draw(c, PT_PROG_SCREEN_COPY);
}

int render_copy(DevFx* fx, DevTex* target)
{
    Dev* c = fx->ctx;
    DevTex* src = sampler(fx, "pathTracedImageBuffer");
    if (!target || target->kind != TEX_RT) return fail(c, PT_ERR_ARG, "screenCopy needs a render target");
    if (!src || src->kind == TEX_U8 || src->w != target->w || src->h != target->h)
        return fail(c, PT_ERR_STATE, "pathTracedImageBuffer must be an RGBA32F texture of the target's size");
    int rc = flush_copy(c);
    if (rc) return rc;
    // deferred: the render loop's next draw is screenOutput of the same source, which writes the
    // copy target in the same pass (render_output); any other use flushes it first (flush_copy)
    if (src != target) c->pending_copy = { true, src, target, c->num_parts, c->part };
    return PT_OK;
}

int render_output(DevFx* fx, DevTex* target)
{
    Dev* c = fx->ctx;
    DevTex* acc = sampler(fx, "accumulationBuffer");
    if (!acc || acc->kind == TEX_U8) return fail(c, PT_ERR_STATE, "accumulationBuffer must be an RGBA32F texture");
    pt::OutputArgs a;
    std::memset(&a, 0, sizeof(a));
    a.acc = (const float4*)acc->d;
    a.acc_w = acc->w;
    a.acc_h = acc->h;
    a.one_over_n = uf(fx, "uOneOverSampleCounter");
    a.exposure = uf(fx, "uToneMappingExposure");
    a.num_parts = c->output_partition ? c->num_parts : 1;
    a.part = c->output_partition ? c->part : 0;
    // fuse the deferred screenCopy when this pass covers exactly its texels: same source, same
    // frame size, same bands, and the copy target is not this pass's output
    const auto& pc = c->pending_copy;
    const int ow = target ? target->w : (c->cw || c->ch ? c->cw : acc->w), oh = target ? target->h : (c->cw || c->ch ? c->ch : acc->h);
#ifdef PT_NO_FUSE_COPY   // experiment builds: the copy as its own kernel (what the fusion saves)
    const bool fuse = false;
#else
    const bool fuse = pc.on && pc.src == acc && pc.dst != target && ow == acc->w && oh == acc->h &&
                      pc.num_parts == a.num_parts && (pc.num_parts == 1 || pc.part == a.part);
#endif
    if (fuse) { a.copy_dst = (float4*)pc.dst->d; c->pending_copy.on = false; }
    else { int frc = flush_copy(c); if (frc) return frc; }
    if (target) {
        if (target->kind != TEX_RT) return fail(c, PT_ERR_ARG, "screenOutput target must be a render target or the canvas");
        a.width = target->w; a.height = target->h; a.out_f = (float4*)target->d;
    } else {
        if (c->cw == 0 && c->ch == 0) {
            int rc = dev_canvas_resize(c, acc->w, acc->h);
            if (rc) return rc;
        }
        a.width = c->cw; a.height = c->ch; a.canvas = c->canvas;
    }
    // the order build rides along only up to 32768 tiles (4K): beyond, the block's 256 threads would
    // loop over memory and outlast the pass, so it runs alone first (1024 threads)
    if (c->pending_order.on && c->pending_order.n > pt::kOrderHeld * 256u)
        if (int frc = flush_order(c)) return frc;
    int rc = begin_draw(c, fx->prog);
    if (rc) return rc;
    if (a.width > 0 && a.height > 0) {
        if (c->pending_order.on) {   // the last megakernel draw's order build rides along as one more block
            const auto& po = c->pending_order;
            a.ob_cost = po.cost; a.ob_order = po.order; a.ob_split = po.split;
            a.ob_ntiles = po.n; a.ob_cap = po.cap; a.ob_dominance = po.dominance; a.ob_near = po.near;
            c->pending_order.on = false;
        }
        // one-wave workgroups while a fused order build fits one wave's registers (<= 8192 tiles: up to
        // ~2 MP, and a rank's share of 4K), else the 4-wave blocks with a 256-thread order build
        const int nb = (a.height + 15) / 16, ob = a.part < nb ? (nb - a.part + a.num_parts - 1) / a.num_parts : 0;
        const unsigned tiles = (unsigned)((a.width + 15) / 16) * (unsigned)ob;   // (as pt_launch_output's grid)
        const bool one = a.ob_cost ? tiles <= pt::kOrderHeld * 64u && a.ob_ntiles <= pt::kOrderHeld * 64u
                                   : tiles <= c->out_1w_tiles;
        HIPCHK(c, pt_launch_output(&a, c->stream, one ? c->main_waves : 0));
    }
    return end_draw(c, fx->prog);
}

DevTex* new_texture(Dev* c, int kind, int w, int h, size_t texel, int* err)
{
    auto* t = new DevTex();
    t->ctx = c; t->kind = kind; t->w = w; t->h = h;
    t->bytes = (size_t)w * (size_t)h * texel;
    if (t->bytes) {
        hipError_t e = hipMalloc(&t->d, t->bytes);
        if (e != hipSuccess) {
            hipfail(c, e, "hipMalloc");
            delete t;
            if (err) *err = PT_ERR_OOM;
            return nullptr;
        }
    }
    c->textures.insert(t);
    return t;
}

DevTex* upload(Dev* c, int kind, int w, int h, const void* data, size_t texel, int sampling, int invert_y, int* err)
{
    if (err) *err = PT_OK;
    if (!c || w <= 0 || h <= 0 || (long long)w * h >= (1ll << 31)) { if (err) *err = PT_ERR_ARG; return nullptr; }
    hipSetDevice(c->device);
    DevTex* t = new_texture(c, kind, w, h, texel, err);
    if (!t) return nullptr;
    t->sampling = sampling; t->invert_y = invert_y;
    hipError_t e = hipSuccess;
    if (!data) e = hipMemsetAsync(t->d, 0, t->bytes, c->stream);
    else if (!invert_y) e = hipMemcpyAsync(t->d, data, t->bytes, hipMemcpyHostToDevice, c->stream);
    else {
        const size_t row = (size_t)w * texel;   // UNPACK_FLIP_Y: source row r lands on row h-1-r
        for (int r = 0; r < h && e == hipSuccess; r++)
            e = hipMemcpyAsync((char*)t->d + (size_t)(h - 1 - r) * row, (const char*)data + (size_t)r * row, row,
                               hipMemcpyHostToDevice, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);   // the caller keeps ownership of data
    if (e != hipSuccess) {
        hipfail(c, e, "texture upload");
        dev_texture_destroy(t);
        if (err) *err = PT_ERR_HIP;
        return nullptr;
    }
    return t;
}

}  // namespace

// ---------------------------------------------------------------------------- device-level API
// (pt_dev.h; the exported C ABI in pt_group.cpp forwards here, once per part of a context)

Dev* dev_ctx_create(int device, int* err)
{
    if (err) *err = PT_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        if (err) *err = PT_ERR_DEVICE;
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        if (err) *err = PT_ERR_DEVICE;   // the code objects are gfx950-only
        return nullptr;
    }
    auto* c = new Dev();
    c->device = device;
    c->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (const char* v = std::getenv("PT_PERSIST_TILES")) c->persist_tiles = (unsigned)std::max(1, std::atoi(v));
    if (const char* v = std::getenv("PT_DRAW_EVENTS")) c->draw_events = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_LPT")) { c->lpt = std::atoi(v) != 0; c->lpt_zig = std::atoi(v) == 2; }
    if (const char* v = std::getenv("PT_LPT_ZIG_CONT")) c->zig_cont = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_XCD_BLOCKED")) c->xcd_blocked = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_PRIO_TILES")) c->prio_tiles = (unsigned)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_SPLIT_TILES")) c->split_tiles = (unsigned)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_FUSE_ORDER")) c->fuse_order = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_MAIN_WAVES")) c->main_waves = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_BLEND_1W_TILES")) c->blend_1w_tiles = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_OUT_1W_TILES")) c->out_1w_tiles = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_ORDER_SIDE_TILES")) c->order_side_tiles = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_OVERLAP")) c->overlap = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_MOVING_SERIAL")) c->moving_serial = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_OVERLAP_DEPTH")) {
        c->depth = std::min(Dev::kDepthMax, std::max(2, std::atoi(v)));
        c->depth_env = true;
    }
    c->depth_run = c->depth;
    if (const char* v = std::getenv("PT_OVERLAP_LAG")) c->lag = std::min(Dev::kLagMax, std::max(-1, std::atoi(v)));
    if (const char* v = std::getenv("PT_OVERLAP_LAG_PIXELS")) c->lag_pixels = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_CONT")) c->cont_mode = std::min(2, std::max(0, std::atoi(v)));
    if (const char* v = std::getenv("PT_CONT_BOUNCE")) c->cont_bounce = (unsigned)std::max(2, std::atoi(v));
    if (const char* v = std::getenv("PT_CONT_LANES")) c->cont_lanes = (unsigned)std::min(64, std::max(1, std::atoi(v)));
    if (const char* v = std::getenv("PT_CONT_REFILL")) c->cont_refill = (unsigned)std::min(64, std::max(1, std::atoi(v)));
    if (const char* v = std::getenv("PT_CONT_SORT")) c->cont_sort = std::atoi(v) != 0;
    if (const char* v = std::getenv("PT_CONT_SORT_CHUNK")) c->sort_chunk = (unsigned)std::max(64, std::atoi(v));
    if (const char* v = std::getenv("PT_CONT_SORT_GRID")) { c->cont_grid_bits = (unsigned)std::min(3, std::max(1, std::atoi(v))); c->cont_grid_env = true; }
    if (const char* v = std::getenv("PT_CONT_SORT_KEY")) c->cont_key_mode = (unsigned)std::min(4, std::max(0, std::atoi(v)));
    if (c->cont_key_mode >= 3u) c->cont_grid_bits = std::min(2u, c->cont_grid_bits);   // (at most kSortBins keys)
    if (const char* v = std::getenv("PT_CONT_WAVES")) { c->cont_waves = (unsigned)std::max(1, std::atoi(v)); c->cont_waves_env = true; }
    if (const char* v = std::getenv("PT_CONT_WAVES_BIG")) c->cont_waves_big = (unsigned)std::max(1, std::atoi(v));
    if (const char* v = std::getenv("PT_CONT_BIG_PIXELS")) c->cont_big_pixels = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_CONT_AUTO_PIXELS")) c->cont_auto_pixels = (size_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("PT_LPT_FLAT")) c->lpt_flat = std::max(-1, std::min(127, std::atoi(v)));
    if (const char* v = std::getenv("PT_LPT_FLAT_TILES")) c->lpt_flat_tiles = (unsigned)std::max(0, std::min(1 << 21, std::atoi(v)));
    if (const char* v = std::getenv("PT_SPLIT_NEAR")) c->split_near = std::max(1, std::min(128, std::atoi(v)));
    if (const char* v = std::getenv("PT_SPLIT_ALWAYS")) c->split_dominance = std::atoi(v) ? 0u : 8u;
    if (const char* v = std::getenv("PT_BVH_LAYOUT"))   // reference | pairs | trail: the context's initial walk
        c->bvh_layout = !std::strcmp(v, "trail") ? PT_BVH_TRAIL : !std::strcmp(v, "reference") ? PT_BVH_REFERENCE
                                                                                  : PT_BVH_PAIRS;
    if (const char* v = std::getenv("PT_PERSIST_REFILL")) c->persist_refill = (unsigned)std::min(64, std::max(1, std::atoi(v)));
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) {
        // (experiment, PT_MAIN_PRIO=1) the context's stream - blend, copy, output - at the device's highest
        // priority, so that its small kernels take freed CU slots before the side streams' path tracing
        const char* mp = std::getenv("PT_MAIN_PRIO");
        int least = 0, greatest = 0;
        if (mp && std::atoi(mp) != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
            e = hipStreamCreateWithPriority(&c->own_stream, hipStreamNonBlocking, greatest);
        else
            e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    }
    c->stream = c->own_stream;
    if (e == hipSuccess) e = hipMalloc(&c->d_err, 256);
    if (e == hipSuccess) e = hipMalloc(&c->d_counters, pt::C_NUM * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemsetAsync(c->d_err, 0, 256, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_counters, 0, pt::C_NUM * sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        if (err) *err = PT_ERR_HIP;
        dev_ctx_destroy(c);
        return nullptr;
    }
    return c;
}

void dev_ctx_destroy(Dev* c)
{
    if (!c) return;
    hipSetDevice(c->device);
    c->pending_copy.on = false;   // nothing can observe its target any more
    c->pending_order.on = false;  // ... nor a next draw the order
    if (c->stream) hipStreamSynchronize(c->stream);
    for (int p = 0; p < Dev::kDepthMax; p++)   // (side-stream order builds may still write the order arrays)
        if (c->ts[p]) hipStreamSynchronize(c->ts[p]);
    std::vector<DevFx*> fx(c->effects.begin(), c->effects.end());
    for (auto* f : fx) dev_effect_destroy(f);
    std::vector<DevTex*> tx(c->textures.begin(), c->textures.end());
    for (auto* t : tx) dev_texture_destroy(t);
    for (auto& pr : c->pool) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
    for (int i = 0; i < kProgSlots; i++) {
        if (c->ev0[i]) hipEventDestroy(c->ev0[i]);
        if (c->ev1[i]) hipEventDestroy(c->ev1[i]);
    }
    if (c->canvas && !c->canvas_external) hipFree(c->canvas);
    if (c->wf_mem) hipFree(c->wf_mem);
    if (c->lpt_mem) hipFree(c->lpt_mem);
    if (c->mk_spill) hipFree(c->mk_spill);
    if (c->rad_mem) hipFree(c->rad_mem);
    if (c->cont_mem) hipFree(c->cont_mem);
    for (auto& e : c->tune_ev) if (e) hipEventDestroy(e);
    for (int p = 0; p < Dev::kSetsMax; p++)
        if (c->ev_mark[p]) hipEventDestroy(c->ev_mark[p]);
    for (int p = 0; p < Dev::kDepthMax; p++) {   // (every side-stream draw was waited for by a blend on the main stream)
        if (c->ts[p]) { hipStreamSynchronize(c->ts[p]); hipStreamDestroy(c->ts[p]); }
        if (c->ev_traced[p]) hipEventDestroy(c->ev_traced[p]);
    }
    if (c->gb_mem) hipFree(c->gb_mem);
    if (c->d_err) hipFree(c->d_err);
    if (c->d_counters) hipFree(c->d_counters);
    if (c->own_stream) hipStreamDestroy(c->own_stream);
    delete c;
}

const char* dev_last_error(Dev* c) { return c ? c->err.c_str() : "no context"; }

int dev_sync(Dev* c)
{
    if (!c) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    unsigned flags = 0;
    HIPCHK(c, hipMemcpy(&flags, c->d_err, sizeof(flags), hipMemcpyDeviceToHost));
    if (flags) {   // (on the main stream, which the next draw's path tracing waits for: not the null stream)
        HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(unsigned), c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->need_fresh = true;
        if (flags & pt::E_STACK) return fail(c, PT_ERR_DATA, "BVH traversal needed more than stackLevels[28]");
    }
    return PT_OK;
}

int dev_canvas_resize(Dev* c, int w, int h)
{
    if (!c || w < 0 || h < 0) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (w == c->cw && h == c->ch && c->canvas && !c->canvas_external) return PT_OK;
    if (c->canvas) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (!c->canvas_external) HIPCHK(c, hipFree(c->canvas));
        c->canvas = nullptr;
    }
    c->canvas_external = false;
    c->cw = w; c->ch = h;
    if (w * (size_t)h) {
        HIPCHK(c, hipMalloc(&c->canvas, (size_t)w * h * sizeof(uchar4)));
        HIPCHK(c, hipMemsetAsync(c->canvas, 0, (size_t)w * h * sizeof(uchar4), c->stream));
    }
    return PT_OK;
}

int dev_canvas_wrap(Dev* c, int w, int h, void* ptr)
{
    if (!c || w <= 0 || h <= 0 || !ptr) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (c->canvas && !c->canvas_external) {   // switching between wrapped canvases needs no sync
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->canvas));
    }
    c->canvas = (uchar4*)ptr;
    c->canvas_external = true;
    c->cw = w; c->ch = h;
    return PT_OK;
}

int dev_set_output_partition(Dev* c, int enable)
{
    if (!c) return PT_ERR_ARG;
    c->output_partition = enable != 0;
    return PT_OK;
}

DevFx* dev_effect_create(Dev* c, const char* src, const char* const* un, int nu, const char* const* sn, int ns, int* err)
{
    if (err) *err = PT_OK;
    if (!c || !src) { if (err) *err = PT_ERR_ARG; return nullptr; }
    int prog = classify(src);
    if (prog == PT_PROG_UNKNOWN) {
        fail(c, PT_ERR_SHADER, "fragment shader not recognised as a reference path-tracing program");
        if (err) *err = PT_ERR_SHADER;
        return nullptr;
    }
    return dev_effect_create_program(c, prog, un, nu, sn, ns, err);
}

DevFx* dev_effect_create_program(Dev* c, int prog, const char* const* un, int nu, const char* const* sn, int ns, int* err)
{
    if (err) *err = PT_OK;
    if (!c || nu < 0 || ns < 0 || prog <= PT_PROG_UNKNOWN || prog > PT_PROG_SKY_MESH) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* fx = new DevFx();
    fx->ctx = c;
    fx->prog = prog;
    for (int i = 0; i < nu; i++) if (un && un[i]) fx->uniforms[un[i]] = Uniform();
    for (int i = 0; i < ns; i++) if (sn && sn[i]) fx->samplers[sn[i]] = nullptr;
    c->effects.insert(fx);
    return fx;
}

void dev_effect_destroy(DevFx* fx)
{
    if (!fx) return;
    fx->ctx->effects.erase(fx);
    delete fx;
}

int dev_effect_program(const DevFx* fx) { return fx ? fx->prog : PT_PROG_UNKNOWN; }

int dev_set_float(DevFx* fx, const char* name, const float* v, int n)
{
    if (!fx || !name || !v || n < 1 || n > 16) return PT_ERR_ARG;
    auto it = fx->uniforms.find(name);
    if (it == fx->uniforms.end()) return PT_OK;   // undeclared: ignored, as in Babylon
    Uniform& u = it->second;
    u.is_int = false; u.n = n; u.set = true;
    for (int k = 0; k < n; k++) u.f[k] = v[k];
    return PT_OK;
}

int dev_set_int(DevFx* fx, const char* name, int v)
{
    if (!fx || !name) return PT_ERR_ARG;
    auto it = fx->uniforms.find(name);
    if (it == fx->uniforms.end()) return PT_OK;
    Uniform& u = it->second;
    u.is_int = true; u.n = 1; u.i = v; u.set = true;
    return PT_OK;
}

int dev_set_texture(DevFx* fx, const char* name, DevTex* t)
{
    if (!fx || !name) return PT_ERR_ARG;
    if (t && t->ctx != fx->ctx) return fail(fx->ctx, PT_ERR_ARG, "texture belongs to another context");
    auto it = fx->samplers.find(name);
    if (it == fx->samplers.end()) return PT_OK;
    it->second = t;
    return PT_OK;
}

DevTex* dev_texture_create_rgba32f(Dev* c, int w, int h, const float* data, int sampling, int invert_y, int* err)
{
    return upload(c, TEX_F32, w, h, data, 16, sampling, invert_y, err);
}

DevTex* dev_texture_create_rgba8(Dev* c, int w, int h, const uint8_t* data, int sampling, int invert_y, int* err)
{
    return upload(c, TEX_U8, w, h, data, 4, sampling, invert_y, err);
}

DevTex* dev_render_target_create(Dev* c, int w, int h, int* err)
{
    return upload(c, TEX_RT, w, h, nullptr, 16, PT_SAMPLING_NEAREST, 0, err);
}

DevTex* dev_render_target_wrap(Dev* c, int w, int h, void* dptr, int* err)
{
    if (err) *err = PT_OK;
    if (!c || w <= 0 || h <= 0 || !dptr) { if (err) *err = PT_ERR_ARG; return nullptr; }
    auto* t = new DevTex();
    t->ctx = c; t->kind = TEX_RT; t->w = w; t->h = h;
    t->bytes = (size_t)w * h * 16;
    t->d = dptr;
    t->external = true;
    c->textures.insert(t);
    return t;
}

int dev_render_target_resize(DevTex* t, int w, int h)
{
    if (!t || t->kind != TEX_RT || w <= 0 || h <= 0) return PT_ERR_ARG;
    if (t->external) return fail(t->ctx, PT_ERR_ARG, "wrapped render targets are not resizable");
    Dev* c = t->ctx;
    if (w == t->w && h == t->h) return PT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (t->d) HIPCHK(c, hipFree(t->d));
    t->d = nullptr;
    t->w = w; t->h = h; t->bytes = (size_t)w * h * 16;
    HIPCHK(c, hipMalloc(&t->d, t->bytes));
    HIPCHK(c, hipMemsetAsync(t->d, 0, t->bytes, c->stream));
    return PT_OK;
}

int dev_texture_size(const DevTex* t, int* w, int* h)
{
    if (!t) return PT_ERR_ARG;
    if (w) *w = t->w;
    if (h) *h = t->h;
    return PT_OK;
}

void dev_texture_destroy(DevTex* t)
{
    if (!t) return;
    Dev* c = t->ctx;
    hipSetDevice(c->device);
    if (c->pending_copy.on && (c->pending_copy.src == t || c->pending_copy.dst == t)) flush_copy(c);
    for (auto* fx : c->effects)
        for (auto& kv : fx->samplers)
            if (kv.second == t) kv.second = nullptr;
    if (t->d && !t->external) { hipStreamSynchronize(c->stream); hipFree(t->d); }
    if (t->pairs_mem) { hipStreamSynchronize(c->stream); hipFree(t->pairs_mem); }
    for (auto* o : c->textures)   // records built against this triangle texture are stale
        if (o->pairs_tri == t) { o->pairs_tri = nullptr; o->pairs_gen = ~0ull; }
    c->textures.erase(t);
    delete t;
}

int dev_render(DevFx* fx, DevTex* target)
{
    if (!fx) return PT_ERR_ARG;
    Dev* c = fx->ctx;
    if (target && target->ctx != c) return fail(c, PT_ERR_ARG, "target belongs to another context");
    HIPCHK(c, hipSetDevice(c->device));
    if (fx->prog != PT_PROG_SCREEN_OUTPUT && fx->prog != PT_PROG_SCREEN_COPY) {
        int rc = flush_copy(c);
        if (rc) return rc;
    }
    switch (fx->prog) {
    case PT_PROG_CORNELL:
    case PT_PROG_QUADRIC:
    case PT_PROG_SKY:
    case PT_PROG_SKY_MESH:
    case PT_PROG_HDRI:
    case PT_PROG_GLTF: return render_trace(fx, target);
    case PT_PROG_SCREEN_COPY: return render_copy(fx, target);
    case PT_PROG_SCREEN_OUTPUT: return render_output(fx, target);
    default: return fail(c, PT_ERR_UNSUPPORTED, "program recognised but not implemented in this build");
    }
}

int dev_read_pixels(Dev* c, const DevTex* t, void* dst, size_t bytes)
{
    if (!c || !dst) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    const void* src = t ? t->d : (const void*)c->canvas;
    size_t need = t ? t->bytes : (size_t)c->cw * c->ch * sizeof(uchar4);
    if (bytes < need) return fail(c, PT_ERR_ARG, "destination too small");
    HIPCHK(c, hipMemcpyAsync(dst, src, need, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int dev_write_pixels(Dev* c, DevTex* t, const void* src, size_t bytes)
{
    if (!c || !t || !src || bytes != t->bytes) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    HIPCHK(c, hipMemcpyAsync(t->d, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    t->gen++;
    return PT_OK;
}

int dev_set_stream(Dev* c, void* stream)
{
    if (!c) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    if (int rc = flush_order(c)) return rc;        // on the stream its draw ran on
    HIPCHK(c, hipStreamSynchronize(c->stream));   // work already queued finishes first
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    c->need_fresh = true;   // the next megakernel draw waits for the new stream's state
    return PT_OK;
}

int dev_set_backend(Dev* c, int backend)
{
    if (!c || (backend != PT_BACKEND_MEGAKERNEL && backend != PT_BACKEND_WAVEFRONT && backend != PT_BACKEND_PERSISTENT))
        return PT_ERR_ARG;
    c->backend = backend;
    return PT_OK;
}

int dev_set_bvh_layout(Dev* c, int layout)
{
    if (!c || layout < PT_BVH_REFERENCE || layout > PT_BVH_TRAIL) return PT_ERR_ARG;
    c->bvh_layout = layout;
    return PT_OK;
}

int dev_bvh_layout_used(Dev* c) { return c ? c->bvh_used : PT_ERR_ARG; }

int dev_set_row_partition(Dev* c, int num_parts, int part)
{
    if (!c || num_parts < 1 || part < 0 || part >= num_parts) return PT_ERR_ARG;
    c->num_parts = num_parts;
    c->part = part;
    return PT_OK;
}

void* dev_texture_device_ptr(DevTex* t) { return t ? t->d : nullptr; }

int dev_last_render_ms(Dev* c, int prog, float* ms)
{
    if (!c || !ms || prog < 0 || prog >= kProgSlots) return PT_ERR_ARG;
    if (!c->draw_events) {   // the first call turns the per-draw events on; later draws report
        c->draw_events = true;
        return fail(c, PT_ERR_ARG, "per-draw timing was off: it is on from now, for the next draws");
    }
    if (!c->ev_used[prog]) return fail(c, PT_ERR_ARG, "no timed draw of this program yet");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipEventElapsedTime(ms, c->ev0[prog], c->ev1[prog]));
    return PT_OK;
}

int dev_timing_begin(Dev* c)
{
    if (!c) return PT_ERR_ARG;
    c->window = true;
    c->window_draws.clear();
    std::fill(c->window_seen, c->window_seen + kProgSlots, 0);
    if (const char* v = std::getenv("PT_TIMING_EVERY")) c->timing_every = std::max(1, std::atoi(v));
    return PT_OK;
}

int dev_timing_end(Dev* c, int prog, double* total_ms, int* launches)
{
    if (!c || !total_ms || !launches) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->window = false;   // the window is closed; its draws stay readable by further dev_timing_end calls
    double t = 0.0;
    int n = 0;
    for (auto& d : c->window_draws) {
        if (d.first != prog) continue;
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->pool[d.second].first, c->pool[d.second].second));
        t += ms;
        n++;
    }
    *total_ms = t;
    *launches = n;
    return PT_OK;
}

int dev_timing_latency(Dev* c, int prog, float* ms, int cap, int* n)
{
    if (!c || !n || cap < 0 || (cap && !ms)) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_copy(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->window = false;
    // each bracketed draw of `prog` with the next bracketed screenOutput draw: the same frame's, as long as
    // every frame draws one of each (the window brackets every timing_every-th draw of each kind)
    int k = 0, open = -1;
    for (auto& d : c->window_draws) {
        if (d.first == prog) open = d.second;
        else if (d.first == PT_PROG_SCREEN_OUTPUT && open >= 0) {
            float t = 0.0f;
            HIPCHK(c, hipEventElapsedTime(&t, c->pool[open].first, c->pool[d.second].second));
            if (k < cap) ms[k] = t;
            k++;
            open = -1;
        }
    }
    *n = std::min(k, cap);
    return PT_OK;
}

int dev_set_counting(Dev* c, int enable)
{
    if (!c) return PT_ERR_ARG;
    c->counting = enable != 0;
    return PT_OK;
}

int dev_read_counters(Dev* c, uint64_t out[PT_NUM_COUNTERS])
{
    if (!c || !out) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->d_counters, pt::C_NUM * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

int dev_reset_counters(Dev* c)
{
    if (!c) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->d_counters, 0, pt::C_NUM * sizeof(unsigned long long), c->stream));
    return PT_OK;
}

int dev_queue_stats(Dev* c, uint32_t out[16])
{
    if (!c || !out) return PT_ERR_ARG;
    std::memset(out, 0, 16 * sizeof(uint32_t));
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = flush_order(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int q = 0; q < Dev::kDepthMax; q++)   // (a side-stream order build may still write the split count)
        if (c->ts[q]) HIPCHK(c, hipStreamSynchronize(c->ts[q]));
    const int p = (int)(c->mk_seq % (unsigned)(c->depth_run + c->lag_run));   // the tiles the next megakernel draw of the same grid splits
    if (c->lpt_mem && c->lpt_key[p].valid)
        HIPCHK(c, hipMemcpy(&out[7], c->lpt_split(p), sizeof(uint32_t), hipMemcpyDeviceToHost));
    // late-bounce compaction of the last megakernel draw: 0 off, 1 auto decided off, 2 auto decided on,
    // 3 forced on (PT_CONT=1), 4 auto trial, 5 / 6 default on / off; bits 8-15: its frames in flight;
    // bits 16-31: the draws that launched pt_cont so far (mod 2^16);
    // out[15]: the auto trial's ms with it on per ms without (the faster depth), x 1000
    out[14] = (uint32_t)c->cont_last | (uint32_t)c->depth_run << 8 | (c->cont_draws & 0xffffu) << 16;
    const float off = std::min(c->tune.ms_off, c->tune.ms_off2);
    out[15] = (c->cont_last == 1 || c->cont_last == 2) && off > 0.0f ? (uint32_t)(1000.0f * c->tune.ms_on / off) : 0u;
    if (!c->wf_mem) return PT_OK;
    std::vector<unsigned> h(16 * pt::kShards);
    HIPCHK(c, hipMemcpy(h.data(), c->wf.cnt, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    for (int b = 0; b < 7; b++)
        for (int s = 0; s < pt::kShards; s++) {
            out[b] += h[b * pt::kShards + s];
            if (b < 6) out[8 + b] += h[(8 + b) * pt::kShards + s];
        }
    return PT_OK;
}

int dev_math_exhaustive(Dev* c, int op, uint64_t* mismatches)
{
    if (!c || !mismatches || op < 0 || op > 1) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    unsigned long long* d = nullptr;
    HIPCHK(c, hipMalloc(&d, sizeof(unsigned long long)));
    HIPCHK(c, hipMemsetAsync(d, 0, sizeof(unsigned long long), c->stream));
    HIPCHK(c, pt_launch_exhaustive(op, d, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    unsigned long long h = 0;
    HIPCHK(c, hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost));
    hipFree(d);
    *mismatches = h;
    return PT_OK;
}

int dev_math_probe(Dev* c, int op, const float* x, const float* y, float* out, int n)
{
    if (!c || !x || !out || n <= 0) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    size_t b = (size_t)n * sizeof(float);
    HIPCHK(c, hipMalloc(&dx, b));
    HIPCHK(c, hipMalloc(&dout, b));
    if (y) HIPCHK(c, hipMalloc(&dy, b));
    HIPCHK(c, hipMemcpy(dx, x, b, hipMemcpyHostToDevice));
    if (y) HIPCHK(c, hipMemcpy(dy, y, b, hipMemcpyHostToDevice));
    HIPCHK(c, pt_launch_math_probe(op, dx, dy, dout, n, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, dout, b, hipMemcpyDeviceToHost));
    hipFree(dx); hipFree(dout);
    if (dy) hipFree(dy);
    return PT_OK;
}


int dev_device(const Dev* c) { return c->device; }
hipStream_t dev_stream(const Dev* c) { return c->stream; }
void* dev_canvas_ptr(Dev* c) { return c->canvas; }
int dev_flush(Dev* c)
{
    HIPCHK(c, hipSetDevice(c->device));
    return flush_copy(c);
}
