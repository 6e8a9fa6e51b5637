// pt_trace.h — the per-pixel path-tracing kernels as templates over the program variant (the
// scene program x PBR code x BVH walk): pt_trace<PROG,COUNT,CONT> (the megakernel; CONT: late-bounce compaction, with pt_cont) and pt_persist<PROG,COUNT>
// (path regeneration). Instantiated per BVH walk in pt_trace_walk*.hip (one translation unit each, so
// the variants compile in parallel); see pt_kernels.hip for the mapping onto CDNA4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_device.h"
#include "pt_glsl.h"
#include "pt_program.h"
#ifdef PT_SECPROF
#define PT_SECPROF_ON 1
#else
#define PT_SECPROF_ON 0
#endif

using namespace ptg;

namespace pt {

// LS = lanes of the block = the stride of one stack level in LDS; NL = stack levels in LDS
template <int LS, int NL, bool SCRATCH>
struct MegaStack {
    lds_float2* lds;
    unsigned slot;
    glb_float2* slab;     // the spill slab (wave-uniform base) ...
    unsigned deep;        // ... and this lane's index in it: level NL, levels `stride` apart
    unsigned stride;      //     (32-bit: a 64-bit per-lane pointer costs two VGPRs for the whole path)
#ifdef PT_SECPROF
    mutable unsigned n_get = 0, n_get_slab = 0, n_put = 0, n_put_slab = 0;
#define PT_SLABCOUNT(x) x
#else
#define PT_SLABCOUNT(x)
#endif
    // the common case without branches: every lane reads LDS level min(si, NL - 1); lanes
    // deeper than the LDS levels then read the slab (or get the sentinel)
    PT_D float2 pop(int si, float2 sentinel) const
    {
        PT_SLABCOUNT(n_get++; if (si >= NL) n_get_slab++;)
        vf2 e = lds[(unsigned)min(si, NL - 1) * LS + slot];
        if (si >= NL) {
            const vf2 s = { sentinel.x, sentinel.y };
            e = si < kStackLevels ? slab[(unsigned)(si - NL) * stride + deep] : s;
        }
        return make_float2(e.x, e.y);
    }
    // SCRATCH (kScratchOf): every lane writes LDS level min(si, NL), level NL being a scratch
    // level that takes the deeper lanes' store, which then also goes to the slab - no exec-mask
    // change. Otherwise lanes within the LDS levels store there (a masked ds_write): where LDS
    // bounds the residency (the 8-wave variants) the scratch level's 512 B per wave is a stack
    // level more (6 instead of 5 + scratch: dragon stand-in +1.5 %, sky + dragon +2.2 %; the
    // textured 4-wave variants keep the scratch form, 1 % faster there).
    // False beyond stackLevels[27].
    PT_D bool push(int si, float2 e)
    {
        const vf2 v = { e.x, e.y };
        PT_SLABCOUNT(n_put++; if (si >= NL) n_put_slab++;)
        if (SCRATCH) lds[(unsigned)min(si, NL) * LS + slot] = v;
        else if (si < NL) lds[(unsigned)si * LS + slot] = v;
        if (si >= NL) {
            if (si >= kStackLevels) return false;
            slab[(unsigned)(si - NL) * stride + deep] = v;
        }
        return true;
    }
};

// the mesh hit's attributes (js/GLTFModelPathTracing_FragmentShader.js:300-346): interpolated
// normal and uv from the triangle texels 2-5, optional bump map, model transform
template <int PROG, bool COUNT>
PT_D void meshHit(const TraceArgs& a, float triID, float triU, float triV, Hit& h, Cnt& cnt)
{
    float4 v2 = fetch32(a.tri, a.tri_texels, triID + 2.0f), v3 = fetch32(a.tri, a.tri_texels, triID + 3.0f),
           v4 = fetch32(a.tri, a.tri_texels, triID + 4.0f), v5 = fetch32(a.tri, a.tri_texels, triID + 5.0f);
    if (COUNT) cnt.hit++;
    float triW = 1.0f - triU - triV;
    f3 nn = normalize(mk(v2.y, v2.z, v2.w) * triW + mk(v3.x, v3.y, v3.z) * triU + mk(v3.w, v4.x, v4.y) * triV);
    h.u = triW * v4.z + triU * v5.x + triV * v5.z;
    h.v = triW * v4.w + triU * v5.y + triV * v5.w;
    if (kHasTex<PROG> && a.uses_bump) {   // perturbNormal(n, vec2(1), uv), js/GLTFModelPathTracing_FragmentShader.js:72-92
        f3 S = onb_u(nn);
        f3 T = cross(nn, S);
        f3 N = normalize(nn);
        if (dot(cross(S, T), N) < 0.0f) { S = S * -1.0f; T = T * -1.0f; }
        float tx[4];
        texBilinear(a.bump, h.u, h.v, tx);
        if (COUNT) cnt.tap += 4;
        f3 mN = normalize(mk(tx[0] * 2.0f - 1.0f, tx[1] * 2.0f - 1.0f, tx[2] * 2.0f - 1.0f));
        mN.x *= 1.0f; mN.y *= 1.0f;
        nn = normalize(S * mN.x + T * mN.y + N * mN.z);
    }
    h.normal = normalize(mul3t(a.model, nn));
    h.type = a.uses_albedo ? PBR_MATERIAL : a.model_mat;
    h.color = mk(1.0f, 1.0f, 1.0f);
    h.id = meshObjectId<PROG>(a);
}

// SceneIntersect: js/BabylonPathTracing_FragmentShader.js:47-112 (Cornell),
// js/TransformedQuadricGeometry_FragmentShader.js:77-317 (quadrics) and
// js/GLTFModelPathTracing_FragmentShader.js:116-346 (glTF, with the BVH walk)
template <int PROG, bool COUNT, int LS>
PT_D void sceneIntersect(const TraceArgs& a, f3 rayO, f3 rayD, Hit& h, float2* lds, unsigned lane_slot,
                         unsigned deep, Cnt& cnt, bool firstHit)
{
    // `firstHit`: of this segment's hit only "the light / nothing / something else" is read (bounceStep
    // decides which segments). The walk may then stop at the first triangle closer than the analytic
    // winner - the reference's walk, visiting the same nodes in the same order up to there, also ends
    // with the mesh in front, as its hitT only falls - and the hit needs no lookup: the mesh's type and
    // colour are the same for every triangle. The counting variant keeps the reference's full
    // closest-hit walk and lookup: it prices the reference's work.
    const bool anyHit = !COUNT && firstHit;
    if (COUNT) cnt.seg++;
    // the analytic winner's t, id and object-space normal; its other attributes are resolved after
    // the walk, and only if the mesh does not win (meshHit sets them all): fewer values live across
    // the walk, same results
    f3 sn;
    PT_SEC(cnt, 4);
    analyticNearest<PROG>(a, rayO, rayD, h, sn);
    PT_SEC(cnt, 1);
    if (!kHasMesh<PROG>) { analyticAttributes<PROG>(a, h, sn); PT_SEC(cnt, 3); return; }

    // ---- BVH walk (js/GLTFModelPathTracing_FragmentShader.js:201-298), pt_device.h
    f3 O = mul(a.model, rayO, 1.0f), D = mul(a.model, rayD, 0.0f);
    f3 inv = mk(grcp(D.x), grcp(D.y), grcp(D.z));
    const bool dbl = (!a.uses_albedo && a.model_mat == TRANSPARENT);
    BvhResult br = { 0.0f, 0.0f, 0.0f, false, 1u, 0u, 0u };
    MegaStack<LS, kStackLdsOf<PROG>, kScratchOf<PROG>> st{ (lds_float2*)lds, lane_slot, (glb_float2*)a.spill, deep, a.spill_stride };
    if (kPairs<PROG>) {   // the root's box from the kernel arguments (the same floats as texels 0-1)
        const float* rb = a.bvh_root_box;
        const float rootT = box(mk(rb[0], rb[1], rb[2]), mk(rb[3], rb[4], rb[5]), O, inv);
        auto walk = [&]() {
            if (kTrail<PROG>) bvhWalkTrail<kRingOf<PROG>>(a, O, D, inv, dbl, rootT, h.t, (lds_float2*)lds, LS, lane_slot, br);
            else bvhWalkPairs(a, O, D, inv, dbl, rootT, h.t, st, br, anyHit);
        };
#ifdef PT_SECPROF
        if (cnt.sec) {
            const int ln_ = __lane_id();
            if (ln_ == __builtin_amdgcn_readfirstlane(ln_)) cnt.sec[9] = 0;
            walk();
            atomicMax(&cnt.sec[9], (unsigned long long)br.steps);
            cnt.lane_steps += br.steps;
            if (ln_ == __builtin_amdgcn_readfirstlane(ln_)) cnt.sec[10] += cnt.sec[9];
        } else
#endif
        walk();
    } else {
        float4 c0 = fetch32(a.aabb, a.aabb_texels, 0.0f), c1 = fetch32(a.aabb, a.aabb_texels, 1.0f);
        const float rootT = box(mk(c0.y, c0.z, c0.w), mk(c1.y, c1.z, c1.w), O, inv);
        bvhWalkRef(a, O, D, inv, dbl, c0, c1, rootT, h.t, st, br);
    }
    if (COUNT) { cnt.node += br.nodes; cnt.leaf += br.leaves; cnt.ovf += br.ovf; }
#ifdef PT_SECPROF
    if (COUNT) { cnt.sget += st.n_get; cnt.sget_slab += st.n_get_slab + br.restarts; cnt.sput += st.n_put; cnt.sput_slab += st.n_put_slab; }
    br.ws.flush(a.walk_stat, cnt.bounce++);
#endif
    PT_SEC(cnt, 2);
    if (br.lookup && anyHit) {   // the mesh occludes: what shadeStep reads of a mesh hit, no lookup
        h.normal = mk(0.0f, 0.0f, 1.0f);
        h.type = a.uses_albedo ? PBR_MATERIAL : a.model_mat;
        h.color = mk(1.0f, 1.0f, 1.0f);
        h.id = meshObjectId<PROG>(a);
    } else if (br.lookup) meshHit<PROG, COUNT>(a, br.triID, br.triU, br.triV, h, cnt);
    else analyticAttributes<PROG>(a, h, sn);
    PT_SEC(cnt, 3);
}

// One iteration of CalculateRadiance's loop: SceneIntersect, then the shading step
template <int PROG, bool COUNT, int LS, class G>
PT_D bool bounceStep(const TraceArgs& a, Path& p, PState& s, G& g, f3& accum, float2* lds, unsigned lane_slot,
                     unsigned deep, Cnt& cnt)
{
    Hit h;
    // segments that read only whether their hit is the light, nothing, or something else:
    //  * a shadow ray (the GLSL's sampleLight) ends its path at whatever it hits: `if (sampleLight)
    //    return false` comes before any use of the hit's normal, uv or material maps, and the G-buffer
    //    is written only at bounce 0, or at bounce 1 after METAL, which never samples the light;
    //  * the sixth segment of a path whose mesh is DIFFUSE, METAL or glass without PBR maps: its
    //    shading only updates state that ends with the path (mask, direction, counters) and, for glass,
    //    the sharpness from the path's counters alone - a clear coat's depends on the Fresnel term of
    //    the hit's normal, and a PBR hit reads its maps. Not in the textured variants (their PBR meshes
    //    never qualify, and the test alone costs the helmet 1 %).
    // (profiles/r04k_envmx_anyhit.txt, r04q_envmx_anyhit_last.txt)
    const bool lastOk = !kHasTex<PROG> && !a.uses_albedo &&
                        (a.model_mat == DIFFUSE || a.model_mat == METAL || a.model_mat == TRANSPARENT);
    sceneIntersect<PROG, COUNT, LS>(a, p.ro, p.rd, h, lds, lane_slot, deep, cnt, s.sampleLight || (s.bounce == 5 && lastOk));
    return shadeStep<PROG, COUNT, G>(a, p, s, g, accum, h, cnt);
}

// ------------------------------------------------------------------------------ late-bounce compaction
// A path's state between two bounces as a 64-B record (pt_cont): ray, throughput, rng / blue-noise state
// (whose bits 24-30 carry the G-buffer sharpness and id, pt_program.h GOutLds), the bounce counters and
// flags. The radiance so far is not stored: CalculateRadiance only ever assigns it when the path ends.
// The G-buffer's normal, colour and id are final from bounce 2 on (the GLSL writes them at bounces 0 and 1).
PT_D void contStore(const TraceArgs& a, unsigned slot, const Path& p, const PState& s)
{
    const unsigned bits = ((unsigned)s.diffuseCount & 0xffu) | (((unsigned)s.hitType & 0xffu) << 8) |
                          (((unsigned)s.bounce & 0xffu) << 16) | (s.coat ? 1u << 24 : 0u) |
                          (s.specular ? 1u << 25 : 0u) | (s.sampleLight ? 1u << 26 : 0u);
    float4* r = a.cont_rec + 4ull * slot;
    r[0] = make_float4(p.ro.x, p.ro.y, p.ro.z, p.rd.x);
    r[1] = make_float4(p.rd.y, p.rd.z, s.mask.x, s.mask.y);
    r[2] = make_float4(s.mask.z, s.roughness, __uint_as_float(p.s0), __uint_as_float(p.s1));
    r[3] = make_float4(__uint_as_float(p.bn), __uint_as_float(bits), 0.0f, 0.0f);
}
PT_D void contLoad(const TraceArgs& a, unsigned slot, Path& p, PState& s)
{
    const float4* r = a.cont_rec + 4ull * slot;
    const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
    p.ro = mk(r0.x, r0.y, r0.z); p.rd = mk(r0.w, r1.x, r1.y);
    s.mask = mk(r1.z, r1.w, r2.x); s.roughness = r2.y;
    p.s0 = __float_as_uint(r2.z); p.s1 = __float_as_uint(r2.w); p.bn = __float_as_uint(r3.x);
    const unsigned bits = __float_as_uint(r3.y);
    s.diffuseCount = (int)(bits & 0xffu);
    s.hitType = (int)(signed char)((bits >> 8) & 0xffu);
    s.bounce = (int)((bits >> 16) & 0xffu);
    s.coat = (bits >> 24) & 1u; s.specular = (bits >> 25) & 1u; s.sampleLight = (bits >> 26) & 1u;
}
// the G-buffer of a continued path: only the sharpness can still change, in the same bits of Path::bn
// as pt_trace keeps it (GOutLds)
struct GBits {
    static constexpr bool kColById = false;
    uint32_t* bn;
    PT_D void clear() {}
    PT_D void pinCol(f3) {}
    PT_D void setNrm(f3) {}
    PT_D void setCol(f3) {}
    PT_D void setId(float) {}
    PT_D float id() const { return 0.0f; }
    PT_D void setSharp(float v)
    {
        const unsigned code = v == 1.01f ? 1u : v == -1.0f ? 2u : 0u;
        *bn = (*bn & ~(3u << 24)) | (code << 24);
    }
    PT_D float sharp() const
    {
        const unsigned code = (*bn >> 24) & 3u;
        return code == 1u ? 1.01f : code == 2u ? -1.0f : 0.0f;
    }
};

// (experiment, PT_CONT_SORT) a stored record's ray key - whether the ray samples the light (the any-hit
// walk), the origin's cell in a 4x4x4 grid over the model's box (Morton order), the direction's octant -
// and its rank among the key's records: the lanes of one key found by a ballot per distinct key, then one
// atomic per key (all in one instruction) on the key's total. pt_cont_scatter places the records by them.
PT_D void contRank(const TraceArgs& a, int slot, const Path& p, const PState& s, bool inside)
{
    unsigned key = 0u;
    if (inside) {
        const float* rb = a.bvh_root_box;
        const f3 o = mul(a.model, p.ro, 1.0f);
        const unsigned gb = a.cont_grid_bits;
        const int top = (1 << gb) - 1;
        const unsigned cx = (unsigned)min(top, max(0, (int)((o.x - rb[0]) * a.cont_cell[0])));
        const unsigned cy = (unsigned)min(top, max(0, (int)((o.y - rb[1]) * a.cont_cell[1])));
        const unsigned cz = (unsigned)min(top, max(0, (int)((o.z - rb[2]) * a.cont_cell[2])));
        auto spread = [](unsigned v) { return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4); };   // bits 0-2 -> 0, 3, 6
        const unsigned cell = spread(cx) | (spread(cy) << 1) | (spread(cz) << 2);
        const unsigned oct = (p.rd.x < 0.0f ? 1u : 0u) | (p.rd.y < 0.0f ? 2u : 0u) | (p.rd.z < 0.0f ? 4u : 0u);
        const unsigned lt = s.sampleLight ? 1u : 0u;
        if (a.cont_key_mode == 3u) {   // 24 directions: the major axis and its sign (cube face), the quadrant
            const float ax = fabsf(p.rd.x), ay = fabsf(p.rd.y), az = fabsf(p.rd.z);
            const unsigned face = ax >= ay && ax >= az ? 0u : ay >= az ? 1u : 2u;
            const float m = face == 0u ? p.rd.x : face == 1u ? p.rd.y : p.rd.z;
            const float u = face == 0u ? p.rd.y : p.rd.x, v = face == 2u ? p.rd.y : p.rd.z;
            const unsigned dir = ((face * 2u + (m < 0.0f ? 1u : 0u)) << 2) | (u < 0.0f ? 1u : 0u) | (v < 0.0f ? 2u : 0u);
            key = (lt << (5u + 3u * gb)) | (cell << 5) | dir;
        } else
        key = a.cont_key_mode == 1u ? (lt << (3u + 3u * gb)) | (oct << (3u * gb)) | cell   // octant-major
            : a.cont_key_mode == 2u ? (cell << 3) | oct                                   // no light flag
            : a.cont_key_mode == 4u   // the paths with more bounces left first (longest first), then as mode 0
                ? (lt << (4u + 3u * gb)) | (((unsigned)s.bounce > a.cont_bounce ? 1u : 0u) << (3u + 3u * gb)) | (cell << 3) | oct
            : (lt << (3u + 3u * gb)) | (cell << 3) | oct;
    }
    unsigned long long todo = __ballot(inside), peers = 0ull;
    while (todo) {   // (wave-uniform)
        const int lead = __ffsll((long long)todo) - 1;
        const unsigned k = __shfl(key, lead, 64);
        const bool mine = inside && key == k;
        const unsigned long long m = __ballot(mine);
        if (mine) peers = m;
        todo &= ~m;
    }
    const int leader = inside ? __ffsll((long long)peers) - 1 : (int)__lane_id();
    unsigned base = 0u;
    if (inside && (int)__lane_id() == leader) base = atomicAdd(&a.cont_bins[key], (unsigned)__popcll(peers));
    base = __shfl(base, leader, 64);
    if (inside) {
        a.cont_key[slot] = (unsigned short)key;
        a.cont_rank[slot] = base + (unsigned)__popcll(peers & ((1ull << __lane_id()) - 1ull));
    }
}

// CalculateRadiance's loop. With late-bounce compaction (a.cont_rec): after a bounce >= cont_bounce, when
// at most cont_lanes of the wave's lanes are still looping (all at the same bounce: a ballot, wave-uniform),
// they leave the loop together and store their paths for pt_cont; `slot` is then the record's index (-1:
// the path ended here, or a helper lane outside the target, whose path no pixel needs - the 2x2
// derivatives only read its G-buffer, final by then). Slots: one atomic per wave, a lane prefix (mbcnt)
// over the ballot of the storing lanes.
// CONT is a kernel variant of its own (pt_trace<PROG, false, true>): the check in the bounce loop costs the
// 8-wave variants at their 64-VGPR budget even where it never fires (dragon stand-in +14 %, r05g)
template <int PROG, bool COUNT, int LS, bool CONT, class G>
PT_D f3 radiance(const TraceArgs& a, Path& p, G& g, float2* lds, unsigned lane_slot, unsigned deep, Cnt& cnt,
                 bool inside, int& slot)
{
    PState s;
    pathBegin(s, g);
    f3 accum = mk(0, 0, 0);
#pragma unroll 1
    while (bounceStep<PROG, COUNT, LS, G>(a, p, s, g, accum, lds, lane_slot, deep, cnt)) {
        if (CONT && (unsigned)s.bounce >= a.cont_bounce && (unsigned)__popcll(__ballot(1)) <= a.cont_lanes) {
            const unsigned long long st = __ballot(inside);
            const int lead = __ffsll((long long)__ballot(1)) - 1;
            unsigned base = 0;
            if (__lane_id() == lead && st) base = atomicAdd(a.cont_count, (unsigned)__popcll(st));
            base = __shfl(base, lead, 64);
            if (inside) {
                slot = (int)(base + (unsigned)__popcll(st & ((1ull << __lane_id()) - 1ull)));
                contStore(a, (unsigned)slot, p, s);
            }
            if (a.cont_bins) contRank(a, slot, p, s, inside);
            break;
        }
    }
    return max3s(accum, 0.0f);
}

// what main() computes of pixel `pi` without the history (js/PathTracingCommon.js:1304-1349): the
// radiance r and the alpha flag from the G-buffer sharpness and the 2x2 edge test - the first three of
// the reference's five `currentPixel.a` assignments (:1339, :1347, :1349); pt_blend applies the two
// that read the history (:1352, :1355) and the blend itself (:1326-1337, :1357). Streamed once per
// frame: a non-temporal store, so that it displaces fewer BVH records in L2.
PT_D void radianceOut(const TraceArgs& a, long long pi, f3 r, float sharp, bool edge)
{
    float ca = 0.0f;
    if (edge) sharp = 1.01f;
    if (sharp == 1.01f) ca = 1.01f;
    if (sharp == -1.0f) ca = -1.0f;
    typedef float nt4 __attribute__((ext_vector_type(4)));
    const nt4 o = { r.x, r.y, r.z, ca };
    __builtin_nontemporal_store(o, (nt4*)&a.rad[pi]);
}

PT_D float xorq(float v, int m) { return __shfl_xor(v, m, 64); }

// longest-first dispatch: wave durations (shader clock) in 8 log-scale buckets per octave (pt_order_build)
constexpr int kCostBuckets = 128;

// One-wave workgroups: every 8x8 wave tile is its own workgroup, so a wave that finishes frees its
// LDS (stack + G-buffer, 5 KB) at once, instead of holding a 4-wave workgroup's share until the
// slowest of the four (sky next to mesh) is done - LDS is what caps residency.
constexpr int kTraceBlock = 64;
constexpr int kTraceSub = 4;   // workgroups per 16x16 tile

// Which pixel a lane of pt_trace shades: the 8x8 wave tile of this wave inside its 16x16 tile
// (grid = tiles_x * kTraceSub x bands). Launch slots come in runs of 32 workgroups = 8 tiles x 4
// quadrants, quadrant-major: the quadrants of one tile are workgroups 8 apart, which the dispatcher
// deals to the same XCD (one L2), while the runs' tiles still go round-robin over the XCDs (a short
// last run keeps the map a bijection). The tiles come in longest-first order (the previous frame's
// costs, pt_order_build) when a.order is set, else row-major.
// Split tiles: the K = *a.split slowest tiles come first, each as 16 waves of 16 lanes (runs of 128
// workgroups = 8 tiles x 16 parts, again 8 apart per tile). A wave ends with its slowest lane of each
// bounce; a 4x4 block waits on fewer of them than an 8x8 one, so the kernel's critical path (the
// slowest tiles' waves, which start first and end last when a few tiles dominate, as the helmet's do)
// shortens. Which lane shades which pixel never changes what a pixel computes: same bits.
// False for the grid's padding.
struct TracePlace {
    int px, py, part;
    unsigned costIdx;
};
PT_D bool tracePlace(const TraceArgs& a, int lane, TracePlace& pl)
{
    int wave, part = -1;
    const unsigned tiles_x = gridDim.x / 4u, ntiles = a.ntiles;
    const unsigned K = (a.order && a.split) ? *a.split : 0u;   // chosen by pt_order_build
    const unsigned L = blockIdx.y * gridDim.x + blockIdx.x;
    unsigned slot;
    constexpr unsigned kPer = 4u * kSplitParts;   // workgroups per split tile
    if (L < kPer * K) {
        const unsigned g = L / (8u * kPer), r = L % (8u * kPer);
        slot = g * 8u + (r & 7u);
        wave = (int)((r >> 3) / kSplitParts);
        part = (int)((r >> 3) % kSplitParts);
    } else {
        const unsigned L2 = L - kPer * K;
        if (L2 >= 4u * (ntiles - K)) return false;
        const unsigned g = L2 >> 5, r = L2 & 31u;
        const unsigned T = min(8u, ntiles - K - g * 8u);
        slot = K + g * 8u + r % T;
        wave = (int)(r / T);
    }
    unsigned rank = slot;   // the slot's place in the longest-first order
    if (a.order_zig == 1u && slot >= K) {   // runs of 8 (one tile per XCD): from the top and the bottom in turn
        const unsigned j = slot - K, m = ntiles - K, g = j >> 3, t = (g >> 1) * 8u + (j & 7u);
        rank = K + ((g & 1u) ? m - 1u - t : t);
    }
    // (experiment, PT_XCD_BLOCKED with PT_LPT=0: XCD j = slot % 8 takes the j-th eighth of the frame's tiles in
    // row-major order - each L2 sees one contiguous strip of the frame, whatever its cost)
    const unsigned tile = a.order ? a.order[rank]
                                  : (a.order_zig == 2u && (ntiles & 7u) == 0u) ? (slot & 7u) * (ntiles >> 3) + (slot >> 3) : slot;
    if (rank < a.prio_tiles) __builtin_amdgcn_s_setprio(3);   // the critical path: issue first
    const int tx = (int)(tile % tiles_x);
    const unsigned bY = tile / tiles_x;
    // lane bits (x0, y0, x1, x2, y1, y2) of an 8x8 block, or (x0, y0, x1, y1) of a split tile's 4x4
    int lx, ly;
    if (part < 0) { lx = (lane & 1) | ((lane >> 1) & 6); ly = ((lane >> 1) & 1) | ((lane >> 3) & 6); }
    else {
        lx = (part & 1) * 4 + ((lane & 1) | ((lane >> 1) & 2));
        ly = (part >> 1) * 4 + (((lane >> 1) & 1) | ((lane >> 2) & 2));
    }
    const int band = (int)bY * a.num_parts + a.part;            // global 16-row band of this block
    pl.px = tx * kTile + (wave & 1) * 8 + lx;
    pl.py = band * kTile + (wave >> 1) * 8 + ly;
    pl.part = part;
    pl.costIdx = tile * 4u + (unsigned)wave;
    return true;
}

template <int PROG, bool COUNT, bool CONT>
__global__ __launch_bounds__(kTraceBlock, kMinWaves<PROG>) void pt_trace(TraceArgs a)
{
    static_assert(!CONT || (kHasMesh<PROG> && !COUNT), "late-bounce compaction: mesh programs, timed kernels");
    // one LDS array: the stack levels (+ the scratch level, kScratchOf) or the trail walk's ring, then
    // the G-buffer's LDS fields (none in some variants: no zero-length array)
    __shared__ float2 lds_stack[kWalkSlotsOf<PROG> * kTraceBlock + (kGoutLdsOf<PROG> * kTraceBlock + 1) / 2];
    float* const lds_gout = (float*)(lds_stack + kWalkSlotsOf<PROG> * kTraceBlock);
    const unsigned tid = threadIdx.x;
    const int lane = tid & 63;
    const unsigned long long t_start = clock64();
#ifdef PT_SECPROF
    const unsigned long long w0_ = wall_clock64();
#endif
    TracePlace pl;
    if (!tracePlace(a, lane, pl)) return;   // the grid's padding
    const int px = pl.px, py = pl.py;
    // stack levels >= kStackLds: a global slab [level][lane of the grid] (a private array would be
    // scratch, which the runtime reserves for every resident wave)
    const unsigned deep = (blockIdx.y * gridDim.x + blockIdx.x) * kTraceBlock + tid;

    // lanes whose whole 2x2 quad lies beyond the (even-rounded) target do no work; quad helpers
    // that only complete a quad at an odd edge are shaded like GL helper invocations
    const bool active = px < ((a.width + 1) & ~1) && py < ((a.height + 1) & ~1) && (pl.part < 0 || lane < (int)(64u / kSplitParts));
    Cnt cnt = { 0, 0, 0, 0, 0, 0, 0 };
#ifdef PT_SECPROF
    __shared__ unsigned long long lds_sec[16];
    if (tid < 16) lds_sec[tid] = tid == 8 ? clock64() : 0ull;
    cnt.sec = lds_sec;
    cnt.lane_steps = 0;
    cnt.sget = cnt.sget_slab = cnt.sput = cnt.sput_slab = 0;
    cnt.bounce = 0;
#endif
    // G-buffer fields beyond the LDS ones: 6 - kGoutLdsOf floats per lane after the slab's stack
    // levels, [field][lane] (pt_capi.cpp spill_reserve)
    glb_float* const gx = kGoutLdsOf<PROG> < 6
        ? (glb_float*)(a.spill + (size_t)(kStackLevels - kStackLdsMin) * a.spill_stride)
        : nullptr;
    Path p;
    p.bn = 0u;
    GOutLds<kTraceBlock, kGoutLdsOf<PROG>> gl{ (lds_float*)lds_gout, tid, gx, deep, a.spill_stride, &p.bn };
    gl.clear();   // pinned: the `out` parameters of CalculateRadiance start at 0 (also lanes without a path)
    f3 r = mk(0, 0, 0);
    int slot = -1;   // late-bounce compaction: this lane's path record for pt_cont
    if (active) {
        cameraRay(a, px, py, p);
        PT_SEC(cnt, 0);
        r = radiance<PROG, COUNT, kTraceBlock, CONT>(a, p, gl, lds_stack, tid, deep, cnt, px < a.width && py < a.height, slot);
    }
    PT_SEC(cnt, 4);
    const GOut g = gl.load([&](float id) {
        f3 c = mk(0.0f, 0.0f, 0.0f);
        int t;
        objectMaterial<PROG>(a, (int)id, c, t);
        return c;
    });

    // ---- 2x2 fine derivatives (js/PathTracingCommon.js:1306-1320): partner lanes ^1 (x) and ^2 (y)
    const bool xodd = lane & 1, yodd = lane & 2;
    auto ddx = [&](float v) { float o = xorq(v, 1); return xodd ? v - o : o - v; };
    auto ddy = [&](float v) { float o = xorq(v, 2); return yodd ? v - o : o - v; };
    float dNx = fabsf(ddx(g.nrm.x)) + fabsf(ddy(g.nrm.x));
    float dNy = fabsf(ddx(g.nrm.y)) + fabsf(ddy(g.nrm.y));
    float dNz = fabsf(ddx(g.nrm.z)) + fabsf(ddy(g.nrm.z));
    float normalDiff = gsmoothstep(0.2f, 0.6f, dNx) + gsmoothstep(0.2f, 0.6f, dNy) + gsmoothstep(0.2f, 0.6f, dNz);
    float dObj = fabsf(ddx(g.id)) > 0.0f ? 1.0f : 0.0f;
    dObj += fabsf(ddy(g.id)) > 0.0f ? 1.0f : 0.0f;
    float objectDiff = gsmoothstep(0.0f, 0.5f, dObj);
    f3 dcx = mk(ddx(g.col.x), ddx(g.col.y), ddx(g.col.z));
    f3 dcy = mk(ddy(g.col.x), ddy(g.col.y), ddy(g.col.z));
    float dCol = length(dcx) > 0.0f ? 1.0f : 0.0f;
    dCol += length(dcy) > 0.0f ? 1.0f : 0.0f;
    float colorDiff = gsmoothstep(0.0f, 0.5f, dCol);

#ifdef PT_SECPROF
    if (!COUNT && a.wave_log) {   // wave timeline in wall-clock ticks (100 MHz), one slot per workgroup
        atomicMax(&lds_sec[11], (unsigned long long)cnt.lane_steps);
        if (tid == 0) {
            const unsigned L = blockIdx.y * gridDim.x + blockIdx.x;
            unsigned long long* wl = a.wave_log + (size_t)kWaveLogSlots * L;
            wl[0] = w0_;
            wl[1] = wall_clock64();
            wl[2] = lds_sec[10];
            wl[3] = lds_sec[11];
            for (int k = 0; k < 8; k++) wl[4 + k] = lds_sec[k];   // section cycle sums (shader clock)
            wl[12] = __smid();   // the CU that ran the wave (XCC, SE, CU id bits): CU occupancy over time
        }
    }
    if (COUNT && active) {   // stack traffic: pops beyond the LDS levels, pushes beyond; node fetches, leaf tests
        atomicAdd(&a.counters[3], (unsigned long long)cnt.sget_slab);
        atomicAdd(&a.counters[4], (unsigned long long)cnt.node);
        atomicAdd(&a.counters[5], (unsigned long long)cnt.leaf);
        atomicAdd(&a.counters[6], 1ull);
    }
#endif
    if (COUNT && active && !PT_SECPROF_ON) {
        unsigned long long* C = a.counters;
        atomicAdd(&C[C_PATHS], 1ull);
        atomicAdd(&C[C_SEGMENTS], (unsigned long long)cnt.seg);
        atomicAdd(&C[C_NODE], (unsigned long long)cnt.node);
        atomicAdd(&C[C_LEAF], (unsigned long long)cnt.leaf);
        atomicAdd(&C[C_HIT], (unsigned long long)cnt.hit);
        atomicAdd(&C[C_RGBA8], (unsigned long long)(cnt.tap + 1));
        atomicAdd(&C[C_OVERFLOW], (unsigned long long)cnt.ovf);
        atomicAdd(&C[C_HDR], (unsigned long long)cnt.hdr);
    }
    if (a.cost && lane == 0) {   // this wave's duration, averaged with the tile's
        // history, for the next order (a split tile's four parts share their quadrant's entry)
        const unsigned long long dur = min(clock64() - t_start, 0xffffffffull);
        a.cost[pl.costIdx] = (unsigned)((dur + (unsigned long long)a.cost[pl.costIdx]) >> 1);
    }
    if (!active || px >= a.width || py >= a.height) return;   // quad helper outside the target, idle lane
    const bool edge = colorDiff >= 1.0f || normalDiff >= 1.0f || objectDiff >= 1.0f;
    const long long pi = (long long)py * a.width + px;
    if (CONT && slot >= 0) {   // the path continues in pt_cont, which writes the pixel's radiance
        a.cont_aux[slot] = (unsigned)pi | (edge ? 0x80000000u : 0u);
        return;
    }
    radianceOut(a, pi, r, g.sharp, edge);
}

// Late-bounce compaction, the second half: the paths pt_trace stored (cont_count[0] of them) run their
// remaining bounces packed into full waves. The one-wave workgroups take records from one queue (an
// atomic head, cont_count[1]) whenever at least cont_refill of their lanes are free (or all are), so no
// wave idles on an exhausted share while others still hold paths: a lane's path is one of the reference's per-pixel paths, resumed with exactly its state, so every
// pixel's bits are those of the uncompacted kernel. It runs after its draw's pt_trace on the same side
// stream, beside the next frame's pt_trace (frame overlap), so its own tail - a wave waits for the longest
// chain of dependent walks among its paths - is filled by that frame's waves.
template <int PROG>
__global__ __launch_bounds__(kTraceBlock, kMinWaves<PROG>) void pt_cont(TraceArgs a)
{
    __shared__ float2 lds_stack[kWalkSlotsOf<PROG> * kTraceBlock];
    const unsigned lane = threadIdx.x;
    const unsigned n = a.cont_count[0];
    unsigned* const head = a.cont_count + 1;   // the queue's next record (zeroed with the counter by pt_blend)
    bool more = true;                          // the queue may still hold records
    const unsigned deep = blockIdx.x * kTraceBlock + lane;
    const unsigned long long below = (1ull << lane) - 1ull;
    Cnt cnt = { 0, 0, 0, 0, 0, 0, 0 };
    Path p;
    p.bn = 0u;
    PState s;
    GBits g{ &p.bn };
    f3 accum = mk(0, 0, 0);
    unsigned slot = 0;
    bool alive = false;
    for (;;) {
        const unsigned long long dead = __ballot(!alive);
        const unsigned ndead = (unsigned)__popcll(dead);
        if (more && (ndead >= a.cont_refill || ndead == 64u)) {   // (wave-uniform: every lane is here)
            unsigned base = 0;
            if (lane == 0) base = atomicAdd(head, ndead);
            base = __shfl(base, 0, 64);
            if (base + ndead >= n) more = false;
            if (!alive) {
                const unsigned q = base + (unsigned)__popcll(dead & below);
                if (q < n) {
                    slot = a.cont_perm ? a.cont_perm[q] : q;
                    contLoad(a, slot, p, s);
                    accum = mk(0, 0, 0);
                    alive = true;
                }
            }
        }
        if (__ballot(alive) == 0ull) {
            if (!more) break;
            continue;
        }
        if (alive && !bounceStep<PROG, false, kTraceBlock>(a, p, s, g, accum, lds_stack, lane, deep, cnt)) {
            const unsigned aux = a.cont_aux[slot];
            radianceOut(a, (long long)(aux & 0x7fffffffu), max3s(accum, 0.0f), g.sharp(), (aux >> 31) != 0u);
            alive = false;
        }
    }
}

// ------------------------------------------------------------------------------ persistent paths
// pt_persist<PROG,COUNT>: the same per-pixel program with path regeneration. A wave owns a list
// of `per_wave` 8x8 wave tiles (the static kernel's lane order) and keeps its 64 lanes busy: when
// at least `refill` lanes have finished their path, they take the next pixels of the list and
// start their camera rays, so the wave no longer idles while its longest path runs out its six
// bounces. A finished path stores its G-buffer (objectNormal/ID/Color, pixelSharpness) and
// radiance by pixel; wf_finish then does the 2x2 derivatives and the accumulation.
template <int PROG, bool COUNT>
__global__ __launch_bounds__(kBlock, kMinWaves<PROG>) void pt_persist(TraceArgs a, WfBufs w, int tiles_x,
                                                                       unsigned n_wave_tiles, unsigned per_wave,
                                                                       unsigned refill)
{
    __shared__ float2 lds_stack[kWalkSlotsOf<PROG> * kBlock];   // stack levels (+ the scratch level, kScratchOf), or the trail walk's ring
    const unsigned tid = threadIdx.x;
    const unsigned lane = tid & 63u, wave = tid >> 6;
    const unsigned long long below = (1ull << lane) - 1ull;
    const unsigned wid = blockIdx.x * (kBlock / 64) + wave;
    unsigned next = wid * per_wave * 64u;
    const unsigned end = min(next + per_wave * 64u, n_wave_tiles * 64u);
    const unsigned deep = blockIdx.x * kBlock + tid;
    Cnt cnt = { 0, 0, 0, 0, 0, 0, 0 };
    unsigned paths = 0;
    Path p;
    PState s;
    GOut g;
    f3 accum = mk(0, 0, 0);
    unsigned pix = 0;
    bool alive = false;
    for (;;) {
        const unsigned long long dead = __ballot(!alive);
        const unsigned ndead = (unsigned)__popcll(dead);
        if (next < end && (ndead >= refill || ndead == 64u)) {
            if (!alive) {
                const unsigned q = next + (unsigned)__popcll(dead & below);
                if (q < end) {
                    const unsigned L = q >> 6, l = q & 63u;
                    const unsigned per_band = (unsigned)tiles_x * 4u;
                    const unsigned bl = L / per_band, rem = L - bl * per_band;
                    const unsigned tx = rem >> 2, sub = rem & 3u;
                    const int band = (int)bl * a.num_parts + a.part;
                    const int lx = (int)((l & 1u) | ((l >> 1) & 6u)), ly = (int)(((l >> 1) & 1u) | ((l >> 3) & 6u));
                    const int px = (int)tx * kTile + (int)(sub & 1u) * 8 + lx;
                    const int py = band * kTile + (int)(sub >> 1) * 8 + ly;
                    if (px < w.wq && py < w.hq) {
                        cameraRay(a, px, py, p);
                        pathBegin(s, g);
                        accum = mk(0, 0, 0);
                        pix = (unsigned)py * (unsigned)w.wq + (unsigned)px;
                        alive = true;
                        if (COUNT) paths++;
                    }
                }
            }
            next += ndead;
        }
        if (__ballot(alive) == 0ull) {
            if (next >= end) break;
            continue;
        }
        if (alive && !bounceStep<PROG, COUNT, kBlock>(a, p, s, g, accum, lds_stack, tid, deep, cnt)) {
            const f3 r = max3s(accum, 0.0f);
            w.gb0[pix] = make_float4(g.nrm.x, g.nrm.y, g.nrm.z, g.id);
            w.gb1[pix] = make_float4(g.col.x, g.col.y, g.col.z, g.sharp);
            w.rad[pix] = make_float4(r.x, r.y, r.z, 0.0f);
            alive = false;
        }
    }
    if (COUNT) {
        unsigned long long* C = a.counters;
        if (paths) atomicAdd(&C[C_PATHS], (unsigned long long)paths);
        atomicAdd(&C[C_SEGMENTS], (unsigned long long)cnt.seg);
        atomicAdd(&C[C_NODE], (unsigned long long)cnt.node);
        atomicAdd(&C[C_LEAF], (unsigned long long)cnt.leaf);
        atomicAdd(&C[C_HIT], (unsigned long long)cnt.hit);
        atomicAdd(&C[C_RGBA8], (unsigned long long)(cnt.tap + paths));
        atomicAdd(&C[C_OVERFLOW], (unsigned long long)cnt.ovf);
        atomicAdd(&C[C_HDR], (unsigned long long)cnt.hdr);
    }
}

} // namespace pt
