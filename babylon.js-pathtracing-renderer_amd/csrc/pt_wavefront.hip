// pt_wavefront.hip — the wavefront form of the path-tracing program (the default backend).
//
// The GLSL runs one fragment = one whole path (<= 6 segments); on a 64-lane wave that leaves most
// lanes idle: paths end at different bounces, branch into different materials, and a few lanes
// descend the BVH while the rest wait (megakernel PMC: ~28% VALU lane utilisation). Here the path
// is cut at its segment boundaries and every segment stage runs as its own kernel over a compacted
// queue of live paths:
//
//   wf_raygen            main() up to SetupScene (js/PathTracingCommon.js:1259-1292): camera ray,
//                        seeds, blue-noise texel; every pixel of the owned bands -> queue 0
//   per bounce b = 0..5:
//     wf_extend   <P>    SceneIntersect's analytic part (2 spheres, 6 quads) + the BVH root-box test;
//                        rays that enter the model's root box are appended to the BVH queue
//     wf_bvh      <P>    the BVH walk (js/GLTFModelPathTracing_FragmentShader.js:201-344) only for
//                        those rays: every lane of a wave traverses
//     wf_shade    <P>    one iteration of CalculateRadiance's loop body; surviving paths are appended
//                        to queue b+1 (wave ballots + block prefix + one atomic per block-iteration
//                        on the shard's counter: kShards counters, never one hot word)
//   wf_finish            main() after CalculateRadiance: 2x2-quad derivatives + accumulation
//
// Path state travels with the queue as four 16-byte SoA records (coalesced dwordx4 loads/stores);
// per-pixel outputs (G-buffer for the derivatives, radiance) are pixel-indexed. Every path performs
// exactly the GLSL's sequence of IEEE ops and random draws, only the schedule differs, so the
// result is bit-identical to the oracle and to the megakernel (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_device.h"
#include "pt_glsl.h"
#include "pt_program.h"

namespace pt {

enum Flag : unsigned {
    F_DIFFUSE_MASK = 7u,     // diffuseCount (0..6)
    F_COAT = 1u << 3,        // coatTypeIntersected
    F_SPECULAR = 1u << 4,    // bounceIsSpecular
    F_SAMPLE_LIGHT = 1u << 5,
    F_TYPE_SHIFT = 8,        // bits 8..15: previousIntersecType + 128 (after the PBR remap)
};
constexpr unsigned kTypeBias = 128u;


PT_D float u2f(unsigned u) { return __uint_as_float(u); }
PT_D unsigned f2u(float f) { return __float_as_uint(f); }

// block-level stream compaction: every thread of the block calls it (block-uniform loop); returns
// this lane's slot offset in the shard (valid only when `alive`). One atomic per call per block.
PT_D unsigned block_append(unsigned* counter, bool alive, unsigned* sh)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(alive);
    if (lane == 0) sh[wave] = (unsigned)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned total = sh[0] + sh[1] + sh[2] + sh[3];
        sh[4] = total ? atomicAdd(counter, total) : 0u;
    }
    __syncthreads();
    unsigned off = sh[4];
    for (int k = 0; k < wave; k++) off += sh[k];
    off += (unsigned)__popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();   // sh[] is reused by the next call
    return off;
}

// the shard a persistent block serves, its rank within the shard, and the shard's block count
struct ShardIter {
    unsigned s, k, nb;
    PT_D ShardIter() : s(blockIdx.x % kShards), k(blockIdx.x / kShards), nb(gridDim.x / kShards) {}
};

template <bool COUNT>
PT_D void count_add(const TraceArgs& a, int which, unsigned v)
{
    if (COUNT && v) atomicAdd(&a.counters[which], (unsigned long long)v);
}

// ============================================================================ raygen
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void wf_raygen(TraceArgs a, WfBufs w)
{
    const unsigned tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lx = (lane & 1) | ((lane >> 1) & 6);
    const int ly = ((lane >> 1) & 1) | ((lane >> 3) & 6);
    const int band = blockIdx.y * a.num_parts + a.part;
    const int px = blockIdx.x * kTile + (wave & 1) * 8 + lx;
    const int py = band * kTile + (wave >> 1) * 8 + ly;
    const bool active = px < w.wq && py < w.hq;
    Path p;
    p.s0 = p.s1 = 0;
    p.ro = p.rd = mk(0, 0, 0);
    unsigned bnb = 0, pix = 0;
    if (active) {
        pix = (unsigned)py * (unsigned)w.wq + (unsigned)px;
        const float* m = a.cam.m;
        f3 camRight = mk(m[0], m[1], m[2]), camUp = mk(m[4], m[5], m[6]), camFwd = mk(m[8], m[9], m[10]);
        f3 camPos = mk(m[12], m[13], m[14]);
        float fcx = (float)px + 0.5f, fcy = (float)py + 0.5f;
        p.s0 = (uint32_t)a.frame * (uint32_t)fcx;
        p.s1 = (uint32_t)(a.frame + 1.0f) * (uint32_t)fcy;
        int bx = (int)gmod(fcx + floorf(a.rnd[0] * 256.0f), 256.0f);
        int by = (int)gmod(fcy + floorf(a.rnd[1] * 256.0f), 256.0f);
        if (bx < a.bluenoise.w && by < a.bluenoise.h) {
            uchar4 b = a.bluenoise.p[by * a.bluenoise.w + bx];
            bnb = (unsigned)b.x | ((unsigned)b.y << 8);
        }
        float ox = tentFilter(rng(p));
        float oy = tentFilter(rng(p));
        float ppx = ((fcx + ox) / a.res[0]) * 2.0f - 1.0f;
        float ppy = ((fcy + oy) / a.res[1]) * 2.0f - 1.0f;
        f3 rayDir = normalize((camRight * ppx) * a.ulen + (camUp * ppy) * a.vlen + camFwd);
        f3 focal = rayDir * a.focus;
        float ang = rng(p) * kTwoPi;
        float rad = rng(p) * a.aperture;
        float sn, cs;
        gsincos(ang, sn, cs);
        f3 apert = (camRight * cs + camUp * sn) * gsqrt(rad);
        p.rd = normalize(focal - apert);
        p.ro = camPos + apert;
        // per-pixel outputs start at the `out` parameters' pinned zero
        w.gb0[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        w.gb1[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        w.rad[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    // tile t -> shard t % kShards, deterministic slot (no atomics); lanes outside the frame are holes
    const unsigned t = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned s = t % kShards;
    const unsigned slot = s * w.shard_cap + (t / kShards) * kBlock + tid;
    if (tid == 0) atomicAdd(&w.cnt[s], (unsigned)kBlock);
    w.qA[0][slot] = make_float4(p.ro.x, p.ro.y, p.ro.z, u2f(active ? pix : kHole));
    if (active) {
        w.qB[0][slot] = make_float4(p.rd.x, p.rd.y, p.rd.z, -1.0f);   // blueNoise counter starts at -1
        w.qC[0][slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);           // mask, roughness
        w.qD[0][slot] = make_float4(u2f(p.s0), u2f(p.s1), u2f(F_SPECULAR | ((kTypeBias - 100u) << F_TYPE_SHIFT)), u2f(bnb));
    }
    if (COUNT && active) { count_add<true>(a, C_PATHS, 1); count_add<true>(a, C_RGBA8, 1); }
}

// ============================================================================ extend (analytic part)
template <int PROG, bool COUNT>
__global__ __launch_bounds__(kBlock) void wf_extend(TraceArgs a, WfBufs w, int b)
{
    __shared__ unsigned sh[8];
    const ShardIter it;
    const unsigned n = w.cnt[b * kShards + it.s];
    const unsigned shard0 = it.s * w.shard_cap;
    const int q = b & 1;
    for (unsigned base = it.k * kBlock; base < n; base += it.nb * kBlock) {
        const unsigned i = shard0 + base + threadIdx.x;
        bool toBvh = false;
        if (base + threadIdx.x < n) {
            float4 A = w.qA[q][i];
            if (f2u(A.w) != kHole) {
                float4 B = w.qB[q][i];
                f3 ro = mk(A.x, A.y, A.z), rd = mk(B.x, B.y, B.z);
                Hit h;
                analyticIntersect<PROG>(a, ro, rd, h);
                const float t = h.t;
                const int id = h.id;
                const f3 hn = id >= 0 ? h.normal : mk(0, 0, 0);
                if (COUNT) count_add<true>(a, C_SEGMENTS, 1);
                if (kHasMesh<PROG>) {
                    f3 O = mul(a.model, ro, 1.0f), D = mul(a.model, rd, 0.0f);
                    f3 inv = mk(grcp(D.x), grcp(D.y), grcp(D.z));
                    float4 c0 = fetch32(a.aabb, a.aabb_texels, 0.0f), c1 = fetch32(a.aabb, a.aabb_texels, 1.0f);
                    if (COUNT) count_add<true>(a, C_NODE, 1);
                    float tRoot = box(mk(c0.y, c0.z, c0.w), mk(c1.y, c1.z, c1.w), O, inv);
                    toBvh = tRoot < t;
                }
                w.hit0[i] = make_float4(t, u2f((unsigned)id), 0.0f, 0.0f);
                w.hit1[i] = make_float4(hn.x, hn.y, hn.z, 0.0f);
            }
        }
        if (kHasMesh<PROG>) {
            const unsigned off = block_append(&w.bcnt[b * kShards + it.s], toBvh, sh);
            if (toBvh) w.bvhq[shard0 + off] = i;
        }
    }
}

// ============================================================================ BVH walk
// stack levels >= kStackLds live in a global slab indexed [level][persistent lane]
struct WfStack {
    lds_float2* lds;
    unsigned slot;
    glb_float2* deep;
    size_t dstride;
    PT_D float2 get(int si) const
    {
        vf2 e;
        if (si < kStackLds) e = lds[si * kBlock + slot];
        else e = deep[(si - kStackLds) * dstride];
        return make_float2(e.x, e.y);
    }
    PT_D void put(int si, float2 e)
    {
        const vf2 v = { e.x, e.y };
        if (si < kStackLds) lds[si * kBlock + slot] = v;
        else deep[(si - kStackLds) * dstride] = v;
    }
    PT_D float2 pop(int si, float2 sentinel) const { return si < kStackLevels ? get(si) : sentinel; }
    PT_D bool push(int si, float2 e)
    {
        if (si >= kStackLevels) return false;
        put(si, e);
        return true;
    }
};

template <int PROG, bool COUNT>
__global__ __launch_bounds__(kBlock, 4) void wf_bvh(TraceArgs a, WfBufs w, int b)
{
    __shared__ float2 lds[(kTrail<PROG> ? kRingOf<PROG> : kStackLds) * kBlock];   // stack levels, or the trail walk's ring
    const ShardIter it;
    const unsigned n = w.bcnt[b * kShards + it.s];
    const unsigned shard0 = it.s * w.shard_cap;
    const int q = b & 1;
    const unsigned tid = threadIdx.x;
    // stack levels beyond LDS: a global slab indexed [level][persistent lane] (no scratch: a
    // scratch-using kernel throttles how many waves the CP keeps resident)
    float2* deep = w.spill + (size_t)blockIdx.x * kBlock + tid;
    const size_t dstride = (size_t)gridDim.x * kBlock;
    for (unsigned base = it.k * kBlock; base < n; base += it.nb * kBlock) {
        const unsigned j = base + tid;
        if (j >= n) continue;
        const unsigned i = w.bvhq[shard0 + j];
        float4 A = w.qA[q][i], B = w.qB[q][i];
        float hitT = w.hit0[i].x;
        f3 ro = mk(A.x, A.y, A.z), rd = mk(B.x, B.y, B.z);
        f3 O = mul(a.model, ro, 1.0f), D = mul(a.model, rd, 0.0f);
        f3 inv = mk(grcp(D.x), grcp(D.y), grcp(D.z));
        const bool dbl = (!a.uses_albedo && a.model_mat == TRANSPARENT);
        // the root was fetched and tested by wf_extend (and counted there); its box is hit
        float4 c0 = fetch32(a.aabb, a.aabb_texels, 0.0f), c1 = fetch32(a.aabb, a.aabb_texels, 1.0f);
        float rootT = box(mk(c0.y, c0.z, c0.w), mk(c1.y, c1.z, c1.w), O, inv);
        BvhResult br = { 0.0f, 0.0f, 0.0f, false, 0u, 0u, 0u };
        WfStack st{ (lds_float2*)lds, tid, (glb_float2*)deep, dstride };
        if (kTrail<PROG>) bvhWalkTrail<kRingOf<PROG>>(a, O, D, inv, dbl, rootT, hitT, (lds_float2*)lds, kBlock, tid, br);
        else if (kPairs<PROG>) bvhWalkPairs(a, O, D, inv, dbl, rootT, hitT, st, br);
        else bvhWalkRef(a, O, D, inv, dbl, c0, c1, rootT, hitT, st, br);
        const unsigned nodes = br.nodes, leaves = br.leaves, ovf = br.ovf;
        const bool lookup = br.lookup;
        const float triID = br.triID, triU = br.triU, triV = br.triV;
        unsigned taps = 0;
        if (lookup) {
            float4 v2 = fetch32(a.tri, a.tri_texels, triID + 2.0f), v3 = fetch32(a.tri, a.tri_texels, triID + 3.0f),
                   v4 = fetch32(a.tri, a.tri_texels, triID + 4.0f), v5 = fetch32(a.tri, a.tri_texels, triID + 5.0f);
            float triW = 1.0f - triU - triV;
            f3 nn = normalize(mk(v2.y, v2.z, v2.w) * triW + mk(v3.x, v3.y, v3.z) * triU + mk(v3.w, v4.x, v4.y) * triV);
            float hu = triW * v4.z + triU * v5.x + triV * v5.z;
            float hv = triW * v4.w + triU * v5.y + triV * v5.w;
            if (kHasTex<PROG> && a.uses_bump) {   // perturbNormal (js/GLTFModelPathTracing_FragmentShader.js:72-92)
                f3 S = onb_u(nn);
                f3 T = cross(nn, S);
                f3 N = normalize(nn);
                if (dot(cross(S, T), N) < 0.0f) { S = S * -1.0f; T = T * -1.0f; }
                float tx[4];
                texBilinear(a.bump, hu, hv, tx);
                taps += 4;
                f3 mN = normalize(mk(tx[0] * 2.0f - 1.0f, tx[1] * 2.0f - 1.0f, tx[2] * 2.0f - 1.0f));
                mN.x *= 1.0f; mN.y *= 1.0f;
                nn = normalize(S * mN.x + T * mN.y + N * mN.z);
            }
            f3 hn = normalize(mul3t(a.model, nn));
            w.hit0[i] = make_float4(hitT, u2f((unsigned)meshObjectId<PROG>(a)), hu, hv);
            w.hit1[i] = make_float4(hn.x, hn.y, hn.z, 0.0f);
        }
        if (COUNT) {
            count_add<true>(a, C_NODE, nodes);
            count_add<true>(a, C_LEAF, leaves);
            count_add<true>(a, C_HIT, lookup ? 1u : 0u);
            count_add<true>(a, C_RGBA8, taps);
            count_add<true>(a, C_OVERFLOW, ovf);
        }
    }
}

// ============================================================================ shade (one loop iteration)
// CalculateRadiance's G-buffer outputs go straight to the pixel's gb0 / gb1 records
struct GOutPix {
    static constexpr bool kColById = false;
    float4* gb0;
    float4* gb1;
    unsigned pix;
    PT_D void clear() {}
    PT_D void pinCol(f3) {}
    PT_D void setNrm(f3 v) { gb0[pix].x = v.x; gb0[pix].y = v.y; gb0[pix].z = v.z; }
    PT_D void setCol(f3 v) { gb1[pix].x = v.x; gb1[pix].y = v.y; gb1[pix].z = v.z; }
    PT_D void setId(float v) { gb0[pix].w = v; }
    PT_D void setSharp(float v) { gb1[pix].w = v; }
};

template <int PROG, bool COUNT>
__global__ __launch_bounds__(kBlock) void wf_shade(TraceArgs a, WfBufs w, int b)
{
    __shared__ unsigned sh[8];
    const ShardIter it;
    const unsigned n = w.cnt[b * kShards + it.s];
    const unsigned shard0 = it.s * w.shard_cap;
    const int q = b & 1, q2 = q ^ 1;
    for (unsigned base = it.k * kBlock; base < n; base += it.nb * kBlock) {
        const unsigned i = shard0 + base + threadIdx.x;
        bool alive = false;
        float4 oA, oB, oC, oD;
        const float4 A = base + threadIdx.x < n ? w.qA[q][i] : make_float4(0.0f, 0.0f, 0.0f, u2f(kHole));
        if (f2u(A.w) != kHole) {
            const float4 B = w.qB[q][i], C = w.qC[q][i], D = w.qD[q][i];
            const float4 H0 = w.hit0[i], H1 = w.hit1[i];
            const unsigned pix = f2u(A.w);
            Path p;
            p.ro = mk(A.x, A.y, A.z);
            p.rd = mk(B.x, B.y, B.z);
            p.s0 = f2u(D.x); p.s1 = f2u(D.y);
            const unsigned flags = f2u(D.z);
            p.bn = f2u(D.w) & 0xffffu;
            setPathCounter(p, B.w);
            PState s;
            s.mask = mk(C.x, C.y, C.z);
            s.roughness = C.w;
            s.diffuseCount = (int)(flags & F_DIFFUSE_MASK);
            s.hitType = (int)((flags >> F_TYPE_SHIFT) & 255u) - (int)kTypeBias;
            s.bounce = b;
            s.coat = flags & F_COAT; s.specular = flags & F_SPECULAR; s.sampleLight = flags & F_SAMPLE_LIGHT;
            // the hit record SceneIntersect would have returned (wf_extend + wf_bvh)
            Hit h;
            h.t = H0.x;
            h.id = (int)f2u(H0.y);
            h.u = H0.z; h.v = H0.w;
            h.normal = mk(H1.x, H1.y, H1.z);
            h.color = mk(0.0f, 0.0f, 0.0f);
            h.type = -100;
            objectMaterial<PROG>(a, h.id, h.color, h.type);
            GOutPix g{ w.gb0, w.gb1, pix };
            f3 accum = mk(0, 0, 0);
            Cnt cnt = { 0, 0, 0, 0, 0, 0, 0 };
            if (shadeStep<PROG, COUNT, GOutPix>(a, p, s, g, accum, h, cnt)) {
                alive = true;
                const unsigned nf = (unsigned)s.diffuseCount | (s.coat ? F_COAT : 0u) | (s.specular ? F_SPECULAR : 0u) |
                                    (s.sampleLight ? F_SAMPLE_LIGHT : 0u) |
                                    ((unsigned)(s.hitType + (int)kTypeBias) << F_TYPE_SHIFT);
                oA = make_float4(p.ro.x, p.ro.y, p.ro.z, A.w);
                oB = make_float4(p.rd.x, p.rd.y, p.rd.z, pathCounter(p));
                oC = make_float4(s.mask.x, s.mask.y, s.mask.z, s.roughness);
                oD = make_float4(u2f(p.s0), u2f(p.s1), u2f(nf), D.w);
            } else {
                const f3 r = max3s(accum, 0.0f);
                w.rad[pix] = make_float4(r.x, r.y, r.z, 0.0f);
            }
            if (COUNT) { count_add<true>(a, C_RGBA8, cnt.tap); count_add<true>(a, C_HDR, cnt.hdr); }
        }
        const unsigned slot = shard0 + block_append(&w.cnt[(b + 1) * kShards + it.s], alive, sh);
        if (alive) {
            w.qA[q2][slot] = oA;
            w.qB[q2][slot] = oB;
            w.qC[q2][slot] = oC;
            w.qD[q2][slot] = oD;
        }
    }
}

// ============================================================================ finish
__global__ __launch_bounds__(kBlock) void wf_finish(TraceArgs a, WfBufs w)
{
    const unsigned tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lx = (lane & 1) | ((lane >> 1) & 6);
    const int ly = ((lane >> 1) & 1) | ((lane >> 3) & 6);
    const int band = blockIdx.y * a.num_parts + a.part;
    const int px = blockIdx.x * kTile + (wave & 1) * 8 + lx;
    const int py = band * kTile + (wave >> 1) * 8 + ly;
    const bool active = px < w.wq && py < w.hq;
    float4 g0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), g1 = g0, r = g0;
    if (active) {
        const unsigned pix = (unsigned)py * (unsigned)w.wq + (unsigned)px;
        g0 = w.gb0[pix]; g1 = w.gb1[pix]; r = w.rad[pix];
    }
    const bool xodd = lane & 1, yodd = lane & 2;
    auto ddx = [&](float v) { float o = __shfl_xor(v, 1, 64); return xodd ? v - o : o - v; };
    auto ddy = [&](float v) { float o = __shfl_xor(v, 2, 64); return yodd ? v - o : o - v; };
    float dNx = fabsf(ddx(g0.x)) + fabsf(ddy(g0.x));
    float dNy = fabsf(ddx(g0.y)) + fabsf(ddy(g0.y));
    float dNz = fabsf(ddx(g0.z)) + fabsf(ddy(g0.z));
    float normalDiff = gsmoothstep(0.2f, 0.6f, dNx) + gsmoothstep(0.2f, 0.6f, dNy) + gsmoothstep(0.2f, 0.6f, dNz);
    float dObj = fabsf(ddx(g0.w)) > 0.0f ? 1.0f : 0.0f;
    dObj += fabsf(ddy(g0.w)) > 0.0f ? 1.0f : 0.0f;
    float objectDiff = gsmoothstep(0.0f, 0.5f, dObj);
    f3 dcx = mk(ddx(g1.x), ddx(g1.y), ddx(g1.z));
    f3 dcy = mk(ddy(g1.x), ddy(g1.y), ddy(g1.z));
    float dCol = length(dcx) > 0.0f ? 1.0f : 0.0f;
    dCol += length(dcy) > 0.0f ? 1.0f : 0.0f;
    float colorDiff = gsmoothstep(0.0f, 0.5f, dCol);
    if (px >= a.width || py >= a.height) return;
    const long long pi = (long long)py * a.width + px;
    float4 prev = a.prev[pi];
    float cr = r.x, cg = r.y, cb = r.z, ca;
    if (a.frame == 1.0f) prev = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    else if (a.moving) {
        prev.x *= 0.5f; prev.y *= 0.5f; prev.z *= 0.5f;
        cr *= 0.5f; cg *= 0.5f; cb *= 0.5f;
        prev.w = 0.0f;
    }
    ca = 0.0f;
    float sharp = g1.w;
    if (colorDiff >= 1.0f || normalDiff >= 1.0f || objectDiff >= 1.0f) sharp = 1.01f;
    if (sharp == 1.01f) ca = 1.01f;
    if (sharp == -1.0f) ca = -1.0f;
    if (prev.w == 1.01f) ca = 1.01f;
    if (prev.w == -1.0f) ca = 0.0f;
    a.out[pi] = make_float4(prev.x + cr, prev.y + cg, prev.z + cb, ca);
}

} // namespace pt

// ------------------------------------------------------------------------------ launcher
extern "C" hipError_t pt_launch_wavefront(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w,
                                          int tiles_x, int bands, int persist_blocks, hipStream_t s)
{
    using namespace pt;
    prog = resolveProgram(prog, a->uses_albedo || a->uses_bump, a->bvh_walk);
    dim3 tiles(tiles_x, bands), blk(kBlock);
    if (count) hipLaunchKernelGGL((wf_raygen<true>), tiles, blk, 0, s, *a, *w);
    else hipLaunchKernelGGL((wf_raygen<false>), tiles, blk, 0, s, *a, *w);
#define WF_BOUNCE(P, C)                                                                              \
    for (int b = 0; b < 6; b++) {                                                                    \
        hipLaunchKernelGGL((wf_extend<P, C>), dim3(persist_blocks), blk, 0, s, *a, *w, b);         \
        if (kHasMesh<P>) hipLaunchKernelGGL((wf_bvh<P, C>), dim3(persist_blocks), blk, 0, s, *a, *w, b); \
        hipLaunchKernelGGL((wf_shade<P, C>), dim3(persist_blocks), blk, 0, s, *a, *w, b);          \
    }
#define WF_CASE_T(P) case P: WF_BOUNCE(P, true) break;
#define WF_CASE_F(P) case P: WF_BOUNCE(P, false) break;
    if (count) {
        switch (prog) {
            PT_FOR_EACH_PROG(WF_CASE_T)
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (prog) {
            PT_FOR_EACH_PROG(WF_CASE_F)
        default: return hipErrorInvalidValue;
        }
    }
#undef WF_CASE_T
#undef WF_CASE_F
#undef WF_BOUNCE
    hipLaunchKernelGGL(wf_finish, tiles, blk, 0, s, *a, *w);
    return hipGetLastError();
}

extern "C" hipError_t pt_launch_finish(const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x, int bands, hipStream_t s)
{
    hipLaunchKernelGGL(pt::wf_finish, dim3(tiles_x, bands), dim3(pt::kBlock), 0, s, *a, *w);
    return hipGetLastError();
}
