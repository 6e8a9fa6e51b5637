// pt_device.h — device routines shared by the megakernel (pt_kernels.hip) and the wavefront
// kernels (pt_wavefront.hip): the reference's random / sampling / material / intersection helpers
// with the pinned GLSL semantics (pt_glsl.h). Each cites the GLSL it restates.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_glsl.h"

namespace pt {
using namespace ptg;

constexpr float kINF = 1000000.0f;   // #define INFINITY 1000000.0 (js/PathTracingCommon.js:329)
constexpr float kTwoPi = 6.28318530717958648f;

enum { PROG_CORNELL = 3, PROG_GLTF = 4, PROG_HDRI = 5, PROG_SKY = 6, PROG_QUADRIC = 7, PROG_SKYMESH = 8 };
// PROG_*_TEX: the mesh programs instantiated with their PBR / normal-map code (models with an
// albedo or bump texture); without +PROG_TEX those branches are compiled out.
enum { PROG_TEX = 100, PROG_GLTF_TEX = 104, PROG_HDRI_TEX = 105, PROG_SKYMESH_TEX = 108 };
// BVH walks (the program variant's thousands digit, chosen per draw by the host, pt_capi.cpp):
// +PROG_PAIRS the child-pair records (bvhWalkPairs) with the reference's short stack instead of the
// reference's texel pairs (bvhWalkRef); +PROG_TRAIL the same records without a stack beyond an LDS ring
// (bvhWalkTrail: the restart trail, PT_BVH_TRAIL)
enum { PROG_PAIRS = 1000, PROG_TRAIL = 2000 };   // = WALK_* (pt_args.h) x 1000
template <int P> constexpr int kBase = P % PROG_PAIRS;
template <int P> constexpr int kScene = kBase<P> % PROG_TEX;
// the programs whose SceneIntersect walks the glTF model's BVH: glTF, HDRI and the physical-sky
// composite (PROG_SKYMESH, DESIGN.md §1: the sky scene with the glTF model block appended)
template <int P> constexpr bool kHasMesh = kScene<P> == PROG_GLTF || kScene<P> == PROG_HDRI || kScene<P> == PROG_SKYMESH;
// the glTF CalculateRadiance (PBR decode, glossy METAL lobe): glTF and HDRI
template <int P> constexpr bool kIsGltf = kScene<P> == PROG_GLTF || kScene<P> == PROG_HDRI;
template <int P> constexpr bool kIsHdri = kScene<P> == PROG_HDRI;
template <int P> constexpr bool kHasTex = kBase<P> >= PROG_TEX;
// the physical-sky CalculateRadiance (js/PhysicalSkyModel_FragmentShader.js:119-379)
template <int P> constexpr bool kIsSky = kScene<P> == PROG_SKY || kScene<P> == PROG_SKYMESH;
template <int P> constexpr bool kIsQuadric = P == PROG_QUADRIC;
// hitObjectID layout: spheres 0-1 (quadric: shapes 0-11), then the quads, then the mesh
// (objectCount after the quads: 8 in the glTF scene, 6 in the HDRI scene and the sky composite)
template <int P> constexpr int kQuadId0 = kIsQuadric<P> ? 12 : 2;
template <int P> constexpr int kWalk = P / PROG_PAIRS;
template <int P> constexpr bool kPairs = P >= PROG_PAIRS;   // child-pair records (any walk but the reference's)
template <int P> constexpr bool kTrail = kWalk<P> == WALK_TRAIL;
// every instantiated program variant, by BVH walk (one translation unit each: pt_trace_walk*.hip)
#define PT_FOR_EACH_PROG_REF(X)                                                                                           \
    X(PROG_CORNELL) X(PROG_SKY) X(PROG_QUADRIC) X(PROG_GLTF) X(PROG_GLTF_TEX) X(PROG_HDRI) X(PROG_HDRI_TEX)           \
    X(PROG_SKYMESH) X(PROG_SKYMESH_TEX)
#define PT_FOR_EACH_MESH_PROG(X, W)                                                                                       \
    X(W + PROG_GLTF) X(W + PROG_GLTF_TEX) X(W + PROG_HDRI) X(W + PROG_HDRI_TEX) X(W + PROG_SKYMESH) X(W + PROG_SKYMESH_TEX)
#define PT_FOR_EACH_PROG_PAIRS(X) PT_FOR_EACH_MESH_PROG(X, PROG_PAIRS)
#define PT_FOR_EACH_PROG_TRAIL(X) PT_FOR_EACH_MESH_PROG(X, PROG_TRAIL)
#define PT_FOR_EACH_PROG(X) PT_FOR_EACH_PROG_REF(X) PT_FOR_EACH_PROG_PAIRS(X) PT_FOR_EACH_PROG_TRAIL(X)

// the kernel variant of a draw: the scene program, +PROG_TEX when the model carries albedo / bump
// maps, + the walk's thousands for the mesh programs
__host__ __device__ inline int resolveProgram(int prog, bool textured, int walk)
{
    if (prog != PROG_GLTF && prog != PROG_HDRI && prog != PROG_SKYMESH) return prog;
    return prog + (textured ? PROG_TEX : 0) + walk * PROG_PAIRS;
}
// Occupancy and LDS per variant (measured; the values are the tuned ones, edit them here
// for an A/B build):
// waves per SIMD the register allocator must leave room for (128 VGPRs -> 4, 64 -> 8): the
// texture-free child-pair walk at 8 (64 VGPRs, a small spill outside the walk loop; 4 % ahead of 6
// waves on the dragon stand-in, 7 waves behind both), the textured variants at 4 (1.3 % ahead of 3),
// the reference walk at 4 (it loses above)
constexpr int kMinWavesTex = 4, kMinWavesPairs = 8, kMinWavesRef = 4;
template <int P> constexpr int kMinWaves = kHasTex<P> ? kMinWavesTex : kPairs<P> ? kMinWavesPairs : kMinWavesRef;
// G-buffer fields in LDS (pt_program.h GOutLds: the normal and colour; the id and sharpness ride in a
// register): the 8-wave child-pair walks keep none of them there - the normal is stored once per path
// to memory and read once, the colour is recomputed from the bounce-0 object id - and have two LDS
// stack levels more in their place (10: dragon stand-in -1.6 %, bunny x16 -1.4 % against 8 levels with 4
// fields in LDS, profiles/r04e_envmx_gbuffer_levels.txt; sky + dragon 4K -2.7 % against all 6 fields
// and 7 levels, -2.1 % for the normal in LDS and 8 levels, profiles/r04aa_envmx_sky_gbuffer.txt)
constexpr int kGoutLdsGltf = 0, kGoutLdsSky = 0;
template <int P> constexpr bool kPairs8 = kPairs<P> && !kHasTex<P>;
template <int P> constexpr int kGoutLdsOf = !kPairs8<P> ? 6 : kIsGltf<P> ? kGoutLdsGltf
                                          : kScene<P> == PROG_SKYMESH ? kGoutLdsSky : 6;
// BVH stack levels in LDS per lane (the rest in the global slab): the 8-wave variants fill 20 floats
// per lane (160 KB per CU at 32 one-wave workgroups) with the G-buffer's LDS fields and the levels
// (2 floats each); the 4-wave variants keep 7
template <int P> constexpr int kStackLdsOf = kPairs8<P> ? (2 * kStackLdsPairs + 8 - kGoutLdsOf<P>) / 2 : kStackLds;
// the restart-trail walk's LDS ring (entries per lane): at 8 waves/SIMD the 80 B per lane (160 KB per
// CU) the stack walk's levels take - 10 entries for every 8-wave mesh scene (glTF, HDRI, sky + mesh),
// whose G-buffer lives in memory (the normal in the spill slab, the colour recomputed) for the trail
// walk as for the stack walk; at 4 waves/SIMD the textured variants have room for 14
template <int P> constexpr int kRingOf = kHasTex<P> ? 14 : kPairs8<P> ? (2 * kStackLdsPairs + 8 - kGoutLdsOf<P>) / 2 : 6;
// the stack walk's push form (pt_trace.h MegaStack::push): a scratch level and unmasked stores for
// the textured 4-wave variants (1 % faster there), masked stores into one more real level where LDS
// caps residency (the 8-wave variants: dragon stand-in +1.5 %, sky + dragon +2.2 %)
template <int P> constexpr bool kScratchOf = !kPairs8<P>;
// LDS float2 slots per lane a walk of program P needs: stack levels (+ the scratch level), or the ring
template <int P> constexpr int kWalkSlotsOf = kTrail<P> ? kRingOf<P> : kStackLdsOf<P> + (kScratchOf<P> ? 1 : 0);

typedef float vf2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) vf2 lds_float2;
typedef __attribute__((address_space(1))) vf2 glb_float2;

// ------------------------------------------------------------------------------ per-lane state
struct Path {
    uint32_t s0, s1;       // uvec2 seed (js/PathTracingCommon.js:500)
    // blueNoise_rand()'s state in one register: bits 0-7 / 8-15 = the blue-noise texel's r / g bytes
    // (randVec4.r / .g: channel = mod(counter, 2) only reaches those two), bits 16-22 = counter + 1
    // (the GLSL's float counter starts at -1.0 and only ever steps by 1.0, at most twice per bounce);
    // bits 23-31 carry pt_trace's packed G-buffer fields (pt_program.h GOutLds)
    uint32_t bn;
    f3 ro, rd;             // rayOrigin, rayDirection
};
PT_D float unorm8(unsigned b);
PT_D float pathCounter(const Path& p) { return (float)((p.bn >> 16) & 0x7fu) - 1.0f; }
PT_D void setPathCounter(Path& p, float c) { p.bn = (p.bn & 0xff80ffffu) | ((unsigned)(c + 1.0f) << 16); }

PT_D float rng(Path& p)
{
    p.s0 += 1u; p.s1 += 1u;
    uint32_t qx = 1103515245u * ((p.s0 >> 1u) ^ p.s1);
    uint32_t qy = 1103515245u * ((p.s1 >> 1u) ^ p.s0);
    uint32_t n = 1103515245u * (qx ^ (qy >> 3u));
    return (float)n * (1.0f / 4294967296.0f);
}
PT_D float blueNoise_rand(Path& p)
{
    p.bn += 1u << 16;   // counter = counter + 1.0; channel = int(mod(counter, 2.0)) of a counter >= 0
    const unsigned channel = ((p.bn >> 16) - 1u) & 1u;
    return gfract(unorm8((p.bn >> (8u * channel)) & 255u));
}
PT_D float tentFilter(float x) { return (x < 0.5f) ? gsqrt(2.0f * x) - 1.0f : 1.0f - gsqrt(2.0f - (2.0f * x)); }
PT_D f3 onb_u(f3 nl)
{
    f3 a = (fabsf(nl.y) < 0.9f) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
    return normalize(cross(a, nl));
}
PT_D f3 cosWeightedDir(Path& p, f3 nl)
{
    float r = gsqrt(rng(p));
    float phi = rng(p) * kTwoPi;
    float sn, cs;
    gsincos(phi, sn, cs);
    float x = r * cs, y = r * sn;
    float z = gsqrt(1.0f - x * x - y * y);
    f3 U = onb_u(nl);
    f3 V = cross(nl, U);
    return normalize(U * x + V * y + nl * z);
}
PT_D f3 specularLobeDir(Path& p, f3 rdir, float roughness)
{
    roughness = gclamp(roughness, 0.0f, 1.0f);
    float exponent = gmix(7.0f, 0.0f, gsqrt(roughness));
    float cosTheta = gpow(rng(p), grcp(gexp(exponent) + 1.0f));
    float sinTheta = gsqrt(gmax(0.0f, 1.0f - cosTheta * cosTheta));
    float phi = rng(p) * kTwoPi;
    float sn, cs;
    gsincos(phi, sn, cs);
    f3 U = onb_u(rdir);
    f3 V = cross(rdir, U);
    f3 lobe = (U * cs) * sinTheta + (V * sn) * sinTheta + rdir * cosTheta;
    return normalize(mix3(rdir, lobe, roughness));
}
PT_D float fresnel(f3 rdir, f3 n, float etai, float etat, float& ratioIoR)
{
    float temp = etai;
    float cosi = gclamp(dot(rdir, n), -1.0f, 1.0f);
    if (cosi > 0.0f) { etai = etat; etat = temp; }
    ratioIoR = etai / etat;
    float sint = ratioIoR * gsqrt(1.0f - (cosi * cosi));
    if (sint >= 1.0f) return 1.0f;
    float cost = gsqrt(1.0f - (sint * sint));
    cosi = fabsf(cosi);
    float Rs = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    float Rp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return gclamp(((Rs * Rs) + (Rp * Rp)) * 0.5f, 0.0f, 1.0f);
}
PT_D f3 sampleQuadLight(Path& p, const TraceArgs& a, f3 x, f3 nl, float& weight)
{
    const QuadArg& L = a.light;
    f3 q;
    q.x = gmix(L.v0.x, L.v2.x, gclamp(rng(p), 0.1f, 0.9f));
    q.y = gmix(L.v0.y, L.v2.y, gclamp(rng(p), 0.1f, 0.9f));
    q.z = gmix(L.v0.z, L.v2.z, gclamp(rng(p), 0.1f, 0.9f));
    f3 d = q - x;
    float d2 = dot(d, d);
    float cos_a_max = gsqrt(1.0f - gclamp(a.light_r2 / d2, 0.0f, 1.0f));
    d = normalize(d);
    float dotNl = gmax(0.0f, dot(nl, d));
    float w = 2.0f * (1.0f - cos_a_max) * gmax(0.0f, -dot(d, L.normal)) * dotNl;
    weight = gclamp(w, 0.0f, 1.0f);
    return d;
}

// ------------------------------------------------------------------------------ intersectors
PT_D float unitSphere(f3 ro, f3 rd, f3& n)
{
    float a = dot(rd, rd);
    float b = 2.0f * dot(rd, ro);
    float c = dot(ro, ro) - 1.0f;
    float invA = grcp(a);          // solveQuadratic, js/PathTracingCommon.js:631-641
    b *= invA;
    c *= invA;
    float nh = -b * 0.5f;
    float u2 = nh * nh - c;
    float u;
    if (u2 < 0.0f) { nh = 0.0f; u = 0.0f; } else u = gsqrt(u2);
    float t0 = nh - u, t1 = nh + u;
    float t = t0 > 0.0f ? t0 : t1 > 0.0f ? t1 : kINF;
    if (t != kINF) { f3 h = ro + rd * t; n = mk(2.0f * h.x, 2.0f * h.y, 2.0f * h.z); }
    return t;
}
// TriangleIntersect, single-sided (QuadIntersect passes isDoubleSided = false), edges precomputed
// 1/x < 0 without the division: x negative and finite (1/x of a finite float never underflows to
// zero), or x = -0 (1/-0 = -inf); -inf (1/-inf = -0) and NaN are not
PT_D bool recipNegative(float x) { return (x < 0.0f && x != -__builtin_inff()) || (x == 0.0f && __builtin_signbit(x)); }

PT_D float quadTriangle(const TriArg& T, f3 ro, f3 rd)
{
    f3 pv = cross(rd, T.e2);
    const float dd = dot(T.e1, pv);
    if (recipNegative(dd)) return kINF;   // det < 0: back face, decided before the division
    float det = grcp(dd);
    f3 tv = ro - T.v0;
    float u = dot(tv, pv) * det;
    if (u < 0.0f || u > 1.0f) return kINF;   // the miss is an OR: its first terms decide early
    f3 qv = cross(tv, T.e1);
    float v = dot(rd, qv) * det;
    float t = dot(T.e2, qv) * det;
    return (u < 0.0f || u > 1.0f || v < 0.0f || u + v > 1.0f || t <= 0.0f) ? kINF : t;
}
PT_D float box(f3 mn, f3 mx, f3 ro, f3 inv)
{
    f3 nr = (mn - ro) * inv;
    f3 fr = (mx - ro) * inv;
    float t0 = gmax(gmax(gmin(nr.x, fr.x), gmin(nr.y, fr.y)), gmin(nr.z, fr.z));
    float t1 = gmin(gmin(gmax(nr.x, fr.x), gmax(nr.y, fr.y)), gmax(nr.z, fr.z));
    return gmax(t0, 0.0f) > t1 ? kINF : t0;
}
// box() for a ray whose model-space origin and inverse direction are finite and nonzero and a box
// without NaN: then no slab product is NaN, and IEEE min/max (v_min / v_max / v_min3 / v_max3) pick
// the same values as the GLSL's y<x?y:x forms up to the sign of a zero, which only ever feeds
// comparisons. The min/max are issued directly: through fminf/fmaxf the compiler adds a quieting
// v_max x,x per operand it cannot prove canonical, 6 per box.
PT_D float vmax0(float a) { float r; asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(a)); return r; }
// as one inline-asm block (nr = (mn - ro) * inv, fr = (mx - ro) * inv; t0 = max3 of the three
// min(nr, fr), t1 = min3 of the three max(nr, fr)): the compiler's hazard recognizer sees one block
// instead of eleven and pads no s_nop between them
PT_D float boxFast(f3 mn, f3 mx, f3 ro, f3 inv)
{
    float t0, t1, a0, a1, a2, b0, b1, b2;
    asm("v_sub_f32 %2, %8, %14\n\t"
        "v_sub_f32 %3, %9, %15\n\t"
        "v_sub_f32 %4, %10, %16\n\t"
        "v_sub_f32 %5, %11, %14\n\t"
        "v_sub_f32 %6, %12, %15\n\t"
        "v_sub_f32 %7, %13, %16\n\t"
        "v_mul_f32 %2, %2, %17\n\t"
        "v_mul_f32 %3, %3, %18\n\t"
        "v_mul_f32 %4, %4, %19\n\t"
        "v_mul_f32 %5, %5, %17\n\t"
        "v_mul_f32 %6, %6, %18\n\t"
        "v_mul_f32 %7, %7, %19\n\t"
        "v_min_f32 %0, %2, %5\n\t"
        "v_max_f32 %2, %2, %5\n\t"
        "v_min_f32 %1, %3, %6\n\t"
        "v_max_f32 %3, %3, %6\n\t"
        "v_min_f32 %5, %4, %7\n\t"
        "v_max_f32 %4, %4, %7\n\t"
        "v_max3_f32 %0, %0, %1, %5\n\t"
        "v_min3_f32 %1, %2, %3, %4"
        : "=&v"(t0), "=&v"(t1), "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(b0), "=&v"(b1), "=&v"(b2)
        : "v"(mn.x), "v"(mn.y), "v"(mn.z), "v"(mx.x), "v"(mx.y), "v"(mx.z), "v"(ro.x), "v"(ro.y), "v"(ro.z),
          "v"(inv.x), "v"(inv.y), "v"(inv.z));
    return vmax0(t0) > t1 ? kINF : t0;
}
PT_D bool finite3(f3 v) { return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z); }

// ---- child-pair lines: the two child boxes of an inner record in 12 floats, A.min.xyz A.max.xyz
// B.min.xyz B.max.xyz (a per-axis layout for packed v_pk_add/mul slab arithmetic measured 2 % slower,
// DESIGN.md §6)
// (a0, a1), (b0, b1): the reference texels of children A and B (.yzw = min, max)
PT_D void pairLineWrite(float4* o, float4 a0, float4 a1, float4 b0, float4 b1)
{
    o[0] = make_float4(a0.y, a0.z, a0.w, a1.y);
    o[1] = make_float4(a1.z, a1.w, b0.y, b0.z);
    o[2] = make_float4(b0.w, b1.y, b1.z, b1.w);
}
// the children's box distances of a child-pair line r0..r2 (tA, tB as BoundingBoxIntersect)
PT_D void pairBoxes(float4 r0, float4 r1, float4 r2, f3 O, f3 inv, bool fast, float& tA, float& tB)
{
    if (fast) {
        tA = boxFast(mk(r0.x, r0.y, r0.z), mk(r0.w, r1.x, r1.y), O, inv);
        tB = boxFast(mk(r1.z, r1.w, r2.x), mk(r2.y, r2.z, r2.w), O, inv);
    } else {
        tA = box(mk(r0.x, r0.y, r0.z), mk(r0.w, r1.x, r1.y), O, inv);
        tB = box(mk(r1.z, r1.w, r2.x), mk(r2.y, r2.z, r2.w), O, inv);
    }
}

// BVH_TriangleIntersect / BVH_DoubleSidedTriangleIntersect (js/PathTracingCommon.js:1214-1245)
// from v0 and the edges e1 = v1 - v0, e2 = v2 - v0
PT_D float bvhTriangleE(f3 v0, f3 e1, f3 e2, f3 ro, f3 rd, float& u, float& v, bool dbl)
{
    f3 pv = cross(rd, e2);
    float det = grcp(dot(e1, pv));
    f3 tv = ro - v0;
    u = dot(tv, pv) * det;
    f3 qv = cross(tv, e1);
    v = dot(rd, qv) * det;
    float t = dot(e2, qv) * det;
    bool miss = u < 0.0f || u > 1.0f || v < 0.0f || u + v > 1.0f || t <= 0.0f;
    if (!dbl) miss = miss || det < 0.0f;
    return miss ? kINF : t;
}
PT_D float bvhTriangle(f3 v0, f3 v1, f3 v2, f3 ro, f3 rd, float& u, float& v, bool dbl)
{
    return bvhTriangleE(v0, v1 - v0, v2 - v0, ro, rd, u, v, dbl);
}

// texelFetch on a RGBA32F data texture by linear texel index (== ivec2(mod(i,2048), i/2048) for
// the reference's 2048-wide textures); outside the texture -> 0 (pinned)
PT_D float4 fetch32(const float4* base, long long n, float idx)
{
    if (!(idx >= 0.0f) || !(idx < (float)n)) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return base[(unsigned)idx];   // data textures hold < 2^31 texels (checked at upload)
}
PT_D float unorm8(unsigned b) { return (float)b / 255.0f; }
// REPEAT wrap of an integer-valued texel coordinate: fmod is exact, so any finite coordinate wraps
// exactly; NaN/inf (degenerate uv) wrap to texel 0 (pinned, as the oracle)
PT_D int wrapTexel(float f, int n)
{
    float r = fmodf(f, (float)n);
    if (!(r == r)) r = 0.0f;
    int i = (int)r;
    return i < 0 ? i + n : i;
}
PT_D void texBilinear(const Tex8& t, float u, float v, float out[4])
{
    if (!t.p || t.w <= 0 || t.h <= 0) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }
    float x = u * (float)t.w - 0.5f, y = v * (float)t.h - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float ax = x - fx, by = y - fy;
    int x0 = wrapTexel(fx, t.w), y0 = wrapTexel(fy, t.h);
    int x1 = x0 + 1 == t.w ? 0 : x0 + 1, y1 = y0 + 1 == t.h ? 0 : y0 + 1;
    uchar4 t00 = t.p[y0 * t.w + x0], t10 = t.p[y0 * t.w + x1], t01 = t.p[y1 * t.w + x0], t11 = t.p[y1 * t.w + x1];
    out[0] = gmix(gmix(unorm8(t00.x), unorm8(t10.x), ax), gmix(unorm8(t01.x), unorm8(t11.x), ax), by);
    out[1] = gmix(gmix(unorm8(t00.y), unorm8(t10.y), ax), gmix(unorm8(t01.y), unorm8(t11.y), ax), by);
    out[2] = gmix(gmix(unorm8(t00.z), unorm8(t10.z), ax), gmix(unorm8(t01.z), unorm8(t11.z), ax), by);
    out[3] = gmix(gmix(unorm8(t00.w), unorm8(t10.w), ax), gmix(unorm8(t01.w), unorm8(t11.w), ax), by);
}

// texture(tHDRTexture, uv) on RGBA32F texels: LOD 0 bilinear, REPEAT (as texBilinear)
PT_D float4 texBilinearF(const TexF& t, float u, float v)
{
    if (!t.p || t.w <= 0 || t.h <= 0) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float x = u * (float)t.w - 0.5f, y = v * (float)t.h - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float ax = x - fx, by = y - fy;
    int x0 = wrapTexel(fx, t.w), y0 = wrapTexel(fy, t.h);
    int x1 = x0 + 1 == t.w ? 0 : x0 + 1, y1 = y0 + 1 == t.h ? 0 : y0 + 1;
    const float4 t00 = t.p[(size_t)y0 * t.w + x0], t10 = t.p[(size_t)y0 * t.w + x1];
    const float4 t01 = t.p[(size_t)y1 * t.w + x0], t11 = t.p[(size_t)y1 * t.w + x1];
    return make_float4(gmix(gmix(t00.x, t10.x, ax), gmix(t01.x, t11.x, ax), by),
                       gmix(gmix(t00.y, t10.y, ax), gmix(t01.y, t11.y, ax), by),
                       gmix(gmix(t00.z, t10.z, ax), gmix(t01.z, t11.z, ax), by),
                       gmix(gmix(t00.w, t10.w, ax), gmix(t01.w, t11.w, ax), by));
}

PT_D f3 pow22(f3 c) { return mk(gpow(c.x, 2.2f), gpow(c.y, 2.2f), gpow(c.z, 2.2f)); }

// ------------------------------------------------------------------------------ BVH walks
// Both walks visit the nodes of js/GLTFModelPathTracing_FragmentShader.js:201-298 in the same
// order, cull with the same comparisons and test the same leaves, so they return the same hit;
// `nodes` counts the reference's node fetches (2 texels each) either way.
//
// The stack policy Stk provides pop(level, sentinel) -> float2 and push(level, float2) -> bool
// (false: beyond stackLevels[27], dropped) for any level >= 0.

#ifdef PT_SECPROF
// Experiment builds: the walk loop's load coherence, per wave and bounce (pt_debug_walk_stats): wave
// iterations, those that load a record, those whose loading lanes all load one record, the loading
// lanes, the loading lanes that load the first loading lane's record
struct WalkStat {
    unsigned iters = 0, loads = 0, uniform = 0, lanes = 0, first = 0;
    PT_D void step(bool live, uint32_t off)
    {
        const unsigned long long ld = __ballot(live);
        iters++;
        if (!ld) return;
        const int fl = __ffsll((long long)ld) - 1;
        const uint32_t f = __shfl(off, fl, 64);
        const unsigned long long same = __ballot(live && off == f);
        loads++;
        uniform += same == ld ? 1u : 0u;
        lanes += (unsigned)__popcll(ld);
        first += (unsigned)__popcll(same);
    }
    // by the wave's first active lane, at bounce `bounce` (the same for every lane in a walk: the
    // megakernel's bounce loop is structured)
    PT_D void flush(unsigned long long* out, unsigned bounce)
    {
        if (!out) return;
        const int ln = __lane_id();
        if (ln != (int)__builtin_amdgcn_readfirstlane(ln)) return;
        unsigned long long* o = out + 5u * min(bounce, 7u);
        atomicAdd(o, (unsigned long long)iters);
        atomicAdd(o + 1, (unsigned long long)loads);
        atomicAdd(o + 2, (unsigned long long)uniform);
        atomicAdd(o + 3, (unsigned long long)lanes);
        atomicAdd(o + 4, (unsigned long long)first);
    }
};
#endif

struct BvhResult {
    float triID, triU, triV;
    bool lookup;
    unsigned nodes, leaves, ovf;
#ifdef PT_SECPROF
    unsigned steps, restarts;   // (value-initialised by the callers' brace initialisers)
    WalkStat ws;
#endif
};
// instrumentation hooks of the walks (no code outside PT_SECPROF builds): a walk-loop iteration (its
// lane loads the record at `off` when `live`), a restart descent's record load
#ifdef PT_SECPROF
PT_D void secWalkStep(BvhResult& r, bool live, uint32_t off) { r.steps++; r.ws.step(live, off); }
PT_D void secRestart(BvhResult& r) { r.restarts++; }
#else
PT_D void secWalkStep(BvhResult&, bool, uint32_t) {}
PT_D void secRestart(BvhResult&) {}
#endif

template <class Stk>
PT_D void stackPush(const TraceArgs& a, Stk& st, int si, float2 e, unsigned& ovf)
{
    if (!st.push(si, e)) { ovf++; atomicOr(a.err, (unsigned)E_STACK); }   // GLSL would write out of bounds: dropped
}
// a pop past stackLevels[27] (undefined in the GLSL) yields `sentinel`, whose tNear = INFINITY the
// walk culls at once (pinned with the oracle; nothing is read out of bounds)
template <class Stk>
PT_D float2 stackPop(const Stk& st, int si, float2 sentinel)
{
    return st.pop(si, sentinel);
}

// The reference layout: a pushed entry is (node id, tNear); a pop re-fetches the node's two texels.
// Entry: c0/c1 = the root's texels, curT = its box distance (already counted by the caller).
template <class Stk>
PT_D void bvhWalkRef(const TraceArgs& a, f3 O, f3 D, f3 inv, bool dbl, float4 c0, float4 c1, float curT,
                     float& hitT, Stk& st, BvhResult& r)
{
    float stackptr = 0.0f, curId = 0.0f;
    bool skip = curT < hitT;
    for (;;) {
        if (!skip) {
            stackptr = stackptr - 1.0f;
            if (stackptr < 0.0f) break;
            float2 e = stackPop(st, (int)stackptr, make_float2(0.0f, kINF));
            curId = e.x; curT = e.y;
            if (curT >= hitT) continue;
            c0 = fetch32(a.aabb, a.aabb_texels, curId * 2.0f);
            c1 = fetch32(a.aabb, a.aabb_texels, curId * 2.0f + 1.0f);
            r.nodes++;
        }
        skip = false;
        if (c0.x < 0.0f) {   // inner node: both children, near first
            float idA = curId + 1.0f, idB = c1.x;
            float4 a0 = fetch32(a.aabb, a.aabb_texels, idA * 2.0f), a1 = fetch32(a.aabb, a.aabb_texels, idA * 2.0f + 1.0f);
            float4 b0 = fetch32(a.aabb, a.aabb_texels, idB * 2.0f), b1 = fetch32(a.aabb, a.aabb_texels, idB * 2.0f + 1.0f);
            r.nodes += 2;
            float tA = box(mk(a0.y, a0.z, a0.w), mk(a1.y, a1.z, a1.w), O, inv);
            float tB = box(mk(b0.y, b0.z, b0.w), mk(b1.y, b1.z, b1.w), O, inv);
            if (tB < tA) {
                float ti = idB; idB = idA; idA = ti;
                float tt = tB; tB = tA; tA = tt;
                float4 x0 = b0; b0 = a0; a0 = x0;
                float4 x1 = b1; b1 = a1; a1 = x1;
            }
            if (tB < hitT) { curId = idB; curT = tB; c0 = b0; c1 = b1; skip = true; }
            if (tA < hitT) {
                if (skip) {
                    stackPush(a, st, (int)stackptr, make_float2(idB, tB), r.ovf);
                    stackptr = stackptr + 1.0f;
                }
                curId = idA; curT = tA; c0 = a0; c1 = a1; skip = true;
            }
            continue;
        }
        // leaf: one triangle per leaf
        float id = 8.0f * c0.x;
        float4 t0 = fetch32(a.tri, a.tri_texels, id), t1 = fetch32(a.tri, a.tri_texels, id + 1.0f),
               t2 = fetch32(a.tri, a.tri_texels, id + 2.0f);
        r.leaves++;
        float tu, tv;
        float d = bvhTriangle(mk(t0.x, t0.y, t0.z), mk(t0.w, t1.x, t1.y), mk(t1.z, t1.w, t2.x), O, D, tu, tv, dbl);
        if (d < hitT) { hitT = d; r.triID = id; r.triU = tu; r.triV = tv; r.lookup = true; }
    }
}

// Child-pair records (pt_pairs_* in pt_kernels.hip; only for trees whose links are exact in-range
// integers, see pt_capi.cpp ensure_pairs). Nodes are addressed by a 32-bit code (pairCode,
// pt_args.h): the byte offset of an inner node's record in the dense inner-record array, or
// kLeafBit | the byte offset of a leaf's record in the dense leaf-record array, kept as float bits
// in records and stack entries. Both arrays are read through buffer descriptors, so an inner code
// is the load's voffset as it stands (no float->int conversion or 64-bit address arithmetic).
//   inner record (64 B, one line): A.min.xyz A.max.x | A.max.yz B.min.xy | B.min.z B.max.xyz | codeA codeB
//     (pairLineWrite)
//     (A = the node's left child n+1, B = its right-child link)
//   leaf record (48 B): the leaf triangle's v0, e1 = v1 - v0, e2 = v2 - v0 (9 floats), its idObject
// An inner step is one 64-byte line instead of two 32-byte nodes in different lines, a pop needs
// no fetch (the stack entry (tNear, code) already says what the node is), and a leaf's vertices
// sit in a dense 48-byte record instead of the first third of a 128-byte triangle texel group:
// both arrays together are about 3.4 MB for StanfordBunny, within one XCD's L2.
// The walk: `pop` = the next step pops the stack (the reference loop's !skip). `fast` = the ray
// qualifies for boxFast (records are NaN-free, checked at build). A schedule that interleaved walk
// steps with other lanes' shading on top of it measured slower.
// the record array as a buffer descriptor, built from kernel arguments and made provably
// wave-uniform (readfirstlane) so that no waterfall loop wraps the loads
struct PairBufs {
    __amdgpu_buffer_rsrc_t rec;
};
PT_D __amdgpu_buffer_rsrc_t uniformRsrc(const void* p, uint32_t bytes)
{
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
PT_D PairBufs pairBufs(const TraceArgs& a)
{
    return PairBufs{ uniformRsrc(a.bvh_pairs, a.bvh_pairs_bytes) };
}
typedef unsigned int vu4 __attribute__((ext_vector_type(4)));
typedef unsigned int vu2 __attribute__((ext_vector_type(2)));
PT_D float4 ldRec4(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const vu4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
PT_D float2 ldRec2(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const vu2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
    return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
PT_D bool pairWalkFast(f3 O, f3 inv)
{
    return finite3(O) && finite3(inv) && inv.x != 0.0f && inv.y != 0.0f && inv.z != 0.0f;
}
// One loop exit (the empty stack), and the walk's flags as integers in VGPRs: a bool lives in an
// SGPR lane mask that every divergent merge rebuilds (s_andn2 / s_and / s_or per flag per merge;
// 73 -> 45 scalar instructions in the loop, dragon stand-in -1.3 %). A pop is a
// predicated LDS read; a culled pop skips the rest of its step. One set of four record loads for
// either kind of record (both live in one array): a wave whose lanes sit at inner and at leaf nodes
// issues 4 vector-memory instructions, not 4 + 3. A leaf record is 48 B; its lane's fourth load reads
// the next record's first 8 B (or 0 past the end of the array) and is not used.
template <class Stk>
PT_D void bvhWalkPairs(const TraceArgs& a, f3 O, f3 D, f3 inv, bool dbl, float curT, float& hitT, Stk& st,
                       BvhResult& r, bool anyHit = false)
{
    const bool fast = pairWalkFast(O, inv);
    const PairBufs b = pairBufs(a);
    uint32_t code = a.bvh_root_code;
    float hT = hitT;
    int sp = 0;
    int pop = curT < hitT ? 0 : 1;
    float tID = -1.0f, tU = 0.0f, tV = 0.0f;
    for (;;) {
        asm volatile("" : "+v"(pop));
        const int sp2 = sp - pop;
        if (sp2 < 0) break;
        sp = sp2;
        const float2 e = stackPop(st, pop ? sp2 : 0, make_float2(kINF, 0.0f));
        const bool live = !pop || e.x < hT;
        if (pop && live) r.nodes++;
        code = pop ? __float_as_uint(e.y) : code;
        pop = 1;
        secWalkStep(r, live, code & ~kLeafBit);
        if (!live) continue;
        const uint32_t off = code & ~kLeafBit;
        const float4 r0 = ldRec4(b.rec, off), r1 = ldRec4(b.rec, off + 16u), r2 = ldRec4(b.rec, off + 32u);
        const float2 r3 = ldRec2(b.rec, off + 48u);
        if (!(code & kLeafBit)) {
            r.nodes += 2;
            float tA, tB;
            pairBoxes(r0, r1, r2, O, inv, fast, tA, tB);
            // the reference's swap and two ifs as selects: the near child is next if it is hit, else
            // the far one; the far one is pushed when both are hit
            const bool sw = tB < tA;
            const float tN = sw ? tB : tA, tF = sw ? tA : tB;
            const bool hitN = tN < hT, hitF = tF < hT;
            const float cN = sw ? r3.y : r3.x, cF = sw ? r3.x : r3.y;   // codes as float bits: only moved
            if (hitN && hitF) {
                stackPush(a, st, sp, make_float2(tF, cF), r.ovf);
                sp++;
            }
            code = __float_as_uint(hitN ? cN : hitF ? cF : __uint_as_float(code));
            pop = (hitN || hitF) ? 0 : 1;
        } else {
            r.leaves++;
            float tu, tv;
            const float d = bvhTriangleE(mk(r0.x, r0.y, r0.z), mk(r0.w, r1.x, r1.y), mk(r1.z, r1.w, r2.x), O, D, tu, tv, dbl);
            if (d < hT) {
                hT = d; tID = 8.0f * r2.y; tU = tu; tV = tv;
                if (anyHit) sp = 0;   // the first occluder ends the walk: the next step's pop finds it empty
            }
            // a use on this side too keeps the codes' load with the other three: sunk into the inner-node
            // branch, it was issued only after a mixed wave's leaf tests (-3 % kernel time)
            asm volatile("" ::"v"(r3.x));
        }
    }
    hitT = hT;
    if (tID >= 0.0f) { r.triID = tID; r.triU = tU; r.triV = tV; r.lookup = true; }
}

// ------------------------------------------------------------------------------ restart-trail walk
// The child-pair records walked without a stack in memory (PT_BVH_TRAIL; north_star's "stackless
// BVH traversal"): the ordered near-first walk of js/GLTFModelPathTracing_FragmentShader.js:211-298
// keeps, per depth d of the current path (bit 31 - d of a register; the root's bit 31 has none),
//   pend   1: both children were hit and the near one is being walked - the far one is pending (the
//             reference stack's entry); the restart trail's 0 bits (Laine 2010), kept inverted so that
//             a pop is two operations: the deepest pending level is pend's lowest set bit;
//   dir    which child the path took: 1 = B (the right link), 0 = A (the left child n + 1).
// A pop clears the deepest pending level's bit and flips its dir bit: its far child is next. The
// pending levels' (tNear, code) entries - the reference stack's contents - are kept in a per-lane ring
// of R LDS slots (R - 1 of them live, the free one takes every step's push store without a branch)
// that drops its oldest (shallowest) entry when full; when a pop finds the ring empty the walk
// restarts (trailRestart): it jumps to a copy of the deepest ancestor held in the jump table of the
// top kTopLevels levels' inner records (indexed by the path's dir bits, so the jump is no load of its
// own) and descends along the dir bits to the pending level's parent, testing on the way the pending
// siblings' boxes to refill the ring. The boxes are the same floats tested by the same function, so a
// re-tested entry carries the bits it was pushed with, and the walk visits the reference walk's nodes
// in its order: same hit, same counters (restart descents are no node fetches of the reference's).
// The host gives it trees of depth <= 28, whose nodes have one parent each (pt_pairs_depth): there
// at most 27 far children are ever pending, so the reference's stack (stackLevels[28]) never
// overflows and no push is dropped; other trees keep the stack walk.
struct TrailWalk {
    uint32_t code;             // record to load next
    float hitT;
    float triID, triU, triV;
    uint32_t pend, dir;        // per depth d: bit 31 - d
    uint32_t lvl;              // the bit of the depth of the node `code` addresses (root: bit 31)
    int rtop, rcnt;            // ring: next slot, entries held (at most R - 1: slot rtop is always free)
    bool pop, lookup;
};
constexpr uint32_t kRootBit = 0x80000000u;
// push onto the ring without a branch: the store always goes to the free slot rtop, and only a real
// push advances the ring (a full ring then frees its oldest slot)
template <int R>
PT_D void ringPush(lds_float2* ring, unsigned stride, unsigned slot, TrailWalk& w, bool push, float t, float code)
{
    const vf2 v = { t, code };
    ring[(unsigned)w.rtop * stride + slot] = v;
    w.rtop = push ? (w.rtop == R - 1 ? 0 : w.rtop + 1) : w.rtop;
    w.rcnt = push ? min(w.rcnt + 1, R - 1) : w.rcnt;
}
// The restart (the ring ran dry at a pop of the level w.lvl): from the jump table's copy of the
// deepest ancestor it holds, down the dir bits to the popped level's parent, pushing the pending
// siblings met on the way back onto the ring; returns the popped level's far child as a ring entry
// would hold it (its box distance, its code).
template <int R>
PT_D float2 trailRestart(const TraceArgs& a, const PairBufs& b, f3 O, f3 inv, bool fast, lds_float2* ring,
                         unsigned stride, unsigned slot, TrailWalk& w, BvhResult& r)
{
    const int p = min(30 - __builtin_ctz(w.lvl), kTopLevels);   // the popped depth - 1, capped
    uint32_t code = a.bvh_top_base + ((1u << p) - 1u + (w.dir >> (31 - p))) * 64u;
    uint32_t l = kRootBit >> p;
    for (;;) {
        secRestart(r);
        const float4 r0 = ldRec4(b.rec, code), r1 = ldRec4(b.rec, code + 16u), r2 = ldRec4(b.rec, code + 32u);
        const float2 r3 = ldRec2(b.rec, code + 48u);
        float tA, tB;
        pairBoxes(r0, r1, r2, O, inv, fast, tA, tB);
        l >>= 1;
        const bool takeB = (w.dir & l) != 0u;
        if (l == w.lvl) return make_float2(takeB ? tB : tA, takeB ? r3.y : r3.x);   // the far child popped
        ringPush<R>(ring, stride, slot, w, (w.pend & l) != 0u, takeB ? tA : tB, takeB ? r3.x : r3.y);   // a pending sibling
        code = __float_as_uint(takeB ? r3.y : r3.x);
    }
}
// one step; false once the walk is over. A step pops (culled: the step ends there) and/or loads one
// record: an inner node's two children or a leaf's triangle.
template <int R>
PT_D bool trailWalkStep(const TraceArgs& a, const PairBufs& b, f3 O, f3 D, f3 inv, bool dbl, bool fast,
                        lds_float2* ring, unsigned stride, unsigned slot, TrailWalk& w, BvhResult& r)
{
    if (w.pop) {
        if (w.pend == 0u) return false;                // no level pending: the walk is over
        w.lvl = w.pend & (0u - w.pend);                // the deepest pending level
        w.pend ^= w.lvl;
        w.dir ^= w.lvl;                                // its far child
        w.rtop = (w.rtop == 0 ? R : w.rtop) - 1;       // (moving an empty ring's top is harmless)
        vf2 e = ring[(unsigned)w.rtop * stride + slot];
        if (w.rcnt == 0) {
            const float2 f = trailRestart<R>(a, b, O, inv, fast, ring, stride, slot, w, r);
            e.x = f.x; e.y = f.y;
        } else
            w.rcnt--;
        if (e.x >= w.hitT) return true;                // culled pop
        w.code = __float_as_uint(e.y);
        r.nodes++;
        w.pop = false;
    }
    w.pop = true;
    const uint32_t off = w.code & ~kLeafBit;
    const float4 r0 = ldRec4(b.rec, off), r1 = ldRec4(b.rec, off + 16u), r2 = ldRec4(b.rec, off + 32u);
    const float2 r3 = ldRec2(b.rec, off + 48u);
    if (!(w.code & kLeafBit)) {
        r.nodes += 2;
        float tA, tB;
        pairBoxes(r0, r1, r2, O, inv, fast, tA, tB);
        // the reference's step: the near child next if it is hit, else the far one; the far one
        // pending when both are hit
        const bool sw = tB < tA;   // the reference's swap: B is the near child
        const float tF = sw ? tA : tB;
        const bool hitN = (sw ? tB : tA) < w.hitT, hitF = tF < w.hitT;
        const bool both = hitN && hitF;
        const uint32_t bk = w.lvl >> 1;
        ringPush<R>(ring, stride, slot, w, both, tF, sw ? r3.x : r3.y);
        const bool takeB = hitN ? sw : !sw;
        w.pend |= both ? bk : 0u;
        w.dir = takeB ? (w.dir | bk) : (w.dir & ~bk);
        w.code = __float_as_uint(takeB ? r3.y : r3.x);
        w.lvl = (hitN || hitF) ? bk : w.lvl;
        w.pop = !(hitN || hitF);
        return true;
    }
    r.leaves++;
    float tu, tv;
    const float d = bvhTriangleE(mk(r0.x, r0.y, r0.z), mk(r0.w, r1.x, r1.y), mk(r1.z, r1.w, r2.x), O, D, tu, tv, dbl);
    if (d < w.hitT) { w.hitT = d; w.triID = 8.0f * r2.y; w.triU = tu; w.triV = tv; w.lookup = true; }
    asm volatile("" ::"v"(r3.x));   // keeps the codes' load with the other three (as pairWalkStep)
    return true;
}
// ring: R float2 slots per lane at ring[k * stride + slot]
template <int R>
PT_D void bvhWalkTrail(const TraceArgs& a, f3 O, f3 D, f3 inv, bool dbl, float curT, float& hitT, lds_float2* ring,
                       unsigned stride, unsigned slot, BvhResult& r)
{
    TrailWalk w;
    w.code = a.bvh_root_code; w.hitT = hitT;
    w.triID = 0.0f; w.triU = 0.0f; w.triV = 0.0f;
    w.pend = 0u; w.dir = 0u; w.lvl = kRootBit; w.rtop = 0; w.rcnt = 0;
    w.pop = !(curT < hitT);
    w.lookup = false;
    const bool fast = pairWalkFast(O, inv);
    const PairBufs b = pairBufs(a);
    while (trailWalkStep<R>(a, b, O, D, inv, dbl, fast, ring, stride, slot, w, r)) secWalkStep(r, false, 0u);
    hitT = w.hitT;
    if (w.lookup) { r.triID = w.triID; r.triU = w.triU; r.triV = w.triV; r.lookup = true; }
}

} // namespace pt
