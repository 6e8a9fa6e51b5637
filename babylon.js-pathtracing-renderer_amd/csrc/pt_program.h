// pt_program.h — the per-path part of the reference's fragment program, shared by the megakernel
// (pt_kernels.hip: pt_trace, pt_persist) and the wavefront kernels (pt_wavefront.hip): the hit
// record, CalculateRadiance's loop body after SceneIntersect (shadeStep), the physical sky and
// main()'s camera ray. Everything keeps the pinned GLSL semantics of pt_glsl.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_device.h"
#include "pt_glsl.h"
#include "pt_quadric.h"

namespace pt {

// SceneIntersect's outputs (hitT, hitNormal, hitColor, hitType, hitObjectID, hit uv)
struct Hit {
    float t;
    f3 normal, color;
    float u, v;
    int type;
    int id;
};

struct Cnt {
    unsigned seg, node, leaf, hit, tap, ovf, hdr;
#ifdef PT_SECPROF
    unsigned long long* sec;   // experiment builds: per-wave LDS slots ([0..7] section sums, [8] last mark,
                               // [9] walk max scratch, [10] wave walk iterations, [11] longest lane's walk steps)
    unsigned lane_steps;
    unsigned sget, sget_slab, sput, sput_slab;   // stack pops / pushes, and those beyond the LDS levels
    unsigned bounce;                             // SceneIntersect calls so far (the walk statistics' bounce)
#endif
};
// section profile (experiment builds only, -DPT_SECPROF): the wave's shader clock between marks,
// charged to section k by the first active lane (divergent code is charged once per wave)
#ifdef PT_SECPROF
#define PT_SEC(cnt, k)                                                                        \
    do {                                                                                      \
        const unsigned long long now_ = clock64();                                            \
        const int ln_ = __lane_id();                                                          \
        if ((cnt).sec && ln_ == __builtin_amdgcn_readfirstlane(ln_)) {                \
            (cnt).sec[k] += now_ - (cnt).sec[8]; (cnt).sec[8] = now_;                         \
        }                                                                                     \
    } while (0)
#else
#define PT_SEC(cnt, k) do {} while (0)
#endif

// CalculateRadiance's `out` parameters objectNormal / objectColor / objectID / pixelSharpness:
// in registers (GOut) or, for the megakernel, packed (GOutLds): the normal and colour in LDS
// [field][lane], which takes six live values out of the VGPR budget of the bounce loop, and the id and
// sharpness as bits of the path's blue-noise register (free bits of a value that is live anyway)
struct GOut {
    static constexpr bool kColById = false;
    f3 nrm, col;
    float id, sharp;
    PT_D void clear() { nrm = mk(0, 0, 0); col = mk(0, 0, 0); id = 0.0f; sharp = 0.0f; }
    PT_D void pinCol(f3) {}
    PT_D void setNrm(f3 v) { nrm = v; }
    PT_D void setCol(f3 v) { col = v; }
    PT_D void setId(float v) { id = v; }
    PT_D void setSharp(float v) { sharp = v; }
};
typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(1))) float glb_float;
// The packed G-buffer of pt_trace. Path::bn bits 24-25 hold the sharpness (0: 0.0, 1: 1.01, 2: -1.0:
// the only values the GLSL assigns), bits 26-30 objectID (an object index < 32: hitObjectID of the
// spheres / quadric shapes, the quads, the mesh), bit 23 "objectNormal's fields beyond LDS were
// written", bit 31 the same for objectColor; the blue-noise counter keeps bits 16-22 (at most 13
// draws per path). LS = lanes of the workgroup = the stride of one field; NF = the normal / colour
// fields in LDS (from the normal's x), the rest at `gx` (after the stack slab's levels), field-major
// [field][lane of the grid] with `gs` lanes per field, so that a wave's store of one field is one
// contiguous 256-B run: stored only by setNrm / setCol and read only when their bit says so - no
// clearing store, no id / sharpness traffic at all.
// With the colour wholly outside LDS (NF <= 3) it is not stored at all: objectColor is the bounce-0
// hit's colour, and every object's hit colour is a constant of the object (objectMaterial), so the
// end of the path recomputes it from the bounce-0 id - unless bounce 1 after METAL replaced the id,
// when pinCol stores it first (bit 31 then says so).
template <int LS, int NF = 6>
struct GOutLds {
    static constexpr bool kColById = NF <= 3;
    lds_float* p;
    unsigned slot;
    glb_float* gx;    // wave-uniform base ...
    unsigned gi, gs;  // ... this lane's index, lanes per field (32-bit: one VGPR, shared with the stack slab's)
    uint32_t* bn;
    // the address formed where it is used (the empty asm keeps it from being hoisted out of the
    // bounce loop as six 64-bit pointers)
    PT_D unsigned at(int f) const
    {
        unsigned i = gi;
        asm volatile("" : "+v"(i));
        return i + (unsigned)(f - NF) * gs;
    }
    PT_D void put(int f, float v)
    {
        if (f < NF) p[f * LS + slot] = v;
        else gx[at(f)] = v;
    }
    PT_D float get(int f) const
    {
        if (f < NF) return p[f * LS + slot];
        return ((*bn >> (f < 3 ? 23 : 31)) & 1u) ? gx[at(f)] : 0.0f;
    }
    PT_D void clear()
    {
        for (int f = 0; f < NF; f++) p[f * LS + slot] = 0.0f;
        *bn &= 0x007fffffu;
    }
    PT_D void setNrm(f3 v)
    {
        put(0, v.x); put(1, v.y); put(2, v.z);
        if (NF < 3 || kColById) *bn |= 1u << 23;   // (kColById: also "bounce 0 hit something" for load)
    }
    PT_D void setCol(f3 v)
    {
        if (kColById) return;
        put(3, v.x); put(4, v.y); put(5, v.z);
        if (NF < 6) *bn |= 1u << 31;
    }
    PT_D void pinCol(f3 v)
    {
        if (!kColById) return;
        put(3, v.x); put(4, v.y); put(5, v.z);
        *bn |= 1u << 31;
    }
    PT_D void setId(float v) { *bn = (*bn & ~(31u << 26)) | (((unsigned)(int)v & 31u) << 26); }
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
    PT_D float id() const { return (float)((*bn >> 26) & 31u); }
    // colOfId(id): the hit colour of object `id` (kColById)
    template <class F>
    PT_D GOut load(F colOfId) const
    {
        GOut g;
        g.nrm = mk(get(0), get(1), get(2)); g.id = id(); g.sharp = sharp();
        if (!kColById) g.col = mk(get(3), get(4), get(5));
        else if (!((*bn >> 23) & 1u)) g.col = mk(0.0f, 0.0f, 0.0f);   // no bounce-0 hit: the pinned zeros
        else g.col = ((*bn >> 31) & 1u) ? mk(get(3), get(4), get(5)) : colOfId(g.id);
        return g;
    }
};

// CalculateRadiance: js/GLTFModelPathTracing_FragmentShader.js:351-609 and
// js/BabylonPathTracing_FragmentShader.js:117-344 (METAL is a mirror there), as one step per
// iteration of its `for (bounces < 6)` loop so that the persistent kernel can interleave paths.
// The reference's per-material branches are folded so that each sampling routine has ONE call
// site (TRANSPARENT and CLEARCOAT_DIFFUSE share the Fresnel split; CLEARCOAT's transmitted branch
// joins DIFFUSE's "cosine bounce or light sample" tail). The sequence of rng()/blueNoise_rand()
// draws and every IEEE op per path are exactly the GLSL's.
struct PState {
    f3 mask;
    float roughness;        // metallicRoughness.g persists across bounces (:368, :496)
    int diffuseCount, hitType, bounce;
    bool coat, specular, sampleLight;
};

template <class G>
PT_D void pathBegin(PState& s, G& g)
{
    s.mask = mk(1, 1, 1);
    s.roughness = 0.0f;
    s.diffuseCount = 0; s.hitType = -100; s.bounce = 0;
    s.coat = false; s.specular = true; s.sampleLight = false;
    g.clear();   // pinned `out` zeros
}

// Get_Sky_Color (js/PathTracingCommon.js:416-475, the three.js SkyShader Preetham model). The
// uniform-only terms (sun intensity, extinction coefficients, sun fade, ...) come precomputed in
// SkyArgs by the host with these same pinned sequences (pt_capi.cpp sky_setup).
PT_D float rayleighPhase(float cosTheta) { return 0.05968310365946075f * (1.0f + (cosTheta * cosTheta)); }
PT_HD float hgPhase(float cosTheta, float g)
{
    float g2 = g * g;
    float inverse = grcp(gpow(gmax(0.0f, 1.0f - 2.0f * g * cosTheta + g2), 1.5f));
    return 0.07957747154594767f * ((1.0f - g2) * inverse);
}
PT_D f3 pow3(f3 v, float e) { return mk(gpow(v.x, e), gpow(v.y, e), gpow(v.z, e)); }
PT_D f3 skyColor(const SkyArgs& k, f3 rayDir)
{
    const f3 vd = normalize(rayDir);
    const float cosViewSunAngle = dot(vd, k.sun);
    const float zenithAngle = gacos(gmax(0.0f, dot(mk(0.0f, 1.0f, 0.0f), vd)));
    const float inverse =
        grcp(gcos(zenithAngle) + 0.15f * gpow(93.885f - ((zenithAngle * 180.0f) / 3.14159265358979323f), -1.253f));
    const float rl = 8400.0f * inverse, ml = 1250.0f * inverse;
    const f3 e = k.rayleigh * rl + k.mie * ml;
    const f3 Fex = mk(gexp(-e.x), gexp(-e.y), gexp(-e.z));
    const f3 betaR = k.rayleigh * rayleighPhase(cosViewSunAngle * 0.5f + 0.5f);
    const f3 betaM = k.mie * hgPhase(cosViewSunAngle, 0.76f);
    const f3 q = (betaR + betaM) / k.rm;
    f3 Lin = pow3((q * k.sunE) * (mk(1.0f, 1.0f, 1.0f) - Fex), 1.5f);
    const f3 m = pow3((q * k.sunE) * Fex, 1.0f / 2.0f);
    Lin = Lin * mk(gmix(1.0f, m.x, k.fade), gmix(1.0f, m.y, k.fade), gmix(1.0f, m.z, k.fade));
    f3 L0 = mk(0.1f, 0.1f, 0.1f) * Fex;
    const float sundisk = gsmoothstep(0.9998f, 0.9998f + 0.00002f, cosViewSunAngle);
    L0 = L0 + (Fex * k.sunE19000) * sundisk;
    const f3 tex = (Lin + L0) * 0.04f + mk(0.0f, 0.0003f, 0.00075f);
    return pow3(tex, k.retExp);
}

// hitObjectID of the glTF model: SceneIntersect's objectCount after the spheres and quads
// (js/GLTFModelPathTracing_FragmentShader.js:343)
template <int PROG>
PT_D int meshObjectId(const TraceArgs& a) { return kQuadId0<PROG> + a.nquads; }

// hitColor / hitType of analytic object `id` (the values SceneIntersect writes with it)
template <int PROG>
PT_D void objectMaterial(const TraceArgs& a, int id, f3& color, int& type)
{
    constexpr int q0 = kQuadId0<PROG>;
    if (kIsQuadric<PROG> && id >= 0 && id < q0) {
        // js/TransformedQuadricGeometry_FragmentShader.js:103-293
        const float cr[12] = { 1.0f, 0.0f, 1.0f, 1.0f, 1.0f, 0.5f, 0.0f, 0.0f, 0.2f, 0.0f, 1.0f, 0.5f };
        const float cg[12] = { 0.0f, 1.0f, 1.0f, 0.0f, 0.1f, 1.0f, 0.4f, 0.0f, 0.0f, 1.0f, 0.3f, 0.0f };
        const float cb[12] = { 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, 1.0f, 1.0f, 1.0f, 0.5f, 0.0f, 1.0f };
        color = mk(cr[id], cg[id], cb[id]);
        type = a.shape_mat;
    } else if (!kIsQuadric<PROG> && id >= 0 && id < 2) {
        color = a.sph[id].color; type = a.sph[id].type;
    } else if (id >= q0 && id < q0 + a.nquads) {
        color = a.qcolor[id - q0]; type = a.qtype[id - q0];
    } else if (kHasMesh<PROG> && id == meshObjectId<PROG>(a)) {
        color = mk(1.0f, 1.0f, 1.0f); type = a.uses_albedo ? PBR_MATERIAL : a.model_mat;
    }
}

// SceneIntersect's analytic objects (spheres or the twelve quadric shapes, then the quads), with
// the closest hit's attributes resolved once (the GLSL writes them at every closer hit; only the
// last write survives). The object loops stay rolled (#pragma unroll 1): each iteration re-reads
// its object from the kernarg segment through the scalar cache, which keeps ~130 wave-uniform
// floats out of VGPRs and the code small enough for the instruction cache.
template <int PROG>
PT_D void analyticNearest(const TraceArgs& a, f3 rayO, f3 rayD, Hit& h, f3& sn)
{
    constexpr int q0 = kQuadId0<PROG>;
    h.t = kINF;
    h.type = -100;
    h.id = -1;
    sn = mk(0, 0, 0);
    if (kIsQuadric<PROG>) {
#pragma unroll 1
        for (int s = 0; s < 12; s++) {
            f3 n = mk(0, 0, 0);
            float d = quadricShape(s, mul(a.shape_inv[s], rayO, 1.0f), mul(a.shape_inv[s], rayD, 0.0f), a.shape_k, n);
            if (d < h.t) { h.t = d; h.id = s; sn = n; }
        }
    } else {
#pragma unroll 1
        for (int s = 0; s < 2; s++) {
            const SphereArg& S = a.sph[s];
            f3 n;
            float d = unitSphere(mul(S.inv, rayO, 1.0f), mul(S.inv, rayD, 0.0f), n);
            if (d < h.t) { h.t = d; h.id = s; sn = n; }
        }
    }
#pragma unroll 1
    for (int i = 0; i < a.nquads; i++) {
        // the quad's 18 floats loaded (scalar) before the tests, one wait instead of one per use
        // (bunny -1 %, dragon stand-in -0.3 %)
        const TriArg A = a.qtri[2 * i], B = a.qtri[2 * i + 1];
        asm volatile("" ::"s"(A.v0.x), "s"(A.v0.y), "s"(A.v0.z), "s"(A.e1.x), "s"(A.e1.y), "s"(A.e1.z), "s"(A.e2.x),
                     "s"(A.e2.y), "s"(A.e2.z), "s"(B.v0.x), "s"(B.v0.y), "s"(B.v0.z), "s"(B.e1.x), "s"(B.e1.y),
                     "s"(B.e1.z), "s"(B.e2.x), "s"(B.e2.y), "s"(B.e2.z));
        float d = gmin(quadTriangle(A, rayO, rayD), quadTriangle(B, rayO, rayD));
        if (d < h.t) { h.t = d; h.id = q0 + i; }
    }
}
// the winner's attributes; `sn` = its object-space normal (spheres / quadric shapes)
template <int PROG>
PT_D void analyticAttributes(const TraceArgs& a, Hit& h, f3 sn)
{
    constexpr int q0 = kQuadId0<PROG>;
    if (h.id >= 0 && h.id < q0) {
        const m4& M = kIsQuadric<PROG> ? a.shape_inv[h.id] : a.sph[h.id].inv;
        // disk and rectangle: hitNormal = vec3(0,-1,0), not normalized before the transform
        const f3 n0 = (kIsQuadric<PROG> && (h.id == 9 || h.id == 10)) ? mk(0.0f, -1.0f, 0.0f) : normalize(sn);
        h.normal = normalize(mul3t(M, n0));
    } else if (h.id >= q0) {
        h.normal = normalize(a.qnormal[h.id - q0]);
    }
    if (h.id >= 0) objectMaterial<PROG>(a, h.id, h.color, h.type);
}
template <int PROG>
PT_D void analyticIntersect(const TraceArgs& a, f3 rayO, f3 rayD, Hit& h)
{
    f3 sn;
    analyticNearest<PROG>(a, rayO, rayD, h, sn);
    analyticAttributes<PROG>(a, h, sn);
}
// Get_HDR_Color (js/HDRIEnvironmentPathTracing_FragmentShader.js:351-360): equirect lookup
template <bool COUNT>
PT_D f3 envColor(const TraceArgs& a, f3 rd, Cnt& cnt)
{
    const float u = gatan2(rd.x, rd.z) * 0.15915494309f + 0.5f;   // ONE_OVER_TWO_PI as the GLSL spells it
    const float v = gacos(-rd.y) * 0.31830988618379067f;
    const float4 t = texBilinearF(a.hdr, u, v);
    if (COUNT) cnt.hdr += 4;
    return mk(t.x, t.y, t.z) * a.hdr_exposure;
}

// The loop body after SceneIntersect, for the intersection `h` of the current ray. Returns false
// when the path has ended; `accum` then holds the radiance before the final max(accum, 0).
template <int PROG, bool COUNT, class G>
PT_D bool shadeStep(const TraceArgs& a, Path& p, PState& s, G& g, f3& accum, Hit& h, Cnt& cnt)
{
    constexpr bool gltf = kIsGltf<PROG>;
    constexpr bool sky = kIsSky<PROG>;
    constexpr bool hdri = kIsHdri<PROG>;
    const int bounces = s.bounce;
    const int prevType = s.hitType;
    int hitType = h.type;
    s.hitType = hitType;
    if (h.t == kINF) {
        if (hdri) {   // js/HDRIEnvironmentPathTracing_FragmentShader.js:404-438 (always ends the path)
            const f3 env = envColor<COUNT>(a, p.rd, cnt);
            if (bounces == 0) { g.setSharp(1.01f); accum = env; }
            else if (s.diffuseCount == 0 && s.specular) { g.setSharp(1.01f); accum = s.mask * env; }
            else if (s.sampleLight) accum = s.mask * env;
            else if (s.diffuseCount == 1 && prevType == TRANSPARENT && s.specular && bounces < 3) {
                if (dot(p.rd, a.sky.sun) > 0.99f) g.setSharp(1.01f);
                accum = s.mask * env;
            } else if (s.diffuseCount > 0) accum = (s.mask * env) * (dot(p.rd, a.sky.sun) < 0.99f ? 1.0f : 0.0f);
            return false;
        }
        if (!sky) return false;
        // js/PhysicalSkyModel_FragmentShader.js:155-189 (also the sky composite's; with diffuseCount == 0 the path is still
        // specular, so one of the five cases always ends it)
        const f3 skyc = skyColor(a.sky, p.rd);
        if (bounces == 0) { g.setSharp(1.01f); accum = skyc; }
        else if (s.diffuseCount == 0 && s.specular) { g.setSharp(1.01f); accum = s.mask * skyc; }
        else if (s.sampleLight) accum = s.mask * skyc;
        else if (s.diffuseCount == 1 && prevType == TRANSPARENT && s.specular) accum = s.mask * skyc;
        else if (s.diffuseCount > 0) accum = (s.mask * skyc) * (dot(p.rd, a.sky.sun) < 0.99f ? 1.0f : 0.0f);
        return false;
    }
    f3 n = normalize(h.normal);
    f3 nl = dot(n, p.rd) < 0.0f ? normalize(n) : normalize(-n);
    f3 x = p.ro + p.rd * h.t;
    if (bounces == 0) { g.setNrm(nl); g.setCol(h.color); g.setId((float)h.id); }
    if (bounces == 1 && prevType == METAL) {
        if constexpr (G::kColById) {   // objectColor stays bounce 0's: keep it before the id changes
            f3 c0 = mk(0.0f, 0.0f, 0.0f);
            int t0;
            objectMaterial<PROG>(a, (int)g.id(), c0, t0);
            g.pinCol(c0);
        }
        g.setNrm(nl); g.setId((float)h.id);
    }

    if (!sky && !hdri && hitType == LIGHT) {   // (commented out / removed in the sky and HDRI shaders)
        if (s.diffuseCount == 0) g.setSharp(1.01f);
        if (s.specular || s.sampleLight) accum = s.mask * h.color;
        return false;
    }
    if (s.sampleLight) return false;

    if (kHasTex<PROG> && gltf && hitType == PBR_MATERIAL) {   // (the sky radiance has no PBR decode)
        float tx[4];
        texBilinear(a.albedo, h.u, h.v, tx);
        if (COUNT) cnt.tap += 4;
        h.color = pow22(mk(tx[0], tx[1], tx[2]));
        f3 emission = mk(0, 0, 0);
        if (a.uses_emissive) { texBilinear(a.emissive, h.u, h.v, tx); if (COUNT) cnt.tap += 4; emission = mk(tx[0], tx[1], tx[2]); }
        emission = pow22(emission);
        float maxE = gmax(emission.x, gmax(emission.y, emission.z));
        if (s.specular && maxE > 0.01f) { g.setSharp(1.01f); accum = s.mask * emission; return false; }
        hitType = DIFFUSE;
        f3 mr = mk(0, 0, 0);
        if (a.uses_metal) { texBilinear(a.metal, h.u, h.v, tx); if (COUNT) cnt.tap += 4; mr = mk(tx[0], tx[1], tx[2]); }
        mr = pow22(mr);
        s.roughness = mr.y;
        if (mr.y > 0.01f) hitType = CLEARCOAT_DIFFUSE;
        if (mr.z > 0.01f) hitType = METAL;
        s.hitType = hitType;
    }

    const bool more = bounces + 1 < 6;
    s.bounce = bounces + 1;
    bool diffuseTail = hitType == DIFFUSE;
    if (hitType == TRANSPARENT || hitType == CLEARCOAT_DIFFUSE) {
        const bool glass = hitType == TRANSPARENT;
        if (glass) {
            if (s.diffuseCount == 0 && !s.coat && !a.moving) g.setSharp(1.01f);
            else if (s.diffuseCount > 0) g.setSharp(0.0f);
            else g.setSharp(-1.0f);
        } else {
            s.coat = true;
            g.setSharp(0.0f);
        }
        float ratio;
        float Re = fresnel(p.rd, glass ? n : nl, 1.0f, glass ? 1.5f : 1.4f, ratio);
        float Tr = 1.0f - Re;
        float P = 0.25f + (0.5f * Re);
        float RP = Re / P, TP = Tr / (1.0f - P);
        if (blueNoise_rand(p) < P) {            // specular reflection off the interface
            if (!glass && s.diffuseCount == 0) g.setSharp(a.frame > 500.0f ? 1.01f : -1.0f);
            s.mask = s.mask * RP;
            p.rd = reflect(p.rd, nl);
            p.ro = x + nl * a.eps;
            return more;
        }
        if (glass) {                             // refraction through the dielectric
            if (kIsQuadric<PROG>) {              // no absorption, a colour filter (:470-471)
                s.mask = s.mask * TP;
                s.mask = s.mask * h.color;
            } else {
                if (distance(n, nl) > 0.1f) {
                    const float thickness = 0.01f;
                    f3 cc = clamp3(h.color, 0.01f, 0.99f);
                    s.mask = s.mask * mk(gexp(glog(cc.x) * thickness * h.t), gexp(glog(cc.y) * thickness * h.t),
                                         gexp(glog(cc.z) * thickness * h.t));
                }
                s.mask = s.mask * TP;
            }
            p.rd = refract(p.rd, nl, ratio);
            p.ro = x - nl * a.eps;
            if (s.diffuseCount == 1) s.specular = true;
            return more;
        }
        s.mask = s.mask * TP;                    // clear coat transmits into its diffuse base
        diffuseTail = true;
    }
    if (diffuseTail) {
        s.diffuseCount++;
        s.mask = s.mask * h.color;
        s.specular = false;
        if ((hdri ? s.diffuseCount <= 2 : s.diffuseCount == 1) && blueNoise_rand(p) < 0.5f) {
            p.rd = cosWeightedDir(p, nl);
        } else if (hdri) {   // shadow ray into the sun's lobe (js/HDRIEnvironmentPathTracing_FragmentShader.js:395-400)
            p.rd = specularLobeDir(p, a.sky.sun, 0.03f);
            s.mask = s.mask * (gmax(0.0f, dot(p.rd, nl)) * a.sun_weight);
            if (hitType == DIFFUSE || bounces < 3) s.sampleLight = true;
        } else if (sky) {   // shadow ray into the sun's lobe (js/PhysicalSkyModel_FragmentShader.js:237-243)
            p.rd = specularLobeDir(p, a.sky.sun, 0.1f);
            s.mask = s.mask * (gmax(0.0f, dot(p.rd, nl)) * 0.05f);
            if (hitType == DIFFUSE || bounces < 3) s.sampleLight = true;
        } else {
            float w;
            f3 dl = sampleQuadLight(p, a, x, nl, w);
            s.mask = s.mask * w;
            p.rd = dl;
            if (hitType == DIFFUSE || bounces < 3) s.sampleLight = true;
        }
        p.ro = x + nl * a.eps;
        return more;
    }
    if (hitType == METAL) {
        s.mask = s.mask * h.color;
        if (gltf) p.rd = specularLobeDir(p, reflect(p.rd, nl), s.roughness);
        else p.rd = reflect(p.rd, nl);
        p.ro = x + nl * a.eps;
    }
    return more;   // any other hitType: the GLSL loop continues with the ray unchanged
}

// main()'s camera ray for pixel (px, py) (js/PathTracingCommon.js:1259-1292)
PT_D void cameraRay(const TraceArgs& a, int px, int py, Path& p)
{
    const float* m = a.cam.m;
    f3 camRight = mk(m[0], m[1], m[2]), camUp = mk(m[4], m[5], m[6]), camFwd = mk(m[8], m[9], m[10]);
    f3 camPos = mk(m[12], m[13], m[14]);
    float fcx = (float)px + 0.5f, fcy = (float)py + 0.5f;
    p.s0 = (uint32_t)a.frame * (uint32_t)fcx;
    p.s1 = (uint32_t)(a.frame + 1.0f) * (uint32_t)fcy;
    int bx = (int)gmod(fcx + floorf(a.rnd[0] * 256.0f), 256.0f);
    int by = (int)gmod(fcy + floorf(a.rnd[1] * 256.0f), 256.0f);
    p.bn = 0u;   // counter = -1.0; randVec4 = 0 outside the texture (pinned)
    if (bx < a.bluenoise.w && by < a.bluenoise.h) {
        uchar4 b = a.bluenoise.p[by * a.bluenoise.w + bx];
        p.bn = (unsigned)b.x | ((unsigned)b.y << 8);
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
}


} // namespace pt
