/* oracle/ptoracle.c — TEST INFRASTRUCTURE (CPU oracle; see ptoracle.h).
 *
 * A scalar C restatement of the reference's per-pixel path-tracing fragment program, following
 * the GLSL line by line with the pinned built-in semantics of glsl_pinned.h:
 *   main()                      js/PathTracingCommon.js:1251-1358
 *   rng / blueNoise_rand        js/PathTracingCommon.js:485-508
 *   cos-weighted / lobe dirs    js/PathTracingCommon.js:518-543;  tentFilter :546-549
 *   calcFresnelReflectance      js/PathTracingCommon.js:556-575
 *   sampleAxisAlignedQuadLight  js/PathTracingCommon.js:582-597
 *   solveQuadratic / UnitSphere js/PathTracingCommon.js:631-641, 664-685
 *   Triangle/QuadIntersect      js/PathTracingCommon.js:1168-1187
 *   BoundingBoxIntersect        js/PathTracingCommon.js:1194-1207
 *   BVH_(DoubleSided)Triangle   js/PathTracingCommon.js:1214-1245
 *   screenOutput                js/PathTracingCommon.js:19-309
 *   Cornell scene               js/BabylonPathTracing_FragmentShader.js:47-378
 *   glTF scene                  js/GLTFModelPathTracing_FragmentShader.js:72-643
 * Pinned choices where the GLSL is implementation-defined: unwritten `out`
 * parameters read as 0; fine 2x2-quad derivatives; texelFetch outside the target returns 0;
 * implicit-LOD texture() = LOD 0 bilinear, REPEAT; unorm8 = b/255; canvas u8 = floor(255c+0.5).
 */
#include "ptoracle.h"
#include "glsl_pinned.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define INFINITY_G 1000000.0f
#define TWO_PI_G 6.28318530717958648f

enum { LIGHT = 0, DIFFUSE = 1, TRANSPARENT = 2, METAL = 3, CLEARCOAT_DIFFUSE = 4, PBR_MATERIAL = 10 };

typedef struct { v3 normal, v0, v1, v2, v3_, color; int type; } Quad;
typedef struct { v3 color; int type; } UnitSphere;

/* per-invocation state (the GLSL globals) */
typedef struct {
    const pto_frame* f;
    uint32_t seed[2];
    float counter;
    float randVec4[4];
    Quad quads[6];
    int nquads;
    UnitSphere spheres[2];
    v3 rayOrigin, rayDirection;
    pto_counters c;
} Inv;

/* ---------------------------------------------------------------- random */
static float rng(Inv* s)
{
    s->seed[0] += 1u; s->seed[1] += 1u;
    uint32_t qx = 1103515245u * ((s->seed[0] >> 1u) ^ s->seed[1]);
    uint32_t qy = 1103515245u * ((s->seed[1] >> 1u) ^ s->seed[0]);
    uint32_t n = 1103515245u * (qx ^ (qy >> 3u));
    return (float)n * (1.0f / 4294967296.0f);
}
static float blueNoise_rand(Inv* s)
{
    s->counter = s->counter + 1.0f;
    int channel = (int)g_mod(s->counter, 2.0f);
    return g_fract(s->randVec4[channel]);
}
static float tentFilter(float x)
{
    return (x < 0.5f) ? sqrtf(2.0f * x) - 1.0f : 1.0f - sqrtf(2.0f - (2.0f * x));
}
static v3 onb_u(v3 nl)
{
    v3 a = (fabsf(nl.y) < 0.9f) ? V3(0.0f, 1.0f, 0.0f) : V3(1.0f, 0.0f, 0.0f);
    return v_normalize(v_cross(a, nl));
}
static v3 randomCosWeightedDirectionInHemisphere(Inv* s, v3 nl)
{
    float r = sqrtf(rng(s));
    float phi = rng(s) * TWO_PI_G;
    float x = r * g_cos(phi);
    float y = r * g_sin(phi);
    float z = sqrtf(1.0f - x * x - y * y);
    v3 U = onb_u(nl);
    v3 V = v_cross(nl, U);
    return v_normalize(v_add(v_add(v_muls(U, x), v_muls(V, y)), v_muls(nl, z)));
}
static v3 randomDirectionInSpecularLobe(Inv* s, v3 reflectionDir, float roughness)
{
    roughness = g_clamp(roughness, 0.0f, 1.0f);
    float exponent = g_mix(7.0f, 0.0f, sqrtf(roughness));
    float cosTheta = g_pow(rng(s), 1.0f / (g_exp(exponent) + 1.0f));
    float sinTheta = sqrtf(g_max(0.0f, 1.0f - cosTheta * cosTheta));
    float phi = rng(s) * TWO_PI_G;
    v3 U = onb_u(reflectionDir);
    v3 V = v_cross(reflectionDir, U);
    v3 lobe = v_add(v_add(v_muls(v_muls(U, g_cos(phi)), sinTheta), v_muls(v_muls(V, g_sin(phi)), sinTheta)),
                    v_muls(reflectionDir, cosTheta));
    return v_normalize(v_mix(reflectionDir, lobe, roughness));
}

/* ---------------------------------------------------------------- materials / lights */
static float calcFresnelReflectance(v3 rayDirection, v3 n, float etai, float etat, float* ratioIoR)
{
    float temp = etai;
    float cosi = g_clamp(v_dot(rayDirection, n), -1.0f, 1.0f);
    if (cosi > 0.0f) { etai = etat; etat = temp; }
    *ratioIoR = etai / etat;
    float sint = *ratioIoR * sqrtf(1.0f - (cosi * cosi));
    if (sint >= 1.0f) return 1.0f;
    float cost = sqrtf(1.0f - (sint * sint));
    cosi = fabsf(cosi);
    float Rs = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    float Rp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return g_clamp(((Rs * Rs) + (Rp * Rp)) * 0.5f, 0.0f, 1.0f);
}
static v3 sampleAxisAlignedQuadLight(Inv* s, v3 x, v3 nl, const Quad* light, float* weight)
{
    v3 p;
    p.x = g_mix(light->v0.x, light->v2.x, g_clamp(rng(s), 0.1f, 0.9f));
    p.y = g_mix(light->v0.y, light->v2.y, g_clamp(rng(s), 0.1f, 0.9f));
    p.z = g_mix(light->v0.z, light->v2.z, g_clamp(rng(s), 0.1f, 0.9f));
    v3 dirToLight = v_sub(p, x);
    float r2 = v_distance(light->v0, light->v1) * v_distance(light->v0, light->v3_);
    float d2 = v_dot(dirToLight, dirToLight);
    float cos_a_max = sqrtf(1.0f - g_clamp(r2 / d2, 0.0f, 1.0f));
    dirToLight = v_normalize(dirToLight);
    float dotNlRayDir = g_max(0.0f, v_dot(nl, dirToLight));
    float w = 2.0f * (1.0f - cos_a_max) * g_max(0.0f, -v_dot(dirToLight, light->normal)) * dotNlRayDir;
    *weight = g_clamp(w, 0.0f, 1.0f);
    return dirToLight;
}

/* ---------------------------------------------------------------- intersectors */
static void solveQuadratic(float A, float B, float C, float* t0, float* t1)
{
    float invA = 1.0f / A;
    B *= invA;
    C *= invA;
    float neg_halfB = -B * 0.5f;
    float u2 = neg_halfB * neg_halfB - C;
    float u;
    if (u2 < 0.0f) { neg_halfB = 0.0f; u = 0.0f; } else u = sqrtf(u2);
    *t0 = neg_halfB - u;
    *t1 = neg_halfB + u;
}
static float UnitSphereIntersect(v3 ro, v3 rd, v3* n)
{
    float t0, t1;
    float a = v_dot(rd, rd);
    float b = 2.0f * v_dot(rd, ro);
    float c = v_dot(ro, ro) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    if (t0 > 0.0f) { v3 h = v_add(ro, v_muls(rd, t0)); *n = V3(2.0f * h.x, 2.0f * h.y, 2.0f * h.z); return t0; }
    if (t1 > 0.0f) { v3 h = v_add(ro, v_muls(rd, t1)); *n = V3(2.0f * h.x, 2.0f * h.y, 2.0f * h.z); return t1; }
    return INFINITY_G;
}
static float TriangleIntersect(v3 v0, v3 v1, v3 v2, v3 ro, v3 rd, int dbl)
{
    v3 edge1 = v_sub(v1, v0), edge2 = v_sub(v2, v0);
    v3 pvec = v_cross(rd, edge2);
    float det = 1.0f / v_dot(edge1, pvec);
    if (!dbl && det < 0.0f) return INFINITY_G;
    v3 tvec = v_sub(ro, v0);
    float u = v_dot(tvec, pvec) * det;
    v3 qvec = v_cross(tvec, edge1);
    float v = v_dot(rd, qvec) * det;
    float t = v_dot(edge2, qvec) * det;
    return (u < 0.0f || u > 1.0f || v < 0.0f || u + v > 1.0f || t <= 0.0f) ? INFINITY_G : t;
}
static float QuadIntersect(const Quad* q, v3 ro, v3 rd)
{
    return g_min(TriangleIntersect(q->v0, q->v1, q->v2, ro, rd, 0), TriangleIntersect(q->v0, q->v2, q->v3_, ro, rd, 0));
}
static float BoundingBoxIntersect(v3 mn, v3 mx, v3 ro, v3 invDir)
{
    v3 near_ = v_mul(v_sub(mn, ro), invDir);
    v3 far_ = v_mul(v_sub(mx, ro), invDir);
    v3 tmin = V3(g_min(near_.x, far_.x), g_min(near_.y, far_.y), g_min(near_.z, far_.z));
    v3 tmax = V3(g_max(near_.x, far_.x), g_max(near_.y, far_.y), g_max(near_.z, far_.z));
    float t0 = g_max(g_max(tmin.x, tmin.y), tmin.z);
    float t1 = g_min(g_min(tmax.x, tmax.y), tmax.z);
    return g_max(t0, 0.0f) > t1 ? INFINITY_G : t0;
}
static float BVH_TriangleIntersect(v3 v0, v3 v1, v3 v2, v3 ro, v3 rd, float* u, float* v, int dbl)
{
    v3 edge1 = v_sub(v1, v0), edge2 = v_sub(v2, v0);
    v3 pvec = v_cross(rd, edge2);
    float det = 1.0f / v_dot(edge1, pvec);
    v3 tvec = v_sub(ro, v0);
    *u = v_dot(tvec, pvec) * det;
    v3 qvec = v_cross(tvec, edge1);
    *v = v_dot(rd, qvec) * det;
    float t = v_dot(edge2, qvec) * det;
    if (dbl)
        return (*u < 0.0f || *u > 1.0f || *v < 0.0f || *u + *v > 1.0f || t <= 0.0f) ? INFINITY_G : t;
    return (det < 0.0f || *u < 0.0f || *u > 1.0f || *v < 0.0f || *u + *v > 1.0f || t <= 0.0f) ? INFINITY_G : t;
}

/* ---------------------------------------------------------------- transformed quadrics */
/* js/PathTracingCommon.js:690-1163: unit shapes in object space (the scene transforms the ray by
 * each shape's inverse matrix). Expression order follows the GLSL exactly. */
static v3 qhit(v3 ro, v3 rd, float t) { return v_add(ro, v_muls(rd, t)); }
static float g_sign(float x) { return x > 0.0f ? 1.0f : x < 0.0f ? -1.0f : 0.0f; }
static float g_step(float edge, float x) { return x < edge ? 0.0f : 1.0f; }

static float UnitCylinderIntersect(v3 ro, v3 rd, v3* n)
{
    float t0, t1;
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t0; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t1; }
    return INFINITY_G;
}
static float UnitConeIntersect(v3 ro, v3 rd, float k, v3* n)
{
    float t0, t1;
    k = g_clamp(k, 0.01f, 1.0f);
    float j = 1.0f / k;
    float h = j * 2.0f - 1.0f;
    float a = j * rd.x * rd.x + j * rd.z * rd.z - (k * 0.25f) * rd.y * rd.y;
    float b = 2.0f * (j * rd.x * ro.x + j * rd.z * ro.z - (k * 0.25f) * rd.y * (ro.y - h));
    float c = j * ro.x * ro.x + j * ro.z * ro.z - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x * j, 2.0f * (h - hit.y) * (k * 0.25f), 2.0f * hit.z * j); return t0; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x * j, 2.0f * (h - hit.y) * (k * 0.25f), 2.0f * hit.z * j); return t1; }
    return INFINITY_G;
}
static float UnitParaboloidIntersect(v3 ro, v3 rd, v3* n)
{
    float t0, t1;
    float k = 0.5f;
    float a = rd.x * rd.x + rd.z * rd.z;
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z) + k * rd.y;
    float c = ro.x * ro.x + ro.z * ro.z + k * (ro.y - 1.0f);
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.5f, 2.0f * hit.z); return t0; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.5f, 2.0f * hit.z); return t1; }
    return INFINITY_G;
}
static float UnitHyperboloidIntersect(v3 ro, v3 rd, float k, v3* n)
{
    float t0, t1;
    k = k * k * k * k + 0.0012f;
    k *= 1000.0f;
    float j = k - 1.0f;
    float a = k * rd.x * rd.x + k * rd.z * rd.z - j * rd.y * rd.y;
    float b = 2.0f * (k * rd.x * ro.x + k * rd.z * ro.z - j * rd.y * ro.y);
    float c = (k * ro.x * ro.x + k * ro.z * ro.z - j * ro.y * ro.y) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x * k, 2.0f * -hit.y * j, 2.0f * hit.z * k); return t0; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x * k, 2.0f * -hit.y * j, 2.0f * hit.z * k); return t1; }
    return INFINITY_G;
}
static float UnitCapsuleIntersect(v3 ro, v3 rd, float k, v3* n)
{
    k += 0.25f;
    float t0, t1, s0t0, s0t1, s1t0, s1t1;
    v3 L = v_sub(ro, V3(0.0f, k, 0.0f));
    float a = v_dot(rd, rd);
    float b = 2.0f * v_dot(rd, L);
    float c = v_dot(L, L) - 1.0f;
    solveQuadratic(a, b, c, &s0t0, &s0t1);
    v3 hit = qhit(ro, rd, s0t0);
    if (s0t0 > 0.0f && hit.y >= k) { *n = V3(2.0f * hit.x, 2.0f * (hit.y - k), 2.0f * hit.z); return s0t0; }
    L = v_sub(ro, V3(0.0f, -k, 0.0f));
    a = v_dot(rd, rd);
    b = 2.0f * v_dot(rd, L);
    c = v_dot(L, L) - 1.0f;
    solveQuadratic(a, b, c, &s1t0, &s1t1);
    hit = qhit(ro, rd, s1t0);
    if (s1t0 > 0.0f && hit.y <= -k) { *n = V3(2.0f * hit.x, 2.0f * (hit.y + k), 2.0f * hit.z); return s1t0; }
    a = (rd.x * rd.x + rd.z * rd.z);
    b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= k) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t0; }
    hit = qhit(ro, rd, s0t1);
    if (s0t1 > 0.0f && hit.y >= k) { *n = V3(2.0f * hit.x, 2.0f * (hit.y - k), 2.0f * hit.z); return s0t1; }
    hit = qhit(ro, rd, s1t1);
    if (s1t1 > 0.0f && hit.y <= -k) { *n = V3(2.0f * hit.x, 2.0f * (hit.y + k), 2.0f * hit.z); return s1t1; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= k) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t1; }
    return INFINITY_G;
}
static float UnitFlattenedRingIntersect(v3 ro, v3 rd, float k, v3* n)
{
    k -= 0.01f;
    float t0, t1, c0, c1;
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit = qhit(ro, rd, t0);
    if (t0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t0; }
    float d0 = (ro.y - 1.0f) / -rd.y;
    hit = qhit(ro, rd, d0);
    float x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y < 0.0f && d0 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { *n = V3(0.0f, 1.0f, 0.0f); return d0; }
    float d1 = (ro.y + 1.0f) / -rd.y;
    hit = qhit(ro, rd, d1);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y > 0.0f && d1 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { *n = V3(0.0f, -1.0f, 0.0f); return d1; }
    c = (ro.x * ro.x + ro.z * ro.z) - k;
    solveQuadratic(a, b, c, &c0, &c1);
    hit = qhit(ro, rd, c0);
    if (c0 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return c0; }
    hit = qhit(ro, rd, c1);
    if (c1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return c1; }
    hit = qhit(ro, rd, t1);
    if (t1 > 0.0f && fabsf(hit.y) <= 1.0f) { *n = V3(2.0f * hit.x, 0.0f, 2.0f * hit.z); return t1; }
    hit = qhit(ro, rd, d0);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y > 0.0f && d0 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { *n = V3(0.0f, 1.0f, 0.0f); return d0; }
    hit = qhit(ro, rd, d1);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y < 0.0f && d1 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { *n = V3(0.0f, -1.0f, 0.0f); return d1; }
    return INFINITY_G;
}
static float UnitBoxIntersect(v3 ro, v3 rd, v3* n)
{
    v3 invDir = V3(1.0f / rd.x, 1.0f / rd.y, 1.0f / rd.z);
    v3 nr = v_mul(v_sub(V3(-1.0f, -1.0f, -1.0f), ro), invDir);
    v3 fr = v_mul(v_sub(V3(1.0f, 1.0f, 1.0f), ro), invDir);
    v3 tmin = V3(g_min(nr.x, fr.x), g_min(nr.y, fr.y), g_min(nr.z, fr.z));
    v3 tmax = V3(g_max(nr.x, fr.x), g_max(nr.y, fr.y), g_max(nr.z, fr.z));
    float t0 = g_max(g_max(tmin.x, tmin.y), tmin.z);
    float t1 = g_min(g_min(tmax.x, tmax.y), tmax.z);
    if (t0 < t1) {
        if (t0 > 0.0f) {   /* -sign(rd) * step(tmin.yzx, tmin) * step(tmin.zxy, tmin) */
            *n = V3(-g_sign(rd.x) * g_step(tmin.y, tmin.x) * g_step(tmin.z, tmin.x),
                    -g_sign(rd.y) * g_step(tmin.z, tmin.y) * g_step(tmin.x, tmin.y),
                    -g_sign(rd.z) * g_step(tmin.x, tmin.z) * g_step(tmin.y, tmin.z));
            return t0;
        }
        if (t1 > 0.0f) {   /* -sign(rd) * step(tmax, tmax.yzx) * step(tmax, tmax.zxy) */
            *n = V3(-g_sign(rd.x) * g_step(tmax.x, tmax.y) * g_step(tmax.x, tmax.z),
                    -g_sign(rd.y) * g_step(tmax.y, tmax.z) * g_step(tmax.y, tmax.x),
                    -g_sign(rd.z) * g_step(tmax.z, tmax.x) * g_step(tmax.z, tmax.y));
            return t1;
        }
    }
    return INFINITY_G;
}
static float PyramidFrustumIntersect(v3 ro, v3 rd, float k, v3* n)
{
    float xt0, xt1, zt0, zt1;
    float xt = INFINITY_G, zt = INFINITY_G;
    v3 hit0, hit1, xn = V3(0, 0, 0), zn = V3(0, 0, 0);
    k = g_clamp(k, 0.01f, 1.0f);
    float j = 1.0f / k;
    float h = j * 2.0f - 1.0f;
    float a = j * rd.x * rd.x - (k * 0.25f) * rd.y * rd.y;
    float b = 2.0f * (j * rd.x * ro.x - (k * 0.25f) * rd.y * (ro.y - h));
    float c = j * ro.x * ro.x - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    solveQuadratic(a, b, c, &xt0, &xt1);
    hit0 = qhit(ro, rd, xt0);
    hit1 = qhit(ro, rd, xt1);
    if (xt0 > 0.0f && fabsf(hit0.x) <= 1.0f && fabsf(hit0.z) <= 1.0f && hit0.y <= 1.0f &&
        (j * hit0.z * hit0.z - k * 0.25f * (hit0.y - h) * (hit0.y - h)) <= 0.0f) {
        xt = xt0;
        xn = V3(2.0f * hit0.x * j, 2.0f * (hit0.y - h) * -(k * 0.25f), 0.0f);
    } else if (xt1 > 0.0f && fabsf(hit1.x) <= 1.0f && fabsf(hit1.z) <= 1.0f && hit1.y <= 1.0f &&
               (j * hit1.z * hit1.z - k * 0.25f * (hit1.y - h) * (hit1.y - h)) <= 0.0f) {
        xt = xt1;
        xn = V3(2.0f * hit1.x * j, 2.0f * (hit1.y - h) * -(k * 0.25f), 0.0f);
    }
    a = j * rd.z * rd.z - (k * 0.25f) * rd.y * rd.y;
    b = 2.0f * (j * rd.z * ro.z - (k * 0.25f) * rd.y * (ro.y - h));
    c = j * ro.z * ro.z - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    solveQuadratic(a, b, c, &zt0, &zt1);
    hit0 = qhit(ro, rd, zt0);
    hit1 = qhit(ro, rd, zt1);
    if (zt0 > 0.0f && fabsf(hit0.x) <= 1.0f && fabsf(hit0.z) <= 1.0f && hit0.y <= 1.0f &&
        (j * hit0.x * hit0.x - k * 0.25f * (hit0.y - h) * (hit0.y - h)) <= 0.0f) {
        zt = zt0;
        zn = V3(0.0f, 2.0f * (hit0.y - h) * -(k * 0.25f), 2.0f * hit0.z * j);
    } else if (zt1 > 0.0f && fabsf(hit1.x) <= 1.0f && fabsf(hit1.z) <= 1.0f && hit1.y <= 1.0f &&
               (j * hit1.x * hit1.x - k * 0.25f * (hit1.y - h) * (hit1.y - h)) <= 0.0f) {
        zt = zt1;
        zn = V3(0.0f, 2.0f * (hit1.y - h) * -(k * 0.25f), 2.0f * hit1.z * j);
    }
    if (xt <= zt) { *n = xn; return xt; }
    *n = zn;
    return zt;
}
static float UnitDiskIntersect(v3 ro, v3 rd)
{
    float t0 = (ro.y + 0.0f) / -rd.y;
    v3 hit = qhit(ro, rd, t0);
    return (t0 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? t0 : INFINITY_G;
}
static float UnitRectangleIntersect(v3 ro, v3 rd)
{
    float t0 = (ro.y + 0.0f) / -rd.y;
    v3 hit = qhit(ro, rd, t0);
    return (t0 > 0.0f && fabsf(hit.x) <= 1.0f && fabsf(hit.z) <= 1.0f) ? t0 : INFINITY_G;
}
static float map_Torus(v3 pos, float k)
{
    float a = sqrtf(pos.x * pos.x + pos.z * pos.z) - (1.0f - k);
    return sqrtf(a * a + pos.y * pos.y) - k;
}
static float UnitTorusIntersect(v3 ro, v3 rd, float k, v3* n)
{
    k = 1.0f - g_clamp(k, 0.01f, 0.99f);
    float d = INFINITY_G;
    float tc, t0, t1;
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    solveQuadratic(a, b, c, &t0, &t1);
    v3 hit0 = qhit(ro, rd, t0), hit1 = qhit(ro, rd, t1);
    tc = (t0 > 0.0f && fabsf(hit0.y) <= k) ? t0 : (t1 > 0.0f && fabsf(hit1.y) <= k) ? t1 : INFINITY_G;
    float d0 = (ro.y + k) / -rd.y;
    v3 hit = qhit(ro, rd, d0);
    d0 = (d0 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? d0 : INFINITY_G;
    float d1 = (ro.y - k) / -rd.y;
    hit = qhit(ro, rd, d1);
    d1 = (d1 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? d1 : INFINITY_G;
    if (tc == INFINITY_G && d0 == INFINITY_G && d1 == INFINITY_G) return INFINITY_G;
    v3 pos = V3(0, 0, 0);
    float t = g_min(g_min(d0, d1), tc);
    for (int i = 0; i < 500; i++) {
        pos = qhit(ro, rd, t);
        d = map_Torus(pos, k);
        if (fabsf(d) < 0.01f) break;
        t += d;
    }
    if (fabsf(d) < 0.01f) {
        float ex = (1.0f * 0.5773f) * 0.0002f, ey = (-1.0f * 0.5773f) * 0.0002f;
        v3 s = v_muls(V3(ex, ey, ey), map_Torus(v_add(pos, V3(ex, ey, ey)), k));
        s = v_add(s, v_muls(V3(ey, ey, ex), map_Torus(v_add(pos, V3(ey, ey, ex)), k)));
        s = v_add(s, v_muls(V3(ey, ex, ey), map_Torus(v_add(pos, V3(ey, ex, ey)), k)));
        s = v_add(s, v_muls(V3(ex, ex, ex), map_Torus(v_add(pos, V3(ex, ex, ex)), k)));
        *n = v_normalize(s);
        return t;
    }
    return INFINITY_G;
}

/* ---------------------------------------------------------------- textures */
static const float* texel32(const float* base, int64_t n, float idx)
{
    /* the GLSL computes ivec2(mod(i, 2048.0), i * (1/2048)); for i < 2^24 that is texel i */
    static const float zero4[4] = { 0, 0, 0, 0 };
    if (!(idx >= 0.0f) || !(idx < (float)n)) return zero4;
    return base + 4 * (int64_t)idx;
}
static float unorm8(uint8_t b) { return (float)b / 255.0f; }
/* texture(sampler, uv) on an RGBA8 map: LOD 0 bilinear, REPEAT wrap, unorm8 texels */
static int wrap_texel(float f, int n)
{
    float r = fmodf(f, (float)n);   /* exact */
    if (!(r == r)) r = 0.0f;         /* NaN / inf coordinates wrap to texel 0 (pinned) */
    int i = (int)r;
    return i < 0 ? i + n : i;
}
static void tex_bilinear(const uint8_t* t, int w, int h, float u, float v, float out[4])
{
    if (!t || w <= 0 || h <= 0) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float a = x - fx, b = y - fy;
    int64_t x0 = wrap_texel(fx, w), y0 = wrap_texel(fy, h);
    int64_t x1 = (x0 + 1) % w, y1 = (y0 + 1) % h;
    for (int c = 0; c < 4; c++) {
        float t00 = unorm8(t[4 * (y0 * w + x0) + c]), t10 = unorm8(t[4 * (y0 * w + x1) + c]);
        float t01 = unorm8(t[4 * (y1 * w + x0) + c]), t11 = unorm8(t[4 * (y1 * w + x1) + c]);
        out[c] = g_mix(g_mix(t00, t10, a), g_mix(t01, t11, a), b);
    }
}

/* texture(sampler, uv) on an RGBA32F map (tHDRTexture): LOD 0 bilinear, REPEAT wrap */
static void tex_bilinear_f(const float* t, int w, int h, float u, float v, float out[4])
{
    if (!t || w <= 0 || h <= 0) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float ax = x - fx, by = y - fy;
    int x0 = wrap_texel(fx, w), y0 = wrap_texel(fy, h);
    int x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
    const float* t00 = t + 4 * ((size_t)y0 * w + x0);
    const float* t10 = t + 4 * ((size_t)y0 * w + x1);
    const float* t01 = t + 4 * ((size_t)y1 * w + x0);
    const float* t11 = t + 4 * ((size_t)y1 * w + x1);
    for (int k = 0; k < 4; k++) out[k] = g_mix(g_mix(t00[k], t10[k], ax), g_mix(t01[k], t11[k], ax), by);
}

/* ---------------------------------------------------------------- scene setup */
static Quad mkquad(v3 n, v3 a, v3 b, v3 c, v3 d, v3 col, int type)
{
    Quad q; q.normal = n; q.v0 = a; q.v1 = b; q.v2 = c; q.v3_ = d; q.color = col; q.type = type; return q;
}
static void SetupScene(Inv* s)
{
    const pto_frame* f = s->f;
    const int sky = f->scene == PTO_SCENE_SKY || f->scene == PTO_SCENE_SKYMESH;
    if (sky || f->scene == PTO_SCENE_HDRI) {
        /* js/PhysicalSkyModel_FragmentShader.js:383-399 and
         * js/HDRIEnvironmentPathTracing_FragmentShader.js:529-542: N_QUADS 4 (no ceiling, no quad light) */
        float W = 50.0f;
        s->spheres[0].color = V3(1.0f, 1.0f, 0.0f); s->spheres[0].type = CLEARCOAT_DIFFUSE;
        s->spheres[1].color = V3(1.0f, 1.0f, 1.0f);
        s->spheres[1].type = sky ? f->uRightSphereMatType : METAL;
        s->quads[0] = mkquad(V3(0, 0, 1), V3(-W, W, W), V3(W, W, W), V3(W, -W, W), V3(-W, -W, W), V3(1.0f, 1.0f, 1.0f), DIFFUSE);
        s->quads[1] = mkquad(V3(1, 0, 0), V3(-W, -W, W), V3(-W, -W, -W), V3(-W, W, -W), V3(-W, W, W), V3(0.7f, 0.05f, 0.05f), DIFFUSE);
        s->quads[2] = mkquad(V3(-1, 0, 0), V3(W, -W, -W), V3(W, -W, W), V3(W, W, W), V3(W, W, -W), V3(0.05f, 0.05f, 0.7f), DIFFUSE);
        s->quads[3] = mkquad(V3(0, 1, 0), V3(-W, -W, W), V3(W, -W, W), V3(W, -W, -W), V3(-W, -W, -W), V3(1.0f, 1.0f, 1.0f), DIFFUSE);
        s->nquads = 4;
        return;
    }
    s->nquads = 6;
    v3 light_emissionColor = v_muls(V3(1.0f, 1.0f, 1.0f), 10.0f);
    float wallRadius = 50.0f;
    float lightRadius = f->uQuadLightRadius * 0.2f;
    float W = wallRadius, L = lightRadius;
    s->spheres[0].color = V3(1.0f, 1.0f, 0.0f); s->spheres[0].type = CLEARCOAT_DIFFUSE;
    s->spheres[1].color = V3(1.0f, 1.0f, 1.0f);
    s->spheres[1].type = f->scene == PTO_SCENE_CORNELL ? f->uRightSphereMatType : METAL;
    s->quads[0] = mkquad(V3(0, 0, 1), V3(-W, W, W), V3(W, W, W), V3(W, -W, W), V3(-W, -W, W), V3(1.0f, 1.0f, 1.0f), DIFFUSE);
    s->quads[1] = mkquad(V3(1, 0, 0), V3(-W, -W, W), V3(-W, -W, -W), V3(-W, W, -W), V3(-W, W, W), V3(0.7f, 0.05f, 0.05f), DIFFUSE);
    s->quads[2] = mkquad(V3(-1, 0, 0), V3(W, -W, -W), V3(W, -W, W), V3(W, W, W), V3(W, W, -W), V3(0.05f, 0.05f, 0.7f), DIFFUSE);
    s->quads[3] = mkquad(V3(0, -1, 0), V3(-W, W, -W), V3(W, W, -W), V3(W, W, W), V3(-W, W, W), V3(1.0f, 1.0f, 1.0f), DIFFUSE);
    s->quads[4] = mkquad(V3(0, 1, 0), V3(-W, -W, W), V3(W, -W, W), V3(W, -W, -W), V3(-W, -W, -W), V3(1.0f, 1.0f, 1.0f), DIFFUSE);
    float sel = f->uQuadLightPlaneSelectionNumber;
    float wm = W - 1.0f, wp = -W + 1.0f;
    memset(&s->quads[5], 0, sizeof(Quad)); /* unselected: GLSL global left at its zero default */
    if (sel == 1.0f)
        s->quads[5] = mkquad(V3(-1, 0, 0), V3(wm, -L, L), V3(wm, L, L), V3(wm, L, -L), V3(wm, -L, -L), light_emissionColor, LIGHT);
    else if (sel == 2.0f)
        s->quads[5] = mkquad(V3(1, 0, 0), V3(wp, -L, -L), V3(wp, L, -L), V3(wp, L, L), V3(wp, -L, L), light_emissionColor, LIGHT);
    else if (sel == 3.0f)
        s->quads[5] = mkquad(V3(0, 0, 1), V3(-L, -L, wp), V3(L, -L, wp), V3(L, L, wp), V3(-L, L, wp), light_emissionColor, LIGHT);
    else if (sel == 4.0f)
        s->quads[5] = mkquad(V3(0, 0, -1), V3(-L, -L, wm), V3(-L, L, wm), V3(L, L, wm), V3(L, -L, wm), light_emissionColor, LIGHT);
    else if (sel == 5.0f)
        s->quads[5] = mkquad(V3(0, 1, 0), V3(-L, wp, -L), V3(-L, wp, L), V3(L, wp, L), V3(L, wp, -L), light_emissionColor, LIGHT);
    else if (sel == 6.0f)
        s->quads[5] = mkquad(V3(0, -1, 0), V3(-L, wm, -L), V3(L, wm, -L), V3(L, wm, L), V3(-L, wm, L), light_emissionColor, LIGHT);
}

/* ---------------------------------------------------------------- glTF helpers */
static v3 perturbNormal(const pto_frame* f, v3 nl, float nsx, float nsy, float u, float v, pto_counters* c)
{
    v3 S = onb_u(nl);
    v3 T = v_cross(nl, S);
    v3 N = v_normalize(nl);
    v3 NfromST = v_cross(S, T);
    if (v_dot(NfromST, N) < 0.0f) { S = v_muls(S, -1.0f); T = v_muls(T, -1.0f); }
    float tx[4];
    tex_bilinear(f->bump, f->bumpW, f->bumpH, u, v, tx);
    c->rgba8_taps += 4;
    v3 mapN = V3(tx[0] * 2.0f - 1.0f, tx[1] * 2.0f - 1.0f, tx[2] * 2.0f - 1.0f);
    mapN = v_normalize(mapN);
    mapN.x *= nsx; mapN.y *= nsy;
    /* mat3(S, T, N) * mapN */
    v3 r = v_add(v_add(v_muls(S, mapN.x), v_muls(T, mapN.y)), v_muls(N, mapN.z));
    return v_normalize(r);
}

typedef struct {
    float t; v3 normal; v3 color; float u, v; int type; float objectID;
} Hit;

#define STACK_LEVELS 28

static void SceneIntersect(Inv* s, v3 rayOrigin, v3 rayDirection, Hit* h)
{
    const pto_frame* f = s->f;
    v3 n;
    float d;
    int objectCount = 0;
    s->c.segments++;
    h->t = INFINITY_G;
    h->type = -100;
    h->objectID = -INFINITY_G;
    if (f->scene == PTO_SCENE_QUADRIC) {
        /* js/TransformedQuadricGeometry_FragmentShader.js:77-317: twelve unit shapes, each behind its
         * inverse matrix, all of material uAllShapesMatType, then the Cornell quads */
        static const float col[12][3] = { { 1.0f, 0.0f, 0.0f }, { 0.0f, 1.0f, 0.0f }, { 1.0f, 1.0f, 0.0f }, { 1.0f, 0.0f, 1.0f },
                                          { 1.0f, 0.1f, 0.0f }, { 0.5f, 1.0f, 0.0f }, { 0.0f, 0.4f, 1.0f }, { 0.0f, 0.0f, 1.0f },
                                          { 0.2f, 0.0f, 1.0f }, { 0.0f, 1.0f, 0.5f }, { 1.0f, 0.3f, 0.0f }, { 0.5f, 0.0f, 1.0f } };
        for (int k = 0; k < 12; k++) {
            const float* M = f->uShapeInvMatrix[k];
            v3 ro = m4_mul(M, rayOrigin, 1.0f), rd = m4_mul(M, rayDirection, 0.0f);
            n = V3(0, 0, 0);
            switch (k) {
            case 0: d = UnitSphereIntersect(ro, rd, &n); break;
            case 1: d = UnitCylinderIntersect(ro, rd, &n); break;
            case 2: d = UnitConeIntersect(ro, rd, f->uShapeK, &n); break;
            case 3: d = UnitParaboloidIntersect(ro, rd, &n); break;
            case 4: d = UnitHyperboloidIntersect(ro, rd, f->uShapeK, &n); break;
            case 5: d = UnitCapsuleIntersect(ro, rd, f->uShapeK, &n); break;
            case 6: d = UnitFlattenedRingIntersect(ro, rd, f->uShapeK, &n); break;
            case 7: d = UnitBoxIntersect(ro, rd, &n); break;
            case 8: d = PyramidFrustumIntersect(ro, rd, f->uShapeK, &n); break;
            case 9: d = UnitDiskIntersect(ro, rd); break;
            case 10: d = UnitRectangleIntersect(ro, rd); break;
            default: d = UnitTorusIntersect(ro, rd, f->uShapeK, &n); break;
            }
            if (d < h->t) {
                h->t = d;
                /* disk and rectangle: hitNormal = vec3(0,-1,0), not normalized before the transform */
                h->normal = (k == 9 || k == 10) ? V3(0.0f, -1.0f, 0.0f) : v_normalize(n);
                h->normal = v_normalize(m3t_mul(M, h->normal));
                h->color = V3(col[k][0], col[k][1], col[k][2]);
                h->type = f->uAllShapesMatType;
                h->objectID = (float)objectCount;
            }
            objectCount++;
        }
        for (int i = 0; i < s->nquads; i++) {
            d = QuadIntersect(&s->quads[i], rayOrigin, rayDirection);
            if (d < h->t) {
                h->t = d;
                h->normal = v_normalize(s->quads[i].normal);
                h->color = s->quads[i].color; h->type = s->quads[i].type; h->objectID = (float)objectCount;
            }
            objectCount++;
        }
        return;
    }

    v3 ro = m4_mul(f->uLeftSphereInvMatrix, rayOrigin, 1.0f);
    v3 rd = m4_mul(f->uLeftSphereInvMatrix, rayDirection, 0.0f);
    d = UnitSphereIntersect(ro, rd, &n);
    if (d < h->t) {
        h->t = d;
        h->normal = v_normalize(n);
        h->normal = v_normalize(m3t_mul(f->uLeftSphereInvMatrix, h->normal));
        h->color = s->spheres[0].color; h->type = s->spheres[0].type; h->objectID = (float)objectCount;
    }
    objectCount++;
    ro = m4_mul(f->uRightSphereInvMatrix, rayOrigin, 1.0f);
    rd = m4_mul(f->uRightSphereInvMatrix, rayDirection, 0.0f);
    d = UnitSphereIntersect(ro, rd, &n);
    if (d < h->t) {
        h->t = d;
        h->normal = v_normalize(n);
        h->normal = v_normalize(m3t_mul(f->uRightSphereInvMatrix, h->normal));
        h->color = s->spheres[1].color; h->type = s->spheres[1].type; h->objectID = (float)objectCount;
    }
    objectCount++;
    for (int i = 0; i < s->nquads; i++) {
        d = QuadIntersect(&s->quads[i], rayOrigin, rayDirection);
        if (d < h->t) {
            h->t = d;
            h->normal = v_normalize(s->quads[i].normal);
            h->color = s->quads[i].color; h->type = s->quads[i].type; h->objectID = (float)objectCount;
        }
        objectCount++;
    }
    if (f->scene != PTO_SCENE_GLTF && f->scene != PTO_SCENE_HDRI && f->scene != PTO_SCENE_SKYMESH) return;

    /* ---- BVH traversal, js/GLTFModelPathTracing_FragmentShader.js:201-298 */
    float stackT[STACK_LEVELS], stackId[STACK_LEVELS];
    const float* M = f->uGLTF_Model_InvMatrix;
    rayOrigin = m4_mul(M, rayOrigin, 1.0f);
    rayDirection = m4_mul(M, rayDirection, 0.0f);
    v3 inverseDir = V3(1.0f / rayDirection.x, 1.0f / rayDirection.y, 1.0f / rayDirection.z);
    const float *c0, *c1, *a0, *a1, *b0, *b1;
    float stackptr = 0.0f;
#define NODE(i, p0, p1) do { p0 = texel32(f->aabb, f->aabbTexels, (i) * 2.0f); p1 = texel32(f->aabb, f->aabbTexels, (i) * 2.0f + 1.0f); s->c.node_fetches++; } while (0)
    NODE(stackptr, c0, c1);
    float curId = stackptr;
    float curT = BoundingBoxIntersect(V3(c0[1], c0[2], c0[3]), V3(c1[1], c1[2], c1[3]), rayOrigin, inverseDir);
    stackId[0] = curId; stackT[0] = curT;
    int skip = (curT < h->t);
    float triangleID = 0.0f, triangleU = 0.0f, triangleV = 0.0f;
    int lookup = 0;
    int dbl = (!f->uModelUsesAlbedoTexture && f->uModelMaterialType == TRANSPARENT);
    for (;;) {
        if (!skip) {
            stackptr = stackptr - 1.0f;
            if (stackptr < 0.0f) break;
            int si = (int)stackptr;
            /* pinned: stackLevels[28] out of bounds (the GLSL is undefined there): a push past
             * level 27 is dropped, a pop past it yields (0, INFINITY), which the cull below skips */
            if (si < STACK_LEVELS) { curId = stackId[si]; curT = stackT[si]; }
            else { curId = 0.0f; curT = INFINITY_G; }
            if (curT >= h->t) continue;
            NODE(curId, c0, c1);
        }
        skip = 0;
        if (c0[0] < 0.0f) {
            float idA = curId + 1.0f, idB = c1[0];
            NODE(idA, a0, a1);
            NODE(idB, b0, b1);
            float tA = BoundingBoxIntersect(V3(a0[1], a0[2], a0[3]), V3(a1[1], a1[2], a1[3]), rayOrigin, inverseDir);
            float tB = BoundingBoxIntersect(V3(b0[1], b0[2], b0[3]), V3(b1[1], b1[2], b1[3]), rayOrigin, inverseDir);
            if (tB < tA) {
                float ti = idB; idB = idA; idA = ti;
                float tt = tB; tB = tA; tA = tt;
                const float* p = b0; b0 = a0; a0 = p;
                p = b1; b1 = a1; a1 = p;
            }
            if (tB < h->t) { curId = idB; curT = tB; c0 = b0; c1 = b1; skip = 1; }
            if (tA < h->t) {
                if (skip) {
                    int si = (int)stackptr;
                    if (si < STACK_LEVELS) { stackId[si] = idB; stackT[si] = tB; }
                    else s->c.stack_overflow++;
                    stackptr = stackptr + 1.0f;
                }
                curId = idA; curT = tA; c0 = a0; c1 = a1; skip = 1;
            }
            continue;
        }
        /* leaf */
        float id = 8.0f * c0[0];
        const float* vd0 = texel32(f->tri, f->triTexels, id + 0.0f);
        const float* vd1 = texel32(f->tri, f->triTexels, id + 1.0f);
        const float* vd2 = texel32(f->tri, f->triTexels, id + 2.0f);
        s->c.leaf_tests++;
        float tu, tv;
        d = BVH_TriangleIntersect(V3(vd0[0], vd0[1], vd0[2]), V3(vd0[3], vd1[0], vd1[1]), V3(vd1[2], vd1[3], vd2[0]),
                                  rayOrigin, rayDirection, &tu, &tv, dbl);
        if (d < h->t) { h->t = d; triangleID = id; triangleU = tu; triangleV = tv; lookup = 1; }
    }
#undef NODE
    if (lookup) {
        const float* vd[8];
        for (int k = 0; k < 8; k++) vd[k] = texel32(f->tri, f->triTexels, triangleID + (float)k);
        s->c.hit_lookups++;
        float triangleW = 1.0f - triangleU - triangleV;
        v3 n0 = V3(vd[2][1], vd[2][2], vd[2][3]);
        v3 n1 = V3(vd[3][0], vd[3][1], vd[3][2]);
        v3 n2 = V3(vd[3][3], vd[4][0], vd[4][1]);
        n = v_normalize(v_add(v_add(v_muls(n0, triangleW), v_muls(n1, triangleU)), v_muls(n2, triangleV)));
        h->u = triangleW * vd[4][2] + triangleU * vd[5][0] + triangleV * vd[5][2];
        h->v = triangleW * vd[4][3] + triangleU * vd[5][1] + triangleV * vd[5][3];
        if (f->uModelUsesBumpTexture) n = perturbNormal(f, n, 1.0f, 1.0f, h->u, h->v, &s->c);
        h->normal = v_normalize(m3t_mul(M, n));
        h->type = f->uModelUsesAlbedoTexture ? PBR_MATERIAL : f->uModelMaterialType;
        h->color = V3(1.0f, 1.0f, 1.0f);
        h->objectID = (float)objectCount;
    }
}

/* ---------------------------------------------------------------- CalculateRadiance */
typedef struct { v3 objectNormal, objectColor; float objectID, pixelSharpness; } GOut;

static v3 v_pow22(v3 a) { return V3(g_pow(a.x, 2.2f), g_pow(a.y, 2.2f), g_pow(a.z, 2.2f)); }

/* Get_HDR_Color, js/HDRIEnvironmentPathTracing_FragmentShader.js:351-360 */
static v3 Get_HDR_Color(Inv* s, v3 rayDirection)
{
    const pto_frame* f = s->f;
    float u = g_atan2(rayDirection.x, rayDirection.z) * 0.15915494309f + 0.5f;
    float v = g_acos(-rayDirection.y) * 0.31830988618379067f;
    float tx[4];
    tex_bilinear_f(f->hdr, f->hdrW, f->hdrH, u, v, tx);
    s->c.hdr_taps += 4;
    return v_muls(V3(tx[0], tx[1], tx[2]), f->uHDRExposure);
}

/* CalculateRadiance of the glTF scene (js/GLTFModelPathTracing_FragmentShader.js:351-609) and of
 * the HDRI scene, which is the same program with an environment on misses, no quad light, shadow
 * rays into the sun lobe and up to three cosine bounces
 * (js/HDRIEnvironmentPathTracing_FragmentShader.js:250-520) */
static v3 CalculateRadiance(Inv* s, GOut* g)
{
    const pto_frame* f = s->f;
    const int hdri = f->scene == PTO_SCENE_HDRI;
    const int quadric = f->scene == PTO_SCENE_QUADRIC;
    const int gltf = f->scene == PTO_SCENE_GLTF || hdri;
    const v3 sun = V3(f->uSunDirection[0], f->uSunDirection[1], f->uSunDirection[2]);
    Hit h;
    memset(&h, 0, sizeof(h));
    v3 accumCol = V3(0, 0, 0), mask = V3(1, 1, 1);
    v3 x, n, nl, dirToLight, tdir;
    v3 metallicRoughness = V3(0, 0, 0), emission = V3(0, 0, 0);
    float ratioIoR, Re, Tr, P, RP, TP, weight, thickness;
    int diffuseCount = 0, previousIntersecType = -100, hitType = -100;
    int coatTypeIntersected = 0, bounceIsSpecular = 1, sampleLight = 0;
    /* pinned: `out` parameters start at 0 (see header) */
    g->objectNormal = V3(0, 0, 0); g->objectColor = V3(0, 0, 0); g->objectID = 0.0f; g->pixelSharpness = 0.0f;

    for (int bounces = 0; bounces < 6; bounces++) {
        previousIntersecType = hitType;
        SceneIntersect(s, s->rayOrigin, s->rayDirection, &h);
        hitType = h.type;
        if (h.t == INFINITY_G) {
            if (!hdri) break;
            v3 environmentColor = Get_HDR_Color(s, s->rayDirection);
            if (bounces == 0) { g->pixelSharpness = 1.01f; accumCol = environmentColor; break; }
            else if (diffuseCount == 0 && bounceIsSpecular) { g->pixelSharpness = 1.01f; accumCol = v_mul(mask, environmentColor); break; }
            else if (sampleLight) { accumCol = v_mul(mask, environmentColor); break; }
            else if (diffuseCount == 1 && previousIntersecType == TRANSPARENT && bounceIsSpecular && bounces < 3) {
                if (v_dot(s->rayDirection, sun) > 0.99f) g->pixelSharpness = 1.01f;
                accumCol = v_mul(mask, environmentColor);
                break;
            } else if (diffuseCount > 0) {
                weight = v_dot(s->rayDirection, sun) < 0.99f ? 1.0f : 0.0f;
                accumCol = v_muls(v_mul(mask, environmentColor), weight);
                break;
            }
        }
        n = v_normalize(h.normal);
        nl = v_dot(n, s->rayDirection) < 0.0f ? v_normalize(n) : v_normalize(v_neg(n));
        x = v_add(s->rayOrigin, v_muls(s->rayDirection, h.t));
        if (bounces == 0) { g->objectNormal = nl; g->objectColor = h.color; g->objectID = h.objectID; }
        if (bounces == 1 && previousIntersecType == METAL) { g->objectNormal = nl; g->objectID = h.objectID; }

        if (!hdri && hitType == LIGHT) {
            if (diffuseCount == 0) g->pixelSharpness = 1.01f;
            if (bounceIsSpecular || sampleLight) accumCol = v_mul(mask, h.color);
            break;
        }
        if (sampleLight) break;

        if (gltf && hitType == PBR_MATERIAL) {
            float tx[4];
            tex_bilinear(f->albedo, f->albedoW, f->albedoH, h.u, h.v, tx); s->c.rgba8_taps += 4;
            h.color = v_pow22(V3(tx[0], tx[1], tx[2]));
            if (f->uModelUsesEmissiveTexture) { tex_bilinear(f->emissive, f->emissiveW, f->emissiveH, h.u, h.v, tx); s->c.rgba8_taps += 4; emission = V3(tx[0], tx[1], tx[2]); }
            else emission = V3(0, 0, 0);
            emission = v_pow22(emission);
            float maxEmission = g_max(emission.x, g_max(emission.y, emission.z));
            if (bounceIsSpecular && maxEmission > 0.01f) {
                g->pixelSharpness = 1.01f;
                accumCol = v_mul(mask, emission);
                break;
            }
            hitType = DIFFUSE;
            if (f->uModelUsesMetallicTexture) { tex_bilinear(f->metallic, f->metallicW, f->metallicH, h.u, h.v, tx); s->c.rgba8_taps += 4; metallicRoughness = V3(tx[0], tx[1], tx[2]); }
            else metallicRoughness = V3(0, 0, 0);
            metallicRoughness = v_pow22(metallicRoughness);
            if (metallicRoughness.y > 0.01f) hitType = CLEARCOAT_DIFFUSE;
            if (metallicRoughness.z > 0.01f) hitType = METAL;
        }

        if (hitType == DIFFUSE) {
            diffuseCount++;
            mask = v_mul(mask, h.color);
            bounceIsSpecular = 0;
            if ((hdri ? diffuseCount <= 2 : diffuseCount == 1) && blueNoise_rand(s) < 0.5f) {
                s->rayDirection = randomCosWeightedDirectionInHemisphere(s, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            if (hdri) {
                s->rayDirection = randomDirectionInSpecularLobe(s, sun, 0.03f);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                weight = g_max(0.0f, v_dot(s->rayDirection, nl)) * (f->uSunPower * f->uSunPower * 0.0000001f);
                mask = v_muls(mask, weight);
                sampleLight = 1;
                continue;
            }
            dirToLight = sampleAxisAlignedQuadLight(s, x, nl, &s->quads[5], &weight);
            mask = v_muls(mask, weight);
            s->rayDirection = dirToLight;
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            sampleLight = 1;
            continue;
        }
        if (hitType == METAL) {
            mask = v_mul(mask, h.color);
            if (gltf) s->rayDirection = randomDirectionInSpecularLobe(s, v_reflect(s->rayDirection, nl), metallicRoughness.y);
            else s->rayDirection = v_reflect(s->rayDirection, nl);
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            continue;
        }
        if (hitType == TRANSPARENT) {
            if (diffuseCount == 0 && !coatTypeIntersected && !f->uCameraIsMoving) g->pixelSharpness = 1.01f;
            else if (diffuseCount > 0) g->pixelSharpness = 0.0f;
            else g->pixelSharpness = -1.0f;
            Re = calcFresnelReflectance(s->rayDirection, n, 1.0f, 1.5f, &ratioIoR);
            Tr = 1.0f - Re;
            P = 0.25f + (0.5f * Re);
            RP = Re / P;
            TP = Tr / (1.0f - P);
            if (blueNoise_rand(s) < P) {
                mask = v_muls(mask, RP);
                s->rayDirection = v_reflect(s->rayDirection, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            if (quadric) {   /* js/TransformedQuadricGeometry_FragmentShader.js:470-471: no absorption */
                mask = v_muls(mask, TP);
                mask = v_mul(mask, h.color);
            } else {
                if (v_distance(n, nl) > 0.1f) {
                    thickness = 0.01f;
                    v3 cc = v_clamps(h.color, 0.01f, 0.99f);
                    v3 e = V3(g_exp(g_log(cc.x) * thickness * h.t), g_exp(g_log(cc.y) * thickness * h.t), g_exp(g_log(cc.z) * thickness * h.t));
                    mask = v_mul(mask, e);
                }
                mask = v_muls(mask, TP);
            }
            tdir = v_refract(s->rayDirection, nl, ratioIoR);
            s->rayDirection = tdir;
            s->rayOrigin = v_sub(x, v_muls(nl, f->uEPS_intersect));
            if (diffuseCount == 1) bounceIsSpecular = 1;
            continue;
        }
        if (hitType == CLEARCOAT_DIFFUSE) {
            coatTypeIntersected = 1;
            g->pixelSharpness = 0.0f;
            Re = calcFresnelReflectance(s->rayDirection, nl, 1.0f, 1.4f, &ratioIoR);
            Tr = 1.0f - Re;
            P = 0.25f + (0.5f * Re);
            RP = Re / P;
            TP = Tr / (1.0f - P);
            if (blueNoise_rand(s) < P) {
                if (diffuseCount == 0) g->pixelSharpness = f->uFrameCounter > 500.0f ? 1.01f : -1.0f;
                mask = v_muls(mask, RP);
                s->rayDirection = v_reflect(s->rayDirection, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            diffuseCount++;
            mask = v_muls(mask, TP);
            mask = v_mul(mask, h.color);
            bounceIsSpecular = 0;
            if ((hdri ? diffuseCount <= 2 : diffuseCount == 1) && blueNoise_rand(s) < 0.5f) {
                s->rayDirection = randomCosWeightedDirectionInHemisphere(s, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            if (hdri) {
                s->rayDirection = randomDirectionInSpecularLobe(s, sun, 0.03f);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                weight = g_max(0.0f, v_dot(s->rayDirection, nl)) * (f->uSunPower * f->uSunPower * 0.0000001f);
                mask = v_muls(mask, weight);
                if (bounces < 3) sampleLight = 1;
                continue;
            }
            dirToLight = sampleAxisAlignedQuadLight(s, x, nl, &s->quads[5], &weight);
            mask = v_muls(mask, weight);
            s->rayDirection = dirToLight;
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            if (bounces < 3) sampleLight = 1;
            continue;
        }
    }
    return v_maxs(accumCol, 0.0f);
}

/* ---------------------------------------------------------------- physical sky */
/* pathtracing_physical_sky_defines / _functions, js/PathTracingCommon.js:373-477 (Preetham sky as
 * in three.js SkyShader). Every literal is the GLSL literal rounded to f32; ops in source order. */
#define SKY_PI 3.14159265358979323f
#define SKY_E 2.71828182845904524f
static float RayleighPhase(float cosTheta)
{
    return 0.05968310365946075f * (1.0f + (cosTheta * cosTheta));
}
static float hgPhase(float cosTheta, float g)
{
    float g2 = g * g;
    float inverse = 1.0f / g_pow(g_max(0.0f, 1.0f - 2.0f * g * cosTheta + g2), 1.5f);
    return 0.07957747154594767f * ((1.0f - g2) * inverse);
}
static v3 totalMie(void)
{
    float c = (0.2f * 0.5f) * 10E-18f;
    return v_muls(V3(1.8399918514433978E14f, 2.7798023919660528E14f, 4.0790479543861094E14f), 0.434f * c);
}
static float SunIntensity(float zenithAngleCos)
{
    zenithAngleCos = g_clamp(zenithAngleCos, -1.0f, 1.0f);
    return 200.0f * g_max(0.0f, 1.0f - g_pow(SKY_E, -((1.6110731556870734f - g_acos(zenithAngleCos)) / 1.5f)));
}
static v3 v_pows(v3 a, float e) { return V3(g_pow(a.x, e), g_pow(a.y, e), g_pow(a.z, e)); }
static v3 v_exp(v3 a) { return V3(g_exp(a.x), g_exp(a.y), g_exp(a.z)); }
static v3 v_div(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static v3 Get_Sky_Color(const pto_frame* f, v3 rayDir)
{
    const v3 sun = V3(f->uSunDirection[0], f->uSunDirection[1], f->uSunDirection[2]);
    const v3 up = V3(0.0f, 1.0f, 0.0f);
    v3 viewDirection = v_normalize(rayDir);
    float cosViewSunAngle = v_dot(viewDirection, sun);
    float cosSunUpAngle = v_dot(up, sun);
    float sunE = SunIntensity(cosSunUpAngle);
    v3 rayleighAtX = v_muls(V3(5.804542996261093E-6f, 1.3562911419845635E-5f, 3.0265902468824876E-5f), 2.0f);
    v3 mieAtX = v_muls(totalMie(), 0.03f);
    float zenithAngle = g_acos(g_max(0.0f, v_dot(up, viewDirection)));
    float inverse = 1.0f / (g_cos(zenithAngle) + 0.15f * g_pow(93.885f - ((zenithAngle * 180.0f) / SKY_PI), -1.253f));
    float rayleighOpticalLength = 8400.0f * inverse;
    float mieOpticalLength = 1250.0f * inverse;
    v3 Fex = v_exp(v_neg(v_add(v_muls(rayleighAtX, rayleighOpticalLength), v_muls(mieAtX, mieOpticalLength))));
    v3 betaRTheta = v_muls(rayleighAtX, RayleighPhase(cosViewSunAngle * 0.5f + 0.5f));
    v3 betaMTheta = v_muls(mieAtX, hgPhase(cosViewSunAngle, 0.76f));
    v3 ratio = v_div(v_add(betaRTheta, betaMTheta), v_add(rayleighAtX, mieAtX));
    v3 Lin = v_pows(v_mul(v_muls(ratio, sunE), v_sub(V3(1.0f, 1.0f, 1.0f), Fex)), 1.5f);
    v3 m = v_pows(v_mul(v_muls(ratio, sunE), Fex), 1.0f / 2.0f);
    Lin = v_mul(Lin, v_mix(V3(1.0f, 1.0f, 1.0f), m, g_clamp(g_pow(1.0f - cosSunUpAngle, 5.0f), 0.0f, 1.0f)));
    v3 L0 = v_mul(V3(0.1f, 0.1f, 0.1f), Fex);
    float sundisk = g_smoothstep(0.9998f, 0.9998f + 0.00002f, cosViewSunAngle);
    L0 = v_add(L0, v_muls(v_muls(Fex, sunE * 19000.0f), sundisk));
    v3 texColor = v_add(v_muls(v_add(Lin, L0), 0.04f), V3(0.0f, 0.0003f, 0.00075f));
    float sunfade = 1.0f - g_clamp(1.0f - g_exp((f->uSunDirection[1] / 450000.0f)), 0.0f, 1.0f);
    return v_pows(texColor, 1.0f / (1.2f + (1.2f * sunfade)));
}

/* CalculateRadiance of js/PhysicalSkyModel_FragmentShader.js:119-379: misses take the sky (five
 * cases), DIFFUSE / CLEARCOAT shadow rays go toward the sun lobe, METAL is a mirror, no quad light */
static v3 CalculateRadianceSky(Inv* s, GOut* g)
{
    const pto_frame* f = s->f;
    const v3 sun = V3(f->uSunDirection[0], f->uSunDirection[1], f->uSunDirection[2]);
    Hit h;
    memset(&h, 0, sizeof(h));
    v3 accumCol = V3(0, 0, 0), mask = V3(1, 1, 1);
    v3 x, n, nl, tdir;
    float ratioIoR, Re, Tr, P, RP, TP, weight, thickness;
    int diffuseCount = 0, previousIntersecType = -100, hitType = -100;
    int coatTypeIntersected = 0, bounceIsSpecular = 1, sampleLight = 0;
    g->objectNormal = V3(0, 0, 0); g->objectColor = V3(0, 0, 0); g->objectID = 0.0f; g->pixelSharpness = 0.0f;

    for (int bounces = 0; bounces < 6; bounces++) {
        previousIntersecType = hitType;
        SceneIntersect(s, s->rayOrigin, s->rayDirection, &h);
        hitType = h.type;
        if (h.t == INFINITY_G) {
            v3 skyColor = Get_Sky_Color(f, s->rayDirection);
            if (bounces == 0) { g->pixelSharpness = 1.01f; accumCol = skyColor; break; }
            else if (diffuseCount == 0 && bounceIsSpecular) { g->pixelSharpness = 1.01f; accumCol = v_mul(mask, skyColor); break; }
            else if (sampleLight) { accumCol = v_mul(mask, skyColor); break; }
            else if (diffuseCount == 1 && previousIntersecType == TRANSPARENT && bounceIsSpecular) { accumCol = v_mul(mask, skyColor); break; }
            else if (diffuseCount > 0) {
                weight = v_dot(s->rayDirection, sun) < 0.99f ? 1.0f : 0.0f;
                accumCol = v_muls(v_mul(mask, skyColor), weight);
                break;
            }
        }
        n = v_normalize(h.normal);
        nl = v_dot(n, s->rayDirection) < 0.0f ? v_normalize(n) : v_normalize(v_neg(n));
        x = v_add(s->rayOrigin, v_muls(s->rayDirection, h.t));
        if (bounces == 0) { g->objectNormal = nl; g->objectColor = h.color; g->objectID = h.objectID; }
        if (bounces == 1 && previousIntersecType == METAL) { g->objectNormal = nl; g->objectID = h.objectID; }
        if (sampleLight) break;

        if (hitType == DIFFUSE) {
            diffuseCount++;
            mask = v_mul(mask, h.color);
            bounceIsSpecular = 0;
            if (diffuseCount == 1 && blueNoise_rand(s) < 0.5f) {
                s->rayDirection = randomCosWeightedDirectionInHemisphere(s, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            s->rayDirection = randomDirectionInSpecularLobe(s, sun, 0.1f);
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            weight = g_max(0.0f, v_dot(s->rayDirection, nl)) * 0.05f;
            mask = v_muls(mask, weight);
            sampleLight = 1;
            continue;
        }
        if (hitType == METAL) {
            mask = v_mul(mask, h.color);
            s->rayDirection = v_reflect(s->rayDirection, nl);
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            continue;
        }
        if (hitType == TRANSPARENT) {
            if (diffuseCount == 0 && !coatTypeIntersected && !f->uCameraIsMoving) g->pixelSharpness = 1.01f;
            else if (diffuseCount > 0) g->pixelSharpness = 0.0f;
            else g->pixelSharpness = -1.0f;
            Re = calcFresnelReflectance(s->rayDirection, n, 1.0f, 1.5f, &ratioIoR);
            Tr = 1.0f - Re;
            P = 0.25f + (0.5f * Re);
            RP = Re / P;
            TP = Tr / (1.0f - P);
            if (blueNoise_rand(s) < P) {
                mask = v_muls(mask, RP);
                s->rayDirection = v_reflect(s->rayDirection, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            if (v_distance(n, nl) > 0.1f) {
                thickness = 0.01f;
                v3 cc = v_clamps(h.color, 0.01f, 0.99f);
                v3 e = V3(g_exp(g_log(cc.x) * thickness * h.t), g_exp(g_log(cc.y) * thickness * h.t), g_exp(g_log(cc.z) * thickness * h.t));
                mask = v_mul(mask, e);
            }
            mask = v_muls(mask, TP);
            tdir = v_refract(s->rayDirection, nl, ratioIoR);
            s->rayDirection = tdir;
            s->rayOrigin = v_sub(x, v_muls(nl, f->uEPS_intersect));
            if (diffuseCount == 1) bounceIsSpecular = 1;
            continue;
        }
        if (hitType == CLEARCOAT_DIFFUSE) {
            coatTypeIntersected = 1;
            g->pixelSharpness = 0.0f;
            Re = calcFresnelReflectance(s->rayDirection, nl, 1.0f, 1.4f, &ratioIoR);
            Tr = 1.0f - Re;
            P = 0.25f + (0.5f * Re);
            RP = Re / P;
            TP = Tr / (1.0f - P);
            if (blueNoise_rand(s) < P) {
                if (diffuseCount == 0) g->pixelSharpness = f->uFrameCounter > 500.0f ? 1.01f : -1.0f;
                mask = v_muls(mask, RP);
                s->rayDirection = v_reflect(s->rayDirection, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            diffuseCount++;
            mask = v_muls(mask, TP);
            mask = v_mul(mask, h.color);
            bounceIsSpecular = 0;
            if (diffuseCount == 1 && blueNoise_rand(s) < 0.5f) {
                s->rayDirection = randomCosWeightedDirectionInHemisphere(s, nl);
                s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
                continue;
            }
            s->rayDirection = randomDirectionInSpecularLobe(s, sun, 0.1f);
            s->rayOrigin = v_add(x, v_muls(nl, f->uEPS_intersect));
            weight = g_max(0.0f, v_dot(s->rayDirection, nl)) * 0.05f;
            mask = v_muls(mask, weight);
            if (bounces < 3) sampleLight = 1;
            continue;
        }
    }
    return v_maxs(accumCol, 0.0f);
}

/* ---------------------------------------------------------------- main(), part 1: per pixel */
typedef struct { float rad[3]; float nrm[3]; float col[3]; float id; float sharp; } Shade;

static void shade_pixel(const pto_frame* f, int px, int py, Shade* out, pto_counters* cnt)
{
    Inv s;
    memset(&s, 0, sizeof(s));
    s.f = f;
    const float* m = f->uCameraMatrix;
    v3 camRight = V3(m[0], m[1], m[2]);
    v3 camUp = V3(m[4], m[5], m[6]);
    v3 camForward = V3(m[8], m[9], m[10]);
    v3 cameraPosition = V3(m[12], m[13], m[14]);
    float fcx = (float)px + 0.5f, fcy = (float)py + 0.5f; /* gl_FragCoord.xy */
    uint32_t fc = (uint32_t)f->uFrameCounter, fc1 = (uint32_t)(f->uFrameCounter + 1.0f);
    s.seed[0] = fc * (uint32_t)fcx;
    s.seed[1] = fc1 * (uint32_t)fcy;
    s.counter = -1.0f;
    int tx = (int)g_mod(fcx + floorf(f->uRandomVec2[0] * 256.0f), 256.0f);
    int ty = (int)g_mod(fcy + floorf(f->uRandomVec2[1] * 256.0f), 256.0f);
    const uint8_t* bn = f->blueNoise + 4 * (ty * 256 + tx);
    for (int c = 0; c < 4; c++) s.randVec4[c] = unorm8(bn[c]);
    s.c.rgba8_taps++;
    float ox = tentFilter(rng(&s));
    float oy = tentFilter(rng(&s));
    float ppx = ((fcx + ox) / f->uResolution[0]) * 2.0f - 1.0f;
    float ppy = ((fcy + oy) / f->uResolution[1]) * 2.0f - 1.0f;
    v3 rayDir = v_normalize(v_add(v_add(v_muls(v_muls(camRight, ppx), f->uULen), v_muls(v_muls(camUp, ppy), f->uVLen)), camForward));
    v3 focalPoint = v_muls(rayDir, f->uFocusDistance);
    float randomAngle = rng(&s) * TWO_PI_G;
    float randomRadius = rng(&s) * f->uApertureSize;
    v3 randomAperturePos = v_muls(v_add(v_muls(camRight, g_cos(randomAngle)), v_muls(camUp, g_sin(randomAngle))), sqrtf(randomRadius));
    v3 finalRayDir = v_normalize(v_sub(focalPoint, randomAperturePos));
    s.rayOrigin = v_add(cameraPosition, randomAperturePos);
    s.rayDirection = finalRayDir;
    SetupScene(&s);
    GOut g;
    v3 r = (f->scene == PTO_SCENE_SKY || f->scene == PTO_SCENE_SKYMESH) ? CalculateRadianceSky(&s, &g) : CalculateRadiance(&s, &g);
    out->rad[0] = r.x; out->rad[1] = r.y; out->rad[2] = r.z;
    out->nrm[0] = g.objectNormal.x; out->nrm[1] = g.objectNormal.y; out->nrm[2] = g.objectNormal.z;
    out->col[0] = g.objectColor.x; out->col[1] = g.objectColor.y; out->col[2] = g.objectColor.z;
    out->id = g.objectID;
    out->sharp = g.pixelSharpness;
    s.c.paths = 1;
    cnt->paths += s.c.paths; cnt->segments += s.c.segments; cnt->node_fetches += s.c.node_fetches;
    cnt->leaf_tests += s.c.leaf_tests; cnt->hit_lookups += s.c.hit_lookups; cnt->rgba8_taps += s.c.rgba8_taps;
    cnt->stack_overflow += s.c.stack_overflow;
    cnt->hdr_taps += s.c.hdr_taps;
}

/* ---------------------------------------------------------------- main(), part 2: quad derivatives + accumulate */
static void finish_pixel(const pto_frame* f, const Shade* sh, int W, int qy0, int x, int y, const float* prev, float* out)
{
    /* fine derivatives inside the 2x2 quad: dFdx = p(x|1) - p(x&~1), dFdy = p(y|1) - p(y&~1) */
    const Shade* c = &sh[(y - qy0) * W + x];
    const Shade* xl = &sh[(y - qy0) * W + (x & ~1)];
    const Shade* xr = &sh[(y - qy0) * W + (x | 1)];
    const Shade* yb = &sh[((y & ~1) - qy0) * W + x];
    const Shade* yt = &sh[((y | 1) - qy0) * W + x];
    float dNx = fabsf(xr->nrm[0] - xl->nrm[0]) + fabsf(yt->nrm[0] - yb->nrm[0]);
    float dNy = fabsf(xr->nrm[1] - xl->nrm[1]) + fabsf(yt->nrm[1] - yb->nrm[1]);
    float dNz = fabsf(xr->nrm[2] - xl->nrm[2]) + fabsf(yt->nrm[2] - yb->nrm[2]);
    float normalDifference = g_smoothstep(0.2f, 0.6f, dNx) + g_smoothstep(0.2f, 0.6f, dNy) + g_smoothstep(0.2f, 0.6f, dNz);
    float difference_obj = fabsf(xr->id - xl->id) > 0.0f ? 1.0f : 0.0f;
    difference_obj += fabsf(yt->id - yb->id) > 0.0f ? 1.0f : 0.0f;
    float objectDifference = g_smoothstep(0.0f, 0.5f, difference_obj);
    v3 dcx = V3(xr->col[0] - xl->col[0], xr->col[1] - xl->col[1], xr->col[2] - xl->col[2]);
    v3 dcy = V3(yt->col[0] - yb->col[0], yt->col[1] - yb->col[1], yt->col[2] - yb->col[2]);
    float difference_col = v_length(dcx) > 0.0f ? 1.0f : 0.0f;
    difference_col += v_length(dcy) > 0.0f ? 1.0f : 0.0f;
    float colorDifference = g_smoothstep(0.0f, 0.5f, difference_col);

    size_t pi = 4 * ((size_t)y * (size_t)f->width + (size_t)x);
    float pr[4] = { prev[pi], prev[pi + 1], prev[pi + 2], prev[pi + 3] };
    float cr[4] = { c->rad[0], c->rad[1], c->rad[2], 0.0f };
    if (f->uFrameCounter == 1.0f) { pr[0] = pr[1] = pr[2] = pr[3] = 0.0f; }
    else if (f->uCameraIsMoving) {
        pr[0] *= 0.5f; pr[1] *= 0.5f; pr[2] *= 0.5f;
        cr[0] *= 0.5f; cr[1] *= 0.5f; cr[2] *= 0.5f;
        pr[3] = 0.0f;
    }
    cr[3] = 0.0f;
    float pixelSharpness = c->sharp;
    if (colorDifference >= 1.0f || normalDifference >= 1.0f || objectDifference >= 1.0f) pixelSharpness = 1.01f;
    if (pixelSharpness == 1.01f) cr[3] = 1.01f;
    if (pixelSharpness == -1.0f) cr[3] = -1.0f;
    if (pr[3] == 1.01f) cr[3] = 1.01f;
    if (pr[3] == -1.0f) cr[3] = 0.0f;
    out[pi + 0] = pr[0] + cr[0];
    out[pi + 1] = pr[1] + cr[1];
    out[pi + 2] = pr[2] + cr[2];
    out[pi + 3] = cr[3];
}

static int shade_rows(const pto_frame* f, int row0, int row1, int nthreads, Shade** shp, int* qy0p, int* qy1p, pto_counters* counters)
{
    int W = f->width;
    int qy0 = row0 & ~1, qy1 = (row1 + 1) & ~1;
    int Wq = (W + 1) & ~1; /* quad helpers beyond an odd edge are shaded, never stored */
    Shade* sh = (Shade*)calloc((size_t)(qy1 - qy0) * Wq, sizeof(Shade));
    if (!sh) return -1;
    pto_counters total;
    memset(&total, 0, sizeof(total));
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        pto_counters local;
        memset(&local, 0, sizeof(local));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int y = qy0; y < qy1; y++)
            for (int x = 0; x < Wq; x++)
                shade_pixel(f, x, y, &sh[(size_t)(y - qy0) * Wq + x], &local);
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            total.paths += local.paths; total.segments += local.segments; total.node_fetches += local.node_fetches;
            total.leaf_tests += local.leaf_tests; total.hit_lookups += local.hit_lookups; total.rgba8_taps += local.rgba8_taps;
            total.stack_overflow += local.stack_overflow;
            total.hdr_taps += local.hdr_taps;
        }
    }
    if (counters) *counters = total;
    *shp = sh; *qy0p = qy0; *qy1p = qy1;
    return Wq;
}

int pto_path_trace(const pto_frame* f, const float* prev, float* out, int row0, int row1, int nthreads, pto_counters* counters)
{
    if (!f || !prev || !out || row0 < 0 || row1 > f->height || row0 >= row1 || !f->blueNoise) return -1;
    if ((f->scene == PTO_SCENE_GLTF || f->scene == PTO_SCENE_HDRI || f->scene == PTO_SCENE_SKYMESH) && (!f->aabb || !f->tri)) return -2;
    Shade* sh; int qy0, qy1;
    int Wq = shade_rows(f, row0, row1, nthreads, &sh, &qy0, &qy1, counters);
    if (Wq < 0) return -3;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int y = row0; y < row1; y++)
        for (int x = 0; x < f->width; x++)
            finish_pixel(f, sh, Wq, qy0, x, y, prev, out);
    free(sh);
    return 0;
}

int pto_gbuffer(const pto_frame* f, float* gbuf, int row0, int row1, int nthreads)
{
    if (!f || !gbuf || row0 < 0 || row1 > f->height || row0 >= row1) return -1;
    Shade* sh; int qy0, qy1;
    int Wq = shade_rows(f, row0, row1, nthreads, &sh, &qy0, &qy1, NULL);
    if (Wq < 0) return -3;
    for (int y = row0; y < row1; y++)
        for (int x = 0; x < f->width; x++) {
            const Shade* c = &sh[(size_t)(y - qy0) * Wq + x];
            float* g = gbuf + 11 * ((size_t)(y - row0) * f->width + x);
            g[0] = c->nrm[0]; g[1] = c->nrm[1]; g[2] = c->nrm[2];
            g[3] = c->col[0]; g[4] = c->col[1]; g[5] = c->col[2];
            g[6] = c->id; g[7] = c->sharp;
            g[8] = c->rad[0]; g[9] = c->rad[1]; g[10] = c->rad[2];
        }
    free(sh);
    return 0;
}

/* ---------------------------------------------------------------- screenOutput */
/* texelFetch(accumulationBuffer, ivec2(gl_FragCoord.xy + vec2(dx, dy)), 0) for pixel (px, py)
 * (js/PathTracingCommon.js:44-72): ivec2() of a float truncates toward zero, so the tap one texel
 * left of (below) the first column (row), at -0.5, reads texel 0; the one two texels out, at -1.5,
 * is outside the texture and reads 0 (pinned). Found by the mechanical transcription of the
 * shader (oracle/xcheck); an earlier reading here dropped both. */
static void fetch_acc(const float* acc, int W, int H, int px, int py, int dx, int dy, float o[4])
{
    const int x = (int)(((float)px + 0.5f) + (float)dx), y = (int)(((float)py + 0.5f) + (float)dy);
    if (x < 0 || y < 0 || x >= W || y >= H) { o[0] = o[1] = o[2] = o[3] = 0.0f; return; }
    const float* p = acc + 4 * ((size_t)y * W + x);
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3];
}

/* out (RGBA8 canvas) or out_f (RGBA32F render target: the tone-mapped floats before unorm8) */
static int screen_output(int W, int H, const float* acc, float oneOverN, float exposure, uint8_t* out, float* out_f)
{
    if (!acc || (!out && !out_f) || W <= 0 || H <= 0) return -1;
    /* m25 index k -> offset (dx, dy): rows dy = +2 .. -2, columns dx = -2 .. +2 */
    static const int taps5[8][3] = {
        /* first-ring tap, then its two outer taps (js/PathTracingCommon.js:82-209) */
        { 11, 10, 5 }, { 13, 14, 19 }, { 7, 2, 3 }, { 17, 22, 21 },
        { 6, 0, 1 }, { 8, 4, 9 }, { 16, 15, 20 }, { 18, 23, 24 },
    };
    static const int ring3[8] = { 11, 13, 7, 17, 6, 8, 16, 18 }; /* m9 order 3,5,1,7,0,2,6,8 */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float m25[25][4];
            for (int k = 0; k < 25; k++) fetch_acc(acc, W, H, x, y, (k % 5) - 2, 2 - (k / 5), m25[k]);
            float th = 1.0f;
            float cp[4] = { m25[12][0], m25[12][1], m25[12][2], m25[12][3] };
            float fr = m25[12][0], fg = m25[12][1], fb = m25[12][2];
            int count = 1;
            for (int r = 0; r < 8; r++) {
                const int* t = taps5[r];
                if (m25[t[0]][3] < th) {
                    fr += m25[t[0]][0]; fg += m25[t[0]][1]; fb += m25[t[0]][2]; count++;
                    if (m25[t[1]][3] < th) { fr += m25[t[1]][0]; fg += m25[t[1]][1]; fb += m25[t[1]][2]; count++; }
                    if (m25[t[2]][3] < th) { fr += m25[t[2]][0]; fg += m25[t[2]][1]; fb += m25[t[2]][2]; count++; }
                }
            }
            fr /= (float)count; fg /= (float)count; fb /= (float)count;
            if (cp[3] > 0.0f || cp[3] == -1.0f) {
                cp[0] = m25[12][0]; cp[1] = m25[12][1]; cp[2] = m25[12][2]; cp[3] = m25[12][3];
                count = 1;
                fr = m25[12][0]; fg = m25[12][1]; fb = m25[12][2];
                for (int r = 0; r < 8; r++) {
                    const float* t = m25[ring3[r]];
                    if (t[3] < th) { fr += t[0]; fg += t[1]; fb += t[2]; count++; }
                }
                fr /= (float)count; fg /= (float)count; fb /= (float)count;
                fr = g_mix(fr, cp[0], 0.5f); fg = g_mix(fg, cp[1], 0.5f); fb = g_mix(fb, cp[2], 0.5f);
            }
            if ((cp[3] == 1.01f && oneOverN < 0.005f) || oneOverN < 0.0002f) { fr = cp[0]; fg = cp[1]; fb = cp[2]; }
            fr *= oneOverN; fg *= oneOverN; fb *= oneOverN;
            float c3[3] = { fr * exposure, fg * exposure, fb * exposure };
            for (int k = 0; k < 3; k++) {
                float v = g_clamp(c3[k] / (1.0f + c3[k]), 0.0f, 1.0f);
                v = g_clamp(g_pow(v, 0.4545f), 0.0f, 1.0f);
                if (out) out[4 * ((size_t)y * W + x) + k] = (uint8_t)floorf(v * 255.0f + 0.5f);
                else out_f[4 * ((size_t)y * W + x) + k] = v;
            }
            if (out) out[4 * ((size_t)y * W + x) + 3] = 255;
            else out_f[4 * ((size_t)y * W + x) + 3] = 1.0f;
        }
    return 0;
}
int pto_screen_output(int W, int H, const float* acc, float oneOverN, float exposure, uint8_t* out, int nthreads)
{
    (void)nthreads;
    return out ? screen_output(W, H, acc, oneOverN, exposure, out, NULL) : -1;
}
int pto_screen_output_f32(int W, int H, const float* acc, float oneOverN, float exposure, float* out)
{
    return out ? screen_output(W, H, acc, oneOverN, exposure, NULL, out) : -1;
}

/* ---------------------------------------------------------------- quadric probe */
int pto_quadric_probe(int shape, float k, const float* ro, const float* rd, float* t, float* nrm, int n)
{
    for (int i = 0; i < n; i++) {
        v3 o = V3(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2]), d = V3(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2]);
        v3 nn = V3(0, 1, 0);
        float r;
        switch (shape) {
        case 0: r = UnitSphereIntersect(o, d, &nn); break;
        case 1: r = UnitCylinderIntersect(o, d, &nn); break;
        case 2: r = UnitConeIntersect(o, d, k, &nn); break;
        case 3: r = UnitParaboloidIntersect(o, d, &nn); break;
        case 4: r = UnitHyperboloidIntersect(o, d, k, &nn); break;
        case 5: r = UnitCapsuleIntersect(o, d, k, &nn); break;
        case 6: r = UnitFlattenedRingIntersect(o, d, k, &nn); break;
        case 7: r = UnitBoxIntersect(o, d, &nn); break;
        case 8: r = PyramidFrustumIntersect(o, d, k, &nn); break;
        case 9: r = UnitDiskIntersect(o, d); break;
        case 10: r = UnitRectangleIntersect(o, d); break;
        case 11: r = UnitTorusIntersect(o, d, k, &nn); break;
        default: return -1;
        }
        t[i] = r;
        nrm[3 * i] = nn.x; nrm[3 * i + 1] = nn.y; nrm[3 * i + 2] = nn.z;
    }
    return 0;
}

/* ---------------------------------------------------------------- sky probe */
int pto_sky_color(const float sun[3], const float* dirs, float* out, int n)
{
    pto_frame f;
    memset(&f, 0, sizeof(f));
    f.scene = PTO_SCENE_SKY;
    f.uSunDirection[0] = sun[0]; f.uSunDirection[1] = sun[1]; f.uSunDirection[2] = sun[2];
    for (int i = 0; i < n; i++) {
        v3 c = Get_Sky_Color(&f, V3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]));
        out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
    }
    return 0;
}

/* ---------------------------------------------------------------- math probes */
int pto_math_probe(int op, const float* x, const float* y2, float* out, int n)
{
    for (int i = 0; i < n; i++) {
        float a = x[i], b = y2 ? y2[i] : 0.0f;
        switch (op) {
        case 0: out[i] = g_exp2(a); break;
        case 1: out[i] = g_log2(a); break;
        case 2: out[i] = g_sin(a); break;
        case 3: out[i] = g_cos(a); break;
        case 4: out[i] = g_atan(a); break;
        case 5: out[i] = g_atan2(a, b); break;
        case 6: out[i] = g_acos(a); break;
        case 7: out[i] = g_pow(a, b); break;
        case 8: out[i] = g_exp(a); break;
        case 9: out[i] = g_log(a); break;
        case 10: out[i] = sqrtf(a); break;
        case 12: out[i] = a / b; break;
        case 13: out[i] = 1.0f / sqrtf(a); break;   /* normalize()'s 1/length */
        case 14: out[i] = 1.0f / a; break;
        case 11: {
            Inv s; memset(&s, 0, sizeof(s));
            s.seed[0] = (uint32_t)a; s.seed[1] = (uint32_t)b;
            out[i] = rng(&s);
            break;
        }
        default: return -1;
        }
    }
    return 0;
}
