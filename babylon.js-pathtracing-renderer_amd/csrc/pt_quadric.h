// pt_quadric.h — the unit-shape intersectors of the transformed-quadric program
// (js/PathTracingCommon.js:690-1163, used by js/TransformedQuadricGeometry_FragmentShader.js:77-317),
// on gfx950 with the pinned GLSL semantics: every expression keeps the GLSL's operand order, so the
// result is bit-identical to the CPU oracle. Each takes the ray already in the shape's object space.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_device.h"
#include "pt_glsl.h"

namespace pt {

struct Roots {
    float t0, t1;
};

// solveQuadratic (js/PathTracingCommon.js:629-638): u2 < 0 -> both roots 0 (the GLSL assigns
// neg_halfB = 0 inside the conditional)
PT_D Roots solveQuadratic(float A, float B, float C)
{
    float invA = grcp(A);
    B *= invA;
    C *= invA;
    float nh = -B * 0.5f;
    float u2 = nh * nh - C;
    float u;
    if (u2 < 0.0f) { nh = 0.0f; u = 0.0f; } else u = gsqrt(u2);
    return Roots{ nh - u, nh + u };
}

PT_D f3 qhit(f3 ro, f3 rd, float t) { return mk(ro.x + rd.x * t, ro.y + rd.y * t, ro.z + rd.z * t); }
PT_D float gsign(float x) { return x > 0.0f ? 1.0f : x < 0.0f ? -1.0f : 0.0f; }
PT_D float gstep(float edge, float x) { return x < edge ? 0.0f : 1.0f; }

PT_D float unitCylinder(f3 ro, f3 rd, f3& n)
{
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    Roots r = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, r.t0);
    if (r.t0 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return r.t0; }
    hit = qhit(ro, rd, r.t1);
    if (r.t1 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return r.t1; }
    return kINF;
}

PT_D float unitCone(f3 ro, f3 rd, float k, f3& n)
{
    k = gclamp(k, 0.01f, 1.0f);
    float j = grcp(k);
    float h = j * 2.0f - 1.0f;
    float a = j * rd.x * rd.x + j * rd.z * rd.z - (k * 0.25f) * rd.y * rd.y;
    float b = 2.0f * (j * rd.x * ro.x + j * rd.z * ro.z - (k * 0.25f) * rd.y * (ro.y - h));
    float c = j * ro.x * ro.x + j * ro.z * ro.z - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    Roots r = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, r.t0);
    if (r.t0 > 0.0f && fabsf(hit.y) <= 1.0f) {
        n = mk(2.0f * hit.x * j, 2.0f * (h - hit.y) * (k * 0.25f), 2.0f * hit.z * j);
        return r.t0;
    }
    hit = qhit(ro, rd, r.t1);
    if (r.t1 > 0.0f && fabsf(hit.y) <= 1.0f) {
        n = mk(2.0f * hit.x * j, 2.0f * (h - hit.y) * (k * 0.25f), 2.0f * hit.z * j);
        return r.t1;
    }
    return kINF;
}

PT_D float unitParaboloid(f3 ro, f3 rd, f3& n)
{
    const float k = 0.5f;
    float a = rd.x * rd.x + rd.z * rd.z;
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z) + k * rd.y;
    float c = ro.x * ro.x + ro.z * ro.z + k * (ro.y - 1.0f);
    Roots r = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, r.t0);
    if (r.t0 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.5f, 2.0f * hit.z); return r.t0; }
    hit = qhit(ro, rd, r.t1);
    if (r.t1 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.5f, 2.0f * hit.z); return r.t1; }
    return kINF;
}

PT_D float unitHyperboloid(f3 ro, f3 rd, float k, f3& n)
{
    k = k * k * k * k + 0.0012f;
    k *= 1000.0f;
    float j = k - 1.0f;
    float a = k * rd.x * rd.x + k * rd.z * rd.z - j * rd.y * rd.y;
    float b = 2.0f * (k * rd.x * ro.x + k * rd.z * ro.z - j * rd.y * ro.y);
    float c = (k * ro.x * ro.x + k * ro.z * ro.z - j * ro.y * ro.y) - 1.0f;
    Roots r = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, r.t0);
    if (r.t0 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x * k, 2.0f * -hit.y * j, 2.0f * hit.z * k); return r.t0; }
    hit = qhit(ro, rd, r.t1);
    if (r.t1 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x * k, 2.0f * -hit.y * j, 2.0f * hit.z * k); return r.t1; }
    return kINF;
}

PT_D float unitCapsule(f3 ro, f3 rd, float k, f3& n)
{
    k += 0.25f;
    f3 L = ro - mk(0.0f, k, 0.0f);
    float a = dot(rd, rd);
    float b = 2.0f * dot(rd, L);
    float c = dot(L, L) - 1.0f;
    const Roots s0 = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, s0.t0);
    if (s0.t0 > 0.0f && hit.y >= k) { n = mk(2.0f * hit.x, 2.0f * (hit.y - k), 2.0f * hit.z); return s0.t0; }
    L = ro - mk(0.0f, -k, 0.0f);
    a = dot(rd, rd);
    b = 2.0f * dot(rd, L);
    c = dot(L, L) - 1.0f;
    const Roots s1 = solveQuadratic(a, b, c);
    hit = qhit(ro, rd, s1.t0);
    if (s1.t0 > 0.0f && hit.y <= -k) { n = mk(2.0f * hit.x, 2.0f * (hit.y + k), 2.0f * hit.z); return s1.t0; }
    a = (rd.x * rd.x + rd.z * rd.z);
    b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    const Roots cy = solveQuadratic(a, b, c);
    hit = qhit(ro, rd, cy.t0);
    if (cy.t0 > 0.0f && fabsf(hit.y) <= k) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return cy.t0; }
    hit = qhit(ro, rd, s0.t1);
    if (s0.t1 > 0.0f && hit.y >= k) { n = mk(2.0f * hit.x, 2.0f * (hit.y - k), 2.0f * hit.z); return s0.t1; }
    hit = qhit(ro, rd, s1.t1);
    if (s1.t1 > 0.0f && hit.y <= -k) { n = mk(2.0f * hit.x, 2.0f * (hit.y + k), 2.0f * hit.z); return s1.t1; }
    hit = qhit(ro, rd, cy.t1);
    if (cy.t1 > 0.0f && fabsf(hit.y) <= k) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return cy.t1; }
    return kINF;
}

PT_D float unitFlattenedRing(f3 ro, f3 rd, float k, f3& n)
{
    k -= 0.01f;
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    const Roots o = solveQuadratic(a, b, c);
    f3 hit = qhit(ro, rd, o.t0);
    if (o.t0 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return o.t0; }
    const float d0 = (ro.y - 1.0f) / -rd.y;
    hit = qhit(ro, rd, d0);
    float x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y < 0.0f && d0 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { n = mk(0.0f, 1.0f, 0.0f); return d0; }
    const float d1 = (ro.y + 1.0f) / -rd.y;
    hit = qhit(ro, rd, d1);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y > 0.0f && d1 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { n = mk(0.0f, -1.0f, 0.0f); return d1; }
    c = (ro.x * ro.x + ro.z * ro.z) - k;
    const Roots in = solveQuadratic(a, b, c);
    hit = qhit(ro, rd, in.t0);
    if (in.t0 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return in.t0; }
    hit = qhit(ro, rd, in.t1);
    if (in.t1 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return in.t1; }
    hit = qhit(ro, rd, o.t1);
    if (o.t1 > 0.0f && fabsf(hit.y) <= 1.0f) { n = mk(2.0f * hit.x, 0.0f, 2.0f * hit.z); return o.t1; }
    hit = qhit(ro, rd, d0);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y > 0.0f && d0 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { n = mk(0.0f, 1.0f, 0.0f); return d0; }
    hit = qhit(ro, rd, d1);
    x2z2 = hit.x * hit.x + hit.z * hit.z;
    if (rd.y < 0.0f && d1 > 0.0f && x2z2 <= 1.0f && x2z2 > k) { n = mk(0.0f, -1.0f, 0.0f); return d1; }
    return kINF;
}

PT_D float unitBox(f3 ro, f3 rd, f3& n)
{
    const f3 inv = mk(grcp(rd.x), grcp(rd.y), grcp(rd.z));
    const f3 nr = (mk(-1.0f, -1.0f, -1.0f) - ro) * inv;
    const f3 fr = (mk(1.0f, 1.0f, 1.0f) - ro) * inv;
    const f3 tmin = mk(gmin(nr.x, fr.x), gmin(nr.y, fr.y), gmin(nr.z, fr.z));
    const f3 tmax = mk(gmax(nr.x, fr.x), gmax(nr.y, fr.y), gmax(nr.z, fr.z));
    const float t0 = gmax(gmax(tmin.x, tmin.y), tmin.z);
    const float t1 = gmin(gmin(tmax.x, tmax.y), tmax.z);
    if (t0 < t1) {
        if (t0 > 0.0f) {   // -sign(rd) * step(tmin.yzx, tmin) * step(tmin.zxy, tmin)
            n = mk(-gsign(rd.x) * gstep(tmin.y, tmin.x) * gstep(tmin.z, tmin.x),
                   -gsign(rd.y) * gstep(tmin.z, tmin.y) * gstep(tmin.x, tmin.y),
                   -gsign(rd.z) * gstep(tmin.x, tmin.z) * gstep(tmin.y, tmin.z));
            return t0;
        }
        if (t1 > 0.0f) {   // -sign(rd) * step(tmax, tmax.yzx) * step(tmax, tmax.zxy)
            n = mk(-gsign(rd.x) * gstep(tmax.x, tmax.y) * gstep(tmax.x, tmax.z),
                   -gsign(rd.y) * gstep(tmax.y, tmax.z) * gstep(tmax.y, tmax.x),
                   -gsign(rd.z) * gstep(tmax.z, tmax.x) * gstep(tmax.z, tmax.y));
            return t1;
        }
    }
    return kINF;
}

PT_D bool frustumSideOk(f3 p, float q, float j, float k, float h)
{
    return fabsf(p.x) <= 1.0f && fabsf(p.z) <= 1.0f && p.y <= 1.0f &&
           (j * q * q - k * 0.25f * (p.y - h) * (p.y - h)) <= 0.0f;
}

PT_D float pyramidFrustum(f3 ro, f3 rd, float k, f3& n)
{
    float xt = kINF, zt = kINF;
    f3 xn = mk(0.0f, 0.0f, 0.0f), zn = xn;
    k = gclamp(k, 0.01f, 1.0f);
    const float j = grcp(k);
    const float h = j * 2.0f - 1.0f;
    float a = j * rd.x * rd.x - (k * 0.25f) * rd.y * rd.y;
    float b = 2.0f * (j * rd.x * ro.x - (k * 0.25f) * rd.y * (ro.y - h));
    float c = j * ro.x * ro.x - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    Roots r = solveQuadratic(a, b, c);
    f3 hit0 = qhit(ro, rd, r.t0), hit1 = qhit(ro, rd, r.t1);
    if (r.t0 > 0.0f && frustumSideOk(hit0, hit0.z, j, k, h)) {
        xt = r.t0;
        xn = mk(2.0f * hit0.x * j, 2.0f * (hit0.y - h) * -(k * 0.25f), 0.0f);
    } else if (r.t1 > 0.0f && frustumSideOk(hit1, hit1.z, j, k, h)) {
        xt = r.t1;
        xn = mk(2.0f * hit1.x * j, 2.0f * (hit1.y - h) * -(k * 0.25f), 0.0f);
    }
    a = j * rd.z * rd.z - (k * 0.25f) * rd.y * rd.y;
    b = 2.0f * (j * rd.z * ro.z - (k * 0.25f) * rd.y * (ro.y - h));
    c = j * ro.z * ro.z - (k * 0.25f) * (ro.y - h) * (ro.y - h);
    r = solveQuadratic(a, b, c);
    hit0 = qhit(ro, rd, r.t0);
    hit1 = qhit(ro, rd, r.t1);
    if (r.t0 > 0.0f && frustumSideOk(hit0, hit0.x, j, k, h)) {
        zt = r.t0;
        zn = mk(0.0f, 2.0f * (hit0.y - h) * -(k * 0.25f), 2.0f * hit0.z * j);
    } else if (r.t1 > 0.0f && frustumSideOk(hit1, hit1.x, j, k, h)) {
        zt = r.t1;
        zn = mk(0.0f, 2.0f * (hit1.y - h) * -(k * 0.25f), 2.0f * hit1.z * j);
    }
    if (xt <= zt) { n = xn; return xt; }
    n = zn;
    return zt;
}

PT_D float unitDisk(f3 ro, f3 rd)
{
    const float t0 = (ro.y + 0.0f) / -rd.y;
    const f3 hit = qhit(ro, rd, t0);
    return (t0 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? t0 : kINF;
}

PT_D float unitRectangle(f3 ro, f3 rd)
{
    const float t0 = (ro.y + 0.0f) / -rd.y;
    const f3 hit = qhit(ro, rd, t0);
    return (t0 > 0.0f && fabsf(hit.x) <= 1.0f && fabsf(hit.z) <= 1.0f) ? t0 : kINF;
}

PT_D float mapTorus(f3 p, float k)
{
    const float a = gsqrt(p.x * p.x + p.z * p.z) - (1.0f - k);
    return gsqrt(a * a + p.y * p.y) - k;
}

// ray-marched torus (<= 500 sphere-tracing steps from the bounding cylinder / caps)
PT_D float unitTorus(f3 ro, f3 rd, float k, f3& n)
{
    k = 1.0f - gclamp(k, 0.01f, 0.99f);
    float d = kINF;
    float a = (rd.x * rd.x + rd.z * rd.z);
    float b = 2.0f * (rd.x * ro.x + rd.z * ro.z);
    float c = (ro.x * ro.x + ro.z * ro.z) - 1.0f;
    const Roots r = solveQuadratic(a, b, c);
    const f3 hit0 = qhit(ro, rd, r.t0), hit1 = qhit(ro, rd, r.t1);
    const float tc = (r.t0 > 0.0f && fabsf(hit0.y) <= k) ? r.t0 : (r.t1 > 0.0f && fabsf(hit1.y) <= k) ? r.t1 : kINF;
    float d0 = (ro.y + k) / -rd.y;
    f3 hit = qhit(ro, rd, d0);
    d0 = (d0 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? d0 : kINF;
    float d1 = (ro.y - k) / -rd.y;
    hit = qhit(ro, rd, d1);
    d1 = (d1 > 0.0f && hit.x * hit.x + hit.z * hit.z <= 1.0f) ? d1 : kINF;
    if (tc == kINF && d0 == kINF && d1 == kINF) return kINF;
    f3 pos = mk(0.0f, 0.0f, 0.0f);
    float t = gmin(gmin(d0, d1), tc);
#pragma unroll 1
    for (int i = 0; i < 500; i++) {
        pos = qhit(ro, rd, t);
        d = mapTorus(pos, k);
        if (fabsf(d) < 0.01f) break;
        t += d;
    }
    if (fabsf(d) < 0.01f) {
        const float ex = (1.0f * 0.5773f) * 0.0002f, ey = (-1.0f * 0.5773f) * 0.0002f;
        f3 s = mk(ex, ey, ey) * mapTorus(pos + mk(ex, ey, ey), k);
        s = s + mk(ey, ey, ex) * mapTorus(pos + mk(ey, ey, ex), k);
        s = s + mk(ey, ex, ey) * mapTorus(pos + mk(ey, ex, ey), k);
        s = s + mk(ex, ex, ex) * mapTorus(pos + mk(ex, ex, ex), k);
        n = normalize(s);
        return t;
    }
    return kINF;
}

// shape s of js/TransformedQuadricGeometry_FragmentShader.js:93-301 (object-space ray)
PT_D float quadricShape(int s, f3 ro, f3 rd, float k, f3& n)
{
    switch (s) {
    case 0: return unitSphere(ro, rd, n);
    case 1: return unitCylinder(ro, rd, n);
    case 2: return unitCone(ro, rd, k, n);
    case 3: return unitParaboloid(ro, rd, n);
    case 4: return unitHyperboloid(ro, rd, k, n);
    case 5: return unitCapsule(ro, rd, k, n);
    case 6: return unitFlattenedRing(ro, rd, k, n);
    case 7: return unitBox(ro, rd, n);
    case 8: return pyramidFrustum(ro, rd, k, n);
    case 9: return unitDisk(ro, rd);
    case 10: return unitRectangle(ro, rd);
    default: return unitTorus(ro, rd, k, n);
    }
}

} // namespace pt
