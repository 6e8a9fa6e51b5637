// pt_glsl.h — device-side GLSL ES 3.00 built-ins for gfx950 with the pinned "pt-glsl v1"
// semantics documented in DESIGN.md §Parity: one IEEE binary32 op per GLSL op, no contraction
// (the library is built with -ffp-contract=off), correctly rounded '/' and sqrt, GLSL-spec
// min/max/clamp/mix, and fixed range-reduction + polynomial sequences for exp2/log2/sin/cos/atan
// built only from IEEE ops, v_floor, v_frexp_* and v_ldexp (all exact on CDNA4).
// These are __host__ __device__: libpt's host code evaluates the uniform-only parts of the scene
// programs (SetupScene, the sky constants) with the very same sequences. Nothing is shared with
// the CPU oracle except the spec.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_D __device__ __forceinline__
#define PT_HD __host__ __device__ __forceinline__

namespace ptg {

constexpr float kInf = __builtin_inff();

// correctly rounded 1/x. On the device: v_rcp_f32 and one FMA Newton step, which equals the IEEE
// quotient for every |x| in [2^-126, 2^126) (checked exhaustively on gfx950 by
// pt_math_exhaustive, tests/test_gpu_parity.py); zero, denormals, |x| >= 2^126 (denormal
// results), inf and NaN take the IEEE division (5 VALU instead of 11 on the common path)
PT_HD float grcp(float x)
{
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t m = __builtin_bit_cast(uint32_t, x) & 0x7fffffffu;
    if (__builtin_expect(m - 0x00800000u < 0x7e000000u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
#endif
    return 1.0f / x;
}

// correctly rounded sqrt(x). On the device, for x in [2^-96, 2^126]: v_sqrt_f32 and the one-ulp
// correction by the signs of the FMA residuals x - s(s -/+ ulp) (the correction hipcc emits too,
// without its tiny-input scaling and special-value selects: 9 VALU instead of 17); every other
// input (zero, tiny, huge, negative, inf, NaN) takes sqrtf. Checked exhaustively on gfx950
// (pt_math_exhaustive op 1).
PT_HD float gsqrt(float x)
{
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t b = __builtin_bit_cast(uint32_t, x);
    if (__builtin_expect(b - 0x0f800000u <= 0x7e800000u - 0x0f800000u, 1)) {
        const float s = __builtin_amdgcn_sqrtf(x);
        const uint32_t sb = __builtin_bit_cast(uint32_t, s);
        const float dn = __builtin_bit_cast(float, sb - 1u), up = __builtin_bit_cast(float, sb + 1u);
        float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
        r = __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
        return r;
    }
#endif
    return sqrtf(x);
}

PT_HD float gmin(float x, float y) { return y < x ? y : x; }
PT_HD float gmax(float x, float y) { return x < y ? y : x; }
PT_HD float gclamp(float x, float a, float b) { return gmin(gmax(x, a), b); }
PT_HD float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
PT_HD float gfract(float x) { return x - floorf(x); }
PT_HD float gmod(float x, float y) { return x - y * floorf(x / y); }
PT_HD float gsmoothstep(float e0, float e1, float x)
{
    float t = gclamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return (t * t) * (3.0f - 2.0f * t);
}

PT_HD float gexp2(float x)
{
    if (x != x) return x;
    if (x >= 128.0f) return kInf;
    if (x < -150.0f) return 0.0f;
    float n = floorf(x + 0.5f);
    float f = x - n;
    float p = 1.5252733804059841e-05f;
    p = p * f + 1.5403530393381609e-04f;
    p = p * f + 1.3333558146428443e-03f;
    p = p * f + 9.6181291076284772e-03f;
    p = p * f + 5.5504108664821580e-02f;
    p = p * f + 2.4022650695910071e-01f;
    p = p * f + 6.9314718055994531e-01f;
    p = p * f + 1.0f;
    return ldexpf(p, (int)n);
}

PT_HD float glog2(float x)
{
    if (x != x || x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -kInf;
    if (x == kInf) return kInf;
    int e;
    float m = frexpf(x, &e);
    if (m < 0.70710678118654752f) { m = m * 2.0f; e = e - 1; }
    float t = (m - 1.0f) / (m + 1.0f);
    float t2 = t * t;
    float p = 0.11111111111111111f;
    p = p * t2 + 0.14285714285714285f;
    p = p * t2 + 0.2f;
    p = p * t2 + 0.33333333333333333f;
    p = p * t2;
    float l = (t + t * p) * 2.8853900817779268f;
    return (float)e + l;
}

PT_HD float gexp(float x) { return gexp2(x * 1.4426950408889634f); }
PT_HD float glog(float x) { return glog2(x) * 0.69314718055994531f; }
PT_HD float gpow(float x, float y) { return gexp2(y * glog2(x)); }

PT_HD void gsincos_reduce(float x, float& r, int& q)
{
    float k = floorf(x * 0.63661977236758134f + 0.5f);
    float rr = x - k * 1.5703125f;
    rr = rr - k * 4.837512969970703125e-4f;
    rr = rr - k * 7.54978995489188216e-8f;
    r = rr;
    q = (int)(k - 4.0f * floorf(k * 0.25f));
}
PT_HD float gsin_poly(float r)
{
    float r2 = r * r;
    float p = -1.9515295891e-4f;
    p = p * r2 + 8.3321608736e-3f;
    p = p * r2 - 1.6666654611e-1f;
    return r + r * (r2 * p);
}
PT_HD float gcos_poly(float r)
{
    float r2 = r * r;
    float p = 2.443315711809948e-5f;
    p = p * r2 - 1.388731625493765e-3f;
    p = p * r2 + 4.166664568298827e-2f;
    return (1.0f - 0.5f * r2) + (r2 * r2) * p;
}
// sin and cos of the same angle share one reduction (the path tracer always needs both)
PT_HD void gsincos(float x, float& s, float& c)
{
    if (!(x - x == 0.0f)) { s = c = __builtin_nanf(""); return; }
    float r; int q;
    gsincos_reduce(x, r, q);
    float sp = gsin_poly(r), cp = gcos_poly(r);
    s = q == 0 ? sp : q == 1 ? cp : q == 2 ? -sp : -cp;
    c = q == 0 ? cp : q == 1 ? -sp : q == 2 ? -cp : sp;
}
PT_HD float gsin(float x) { float s, c; gsincos(x, s, c); return s; }
PT_HD float gcos(float x) { float s, c; gsincos(x, s, c); return c; }

PT_HD float gatan(float x)
{
    if (x != x) return x;
    float sgn = x < 0.0f ? -1.0f : 1.0f;
    float a = x < 0.0f ? -x : x;
    float y = 0.0f;
    if (a > 2.414213562373095f) { y = 1.5707963267948966f; a = -grcp(a); }
    else if (a > 0.4142135623730950f) { y = 0.7853981633974483f; a = (a - 1.0f) / (a + 1.0f); }
    float z = a * a;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    y = y + (p * z * a + a);
    return sgn * y;
}
PT_HD float gatan2(float y, float x)
{
    if (x != x || y != y) return x + y;
    if (x == 0.0f) {
        if (y > 0.0f) return 1.5707963267948966f;
        if (y < 0.0f) return -1.5707963267948966f;
        return 0.0f;
    }
    float t = gatan(y / x);
    if (x > 0.0f) return t;
    return y < 0.0f ? t - 3.14159265358979323f : t + 3.14159265358979323f;
}
PT_HD float gacos(float x)
{
    if (!(x >= -1.0f && x <= 1.0f)) return __builtin_nanf("");
    if (x == -1.0f) return 3.14159265358979323f;
    return 2.0f * gatan(gsqrt((1.0f - x) / (1.0f + x)));
}

// ------------------------------------------------------------------------------------- vec3
struct f3 { float x, y, z; };
PT_HD f3 mk(float x, float y, float z) { return f3{ x, y, z }; }
PT_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PT_HD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
PT_HD f3 operator/(f3 a, f3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
PT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD f3 cross(f3 a, f3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
PT_HD float length(f3 a) { return gsqrt(dot(a, a)); }
PT_HD f3 normalize(f3 a) { float inv = grcp(gsqrt(dot(a, a))); return a * inv; }
PT_HD float distance(f3 a, f3 b) { return length(a - b); }
PT_HD f3 reflect(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }
PT_HD f3 refract(f3 I, f3 N, float eta)
{
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    return I * eta - N * (eta * d + gsqrt(k));
}
PT_HD f3 mix3(f3 a, f3 b, float t) { return mk(gmix(a.x, b.x, t), gmix(a.y, b.y, t), gmix(a.z, b.z, t)); }
PT_HD f3 clamp3(f3 a, float lo, float hi) { return mk(gclamp(a.x, lo, hi), gclamp(a.y, lo, hi), gclamp(a.z, lo, hi)); }
PT_HD f3 max3s(f3 a, float s) { return mk(gmax(a.x, s), gmax(a.y, s), gmax(a.z, s)); }

// GLSL mat4 from Babylon Matrix.m (column-major): M * vec4(v, w)
struct m4 { float m[16]; };
PT_HD f3 mul(const m4& M, f3 v, float w)
{
    const float* m = M.m;
    return mk(m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * w,
              m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * w,
              m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * w);
}
// transpose(mat3(M)) * n
PT_HD f3 mul3t(const m4& M, f3 n)
{
    const float* m = M.m;
    return mk(m[0] * n.x + m[1] * n.y + m[2] * n.z,
              m[4] * n.x + m[5] * n.y + m[6] * n.z,
              m[8] * n.x + m[9] * n.y + m[10] * n.z);
}

} // namespace ptg
