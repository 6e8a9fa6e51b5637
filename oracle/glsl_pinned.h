/* oracle/glsl_pinned.h — TEST INFRASTRUCTURE (CPU oracle only; never linked into the product).
 *
 * GLSL ES 3.00 built-ins restated with ONE pinned meaning, so that the CPU restatement and the
 * HIP kernel can be compared bit-for-bit. The reference runs these built-ins on whatever the
 * browser's GL driver provides (ANGLE/Mesa/vendor): their rounding is not specified by the
 * reference, so "parity vs the GLSL render" is unpinned for radiance.
 *
 * The pinned semantics ("pt-glsl v1"), shared with csrc/pt_glsl.h by specification, not by code:
 *   - every f32 op is one IEEE-754 binary32 operation, round-to-nearest-even, no FMA contraction,
 *     no reassociation, denormals preserved;  '/' and sqrt correctly rounded;
 *   - min(x,y) = y < x ? y : x;  max(x,y) = x < y ? y : x   (GLSL spec text, NaN-propagating as
 *     written), clamp(x,a,b) = min(max(x,a),b), mix(x,y,a) = x*(1-a) + y*a;
 *   - exp2 / log2 / sin / cos / atan are the polynomial + range-reduction sequences below, built
 *     only from IEEE +,-,*,/, floor, frexp, ldexp; exp(x)=exp2(x*LOG2E), log(x)=log2(x)*LN2,
 *     pow(x,y)=exp2(y*log2(x)) (the GLSL spec's own definition of pow).
 */
#ifndef PT_ORACLE_GLSL_PINNED_H
#define PT_ORACLE_GLSL_PINNED_H

#include <math.h>
#include <stdint.h>

#define G_INF_F (__builtin_inff())

static inline float g_min(float x, float y) { return y < x ? y : x; }
static inline float g_max(float x, float y) { return x < y ? y : x; }
static inline float g_clamp(float x, float a, float b) { return g_min(g_max(x, a), b); }
static inline float g_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline float g_fract(float x) { return x - floorf(x); }
static inline float g_mod(float x, float y) { return x - y * floorf(x / y); }
static inline float g_smoothstep(float e0, float e1, float x)
{
    float t = g_clamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return (t * t) * (3.0f - 2.0f * t);
}

#ifdef PTO_LIBM
/* TOLERANCE STUDY ONLY (oracle/Makefile: libptoracle_libm.so, libptoracle_gpu.so; tools/tolerance.py):
 * another built-in set a GL driver may legally use - the C library's correctly rounded or
 * near-correctly rounded transcendentals (glibc expf/exp2f/logf/log2f/powf/sinf/cosf/atanf/atan2f/
 * acosf) instead of the pinned sequences below - to measure how far a render moves when only the
 * built-ins' rounding changes (the tolerance table). Never used by the parity tests. */
static inline float g_exp2(float x) { return exp2f(x); }
static inline float g_log2(float x) { return log2f(x); }
static inline float g_exp(float x) { return expf(x); }
static inline float g_log(float x) { return logf(x); }
static inline float g_pow(float x, float y) { return powf(x, y); }
static inline float g_sin(float x) { return sinf(x); }
static inline float g_cos(float x) { return cosf(x); }
static inline float g_atan(float x) { return atanf(x); }
static inline float g_atan2(float y, float x) { return atan2f(y, x); }
static inline float g_acos(float x) { return acosf(x); }
#else
/* 2^x: round-to-nearest integer split, degree-7 Taylor of 2^f on |f| <= 0.5, exact ldexp. */
static inline float g_exp2(float x)
{
    if (x != x) return x;
    if (x >= 128.0f) return G_INF_F;
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

/* log2(x): frexp split into [sqrt(1/2), sqrt(2)), atanh series in t=(m-1)/(m+1). */
static inline float g_log2(float x)
{
    if (x != x || x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -G_INF_F;
    if (x == G_INF_F) return G_INF_F;
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

static inline float g_exp(float x) { return g_exp2(x * 1.4426950408889634f); }
static inline float g_log(float x) { return g_log2(x) * 0.69314718055994531f; }
static inline float g_pow(float x, float y) { return g_exp2(y * g_log2(x)); }

/* sin/cos: quadrant reduction k = floor(x*2/pi + 0.5), three-part Cody–Waite pi/2, cephes-style
 * minimax polynomials on [-pi/4, pi/4]. */
static inline void g_sincos_reduce(float x, float* r, int* q)
{
    float k = floorf(x * 0.63661977236758134f + 0.5f);
    float rr = x - k * 1.5703125f;
    rr = rr - k * 4.837512969970703125e-4f;
    rr = rr - k * 7.54978995489188216e-8f;
    *r = rr;
    *q = (int)(k - 4.0f * floorf(k * 0.25f));
}
static inline float g_sin_poly(float r)
{
    float r2 = r * r;
    float p = -1.9515295891e-4f;
    p = p * r2 + 8.3321608736e-3f;
    p = p * r2 - 1.6666654611e-1f;
    return r + r * (r2 * p);
}
static inline float g_cos_poly(float r)
{
    float r2 = r * r;
    float p = 2.443315711809948e-5f;
    p = p * r2 - 1.388731625493765e-3f;
    p = p * r2 + 4.166664568298827e-2f;
    return (1.0f - 0.5f * r2) + (r2 * r2) * p;
}
static inline float g_sin(float x)
{
    if (!(x - x == 0.0f)) return __builtin_nanf("");
    float r; int q;
    g_sincos_reduce(x, &r, &q);
    float s = g_sin_poly(r), c = g_cos_poly(r);
    return q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
}
static inline float g_cos(float x)
{
    if (!(x - x == 0.0f)) return __builtin_nanf("");
    float r; int q;
    g_sincos_reduce(x, &r, &q);
    float s = g_sin_poly(r), c = g_cos_poly(r);
    return q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
}

/* atan(x): cephes atanf reduction (tan(3pi/8), tan(pi/8) breakpoints). */
static inline float g_atan(float x)
{
    if (x != x) return x;
    float sgn = x < 0.0f ? -1.0f : 1.0f;
    float a = x < 0.0f ? -x : x;
    float y = 0.0f;
    if (a > 2.414213562373095f) { y = 1.5707963267948966f; a = -1.0f / a; }
    else if (a > 0.4142135623730950f) { y = 0.7853981633974483f; a = (a - 1.0f) / (a + 1.0f); }
    float z = a * a;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    y = y + (p * z * a + a);
    return sgn * y;
}
/* atan(y, x) (GLSL two-argument form). */
static inline float g_atan2(float y, float x)
{
    if (x != x || y != y) return x + y;
    if (x == 0.0f) {
        if (y > 0.0f) return 1.5707963267948966f;
        if (y < 0.0f) return -1.5707963267948966f;
        return 0.0f;
    }
    float t = g_atan(y / x);
    if (x > 0.0f) return t;
    return y < 0.0f ? t - 3.14159265358979323f : t + 3.14159265358979323f;
}
/* acos(x) = 2*atan(sqrt((1-x)/(1+x))), NaN outside [-1,1]. */
static inline float g_acos(float x)
{
    if (!(x >= -1.0f && x <= 1.0f)) return __builtin_nanf("");
    if (x == -1.0f) return 3.14159265358979323f;
    return 2.0f * g_atan(sqrtf((1.0f - x) / (1.0f + x)));
}

#endif /* PTO_LIBM */

/* ------------------------------------------------------------------ vec3 */
typedef struct { float x, y, z; } v3;
static inline v3 V3(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static inline v3 v_add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v_sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v_mul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 v_muls(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 v_neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float v_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 v_cross(v3 a, v3 b)
{
    return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float v_length(v3 a) { return sqrtf(v_dot(a, a)); }
#ifdef PTO_APPROX_RSQ
/* TOLERANCE STUDY ONLY (libptoracle_gpu.so): normalize as a GPU driver compiles it, v * rsq(dot(v, v)),
 * with the reciprocal square root rounded toward zero (within 1 ulp, as v_rsq_f32; GLSL ES 3.00 allows
 * 2 ulp for inversesqrt) instead of a correctly rounded 1 / sqrt */
static inline float g_rsq_approx(float x)
{
    const double r = 1.0 / sqrt((double)x);
    float f = (float)r;
    if ((double)f > r) f = nextafterf(f, 0.0f);
    return f;
}
static inline v3 v_normalize(v3 a) { return v_muls(a, g_rsq_approx(v_dot(a, a))); }
#else
static inline v3 v_normalize(v3 a) { float inv = 1.0f / sqrtf(v_dot(a, a)); return v_muls(a, inv); }
#endif
static inline float v_distance(v3 a, v3 b) { return v_length(v_sub(a, b)); }
static inline v3 v_reflect(v3 I, v3 N) { return v_sub(I, v_muls(N, 2.0f * v_dot(N, I))); }
static inline v3 v_refract(v3 I, v3 N, float eta)
{
    float d = v_dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return V3(0.0f, 0.0f, 0.0f);
    return v_sub(v_muls(I, eta), v_muls(N, eta * d + sqrtf(k)));
}
static inline v3 v_mix(v3 a, v3 b, float t) { return V3(g_mix(a.x, b.x, t), g_mix(a.y, b.y, t), g_mix(a.z, b.z, t)); }
static inline v3 v_clamps(v3 a, float lo, float hi) { return V3(g_clamp(a.x, lo, hi), g_clamp(a.y, lo, hi), g_clamp(a.z, lo, hi)); }
static inline v3 v_maxs(v3 a, float s) { return V3(g_max(a.x, s), g_max(a.y, s), g_max(a.z, s)); }

/* GLSL mat4 uploaded column-major (Babylon Matrix.m): M[c][r] = m[4c+r].  M * vec4(v, w). */
static inline v3 m4_mul(const float* m, v3 v, float w)
{
    return V3(m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * w,
              m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * w,
              m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * w);
}
/* transpose(mat3(M)) * n */
static inline v3 m3t_mul(const float* m, v3 n)
{
    return V3(m[0] * n.x + m[1] * n.y + m[2] * n.z,
              m[4] * n.x + m[5] * n.y + m[6] * n.z,
              m[8] * n.x + m[9] * n.y + m[10] * n.z);
}

#endif
