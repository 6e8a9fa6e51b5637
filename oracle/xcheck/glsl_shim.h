// oracle/xcheck/glsl_shim.h — TEST INFRASTRUCTURE (the GLSL cross-check only; never linked into
// the product, never loaded on the GPU box).
//
// A C++20 stand-in for the GLSL ES 3.00 language the reference's fragment shaders are written in,
// so that oracle/xcheck/transcribe.py can compile the reference's own shader TEXT mechanically
// (js/PathTracingCommon.js + js/*_FragmentShader.js, read from /root/reference at build time) and
// run it on the CPU. It exists to check the C oracle's hand restatement of that text: same
// expressions, constants, control flow and rng() call order. The built-ins follow the pinned
// "pt-glsl v1" semantics: the transcendental sequences are the pinned ones
// (oracle/glsl_pinned.h); everything else below is written from the GLSL spec, independently of
// the oracle's own helpers.
//
// Types: tvec<T,N> with .x/.y/.z/.w (and rgba / stpq) members, swizzles as sw<i...>() proxies
// (the transcriber rewrites v.xzy into v.sw<0,2,1>()), component-flattening constructors; mat3 /
// mat4 as columns; sampler2D over RGBA8 or RGBA32F texels in GL row order. Every operator is a
// plain function of concrete types so that swizzle proxies convert implicitly.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <type_traits>

extern "C" {
#include "../glsl_pinned.h"
}

namespace glx {

typedef unsigned int uint;

template <class T, int N> struct tvec;

template <class T, int N> struct vstore;
template <class T> struct vstore<T, 2> {
    union { T v[2]; struct { T x, y; }; struct { T r, g; }; struct { T s, t; }; };
};
template <class T> struct vstore<T, 3> {
    union { T v[3]; struct { T x, y, z; }; struct { T r, g, b; }; struct { T s, t, p; }; };
};
template <class T> struct vstore<T, 4> {
    union { T v[4]; struct { T x, y, z, w; }; struct { T r, g, b, a; }; struct { T s, t, p, q; }; };
};

// swizzle proxy: components I... of a vector, readable as tvec<T, M> and assignable
template <class T, int... I> struct Swz {
    static constexpr int M = sizeof...(I);
    T* p;
    operator tvec<T, M>() const { tvec<T, M> r; int k = 0; ((r.v[k++] = p[I]), ...); return r; }
    Swz& operator=(const tvec<T, M>& o) { int k = 0; ((p[I] = o.v[k++]), ...); return *this; }
    Swz& operator=(const Swz& o) { return *this = (tvec<T, M>)o; }
    Swz& operator+=(const tvec<T, M>& o) { return *this = (tvec<T, M>)*this + o; }
    Swz& operator-=(const tvec<T, M>& o) { return *this = (tvec<T, M>)*this - o; }
    Swz& operator*=(const tvec<T, M>& o) { return *this = (tvec<T, M>)*this * o; }
    Swz& operator/=(const tvec<T, M>& o) { return *this = (tvec<T, M>)*this / o; }
    Swz& operator*=(T s) { return *this = (tvec<T, M>)*this * s; }
    Swz& operator/=(T s) { return *this = (tvec<T, M>)*this / s; }
    Swz& operator+=(T s) { return *this = (tvec<T, M>)*this + s; }
    Swz& operator-=(T s) { return *this = (tvec<T, M>)*this - s; }
};

// component count and element type of a constructor argument
template <class X> struct Comps { static constexpr int n = 1; typedef X elem; };
template <class T, int N> struct Comps<tvec<T, N>> { static constexpr int n = N; typedef T elem; };
template <class T, int... I> struct Comps<Swz<T, I...>> { static constexpr int n = sizeof...(I); typedef T elem; };

template <class T, int N> struct tvec : vstore<T, N> {
    using vstore<T, N>::v;
    tvec() { for (int i = 0; i < N; i++) v[i] = T(0); }
    // GLSL constructors (explicit: the transcriber writes every one as T{...}, which also fixes
    // the left-to-right evaluation order of the arguments)
    template <class A> explicit tvec(const A& a)
    {
        if constexpr (Comps<A>::n == 1) { for (int i = 0; i < N; i++) v[i] = static_cast<T>(a); }   // splat
        else { int k = 0; put(k, a); }                                                                // truncate
    }
    template <class A, class B, class... R> explicit tvec(const A& a, const B& b, const R&... rest)
    {
        int k = 0;
        put(k, a); put(k, b); (put(k, rest), ...);
    }
    T& operator[](int i) { return v[i]; }
    const T& operator[](int i) const { return v[i]; }
    template <int... J> Swz<T, J...> sw() const { return { const_cast<T*>(v) }; }

  private:
    template <class X> void put(int& k, const X& x)
    {
        if constexpr (Comps<X>::n == 1) { if (k < N) v[k] = static_cast<T>(x); k++; }
        else {
            const tvec<typename Comps<X>::elem, Comps<X>::n> c = x;
            for (int i = 0; i < Comps<X>::n; i++) { if (k < N) v[k] = static_cast<T>(c.v[i]); k++; }
        }
    }
};

typedef tvec<float, 2> vec2;
typedef tvec<float, 3> vec3;
typedef tvec<float, 4> vec4;
typedef tvec<int, 2> ivec2;
typedef tvec<int, 3> ivec3;
typedef tvec<int, 4> ivec4;
typedef tvec<uint, 2> uvec2;
typedef tvec<uint, 3> uvec3;
typedef tvec<uint, 4> uvec4;

// ---- per-component operators of the concrete vector types (non-template: proxies convert)
#define GLX_BINOP(V, S, N, OP)                                                                     \
    inline V operator OP(const V& a, const V& b) { V r; for (int i = 0; i < N; i++) r.v[i] = a.v[i] OP b.v[i]; return r; } \
    inline V operator OP(const V& a, S s) { V r; for (int i = 0; i < N; i++) r.v[i] = a.v[i] OP s; return r; }           \
    inline V operator OP(S s, const V& a) { V r; for (int i = 0; i < N; i++) r.v[i] = s OP a.v[i]; return r; }           \
    inline V& operator OP##=(V& a, const V& b) { a = a OP b; return a; }                                                  \
    inline V& operator OP##=(V& a, S s) { a = a OP s; return a; }
#define GLX_VOPS(V, S, N)                                                                          \
    GLX_BINOP(V, S, N, +) GLX_BINOP(V, S, N, -) GLX_BINOP(V, S, N, *) GLX_BINOP(V, S, N, /)        \
    inline V operator-(const V& a) { V r; for (int i = 0; i < N; i++) r.v[i] = -a.v[i]; return r; } \
    inline bool operator==(const V& a, const V& b) { for (int i = 0; i < N; i++) if (!(a.v[i] == b.v[i])) return false; return true; } \
    inline bool operator!=(const V& a, const V& b) { return !(a == b); }
GLX_VOPS(vec2, float, 2)
GLX_VOPS(vec3, float, 3)
GLX_VOPS(vec4, float, 4)
GLX_VOPS(ivec2, int, 2)
GLX_VOPS(ivec3, int, 3)
GLX_VOPS(ivec4, int, 4)
GLX_VOPS(uvec2, uint, 2)
GLX_VOPS(uvec3, uint, 3)
GLX_VOPS(uvec4, uint, 4)
#define GLX_IBIT(V, S, N, OP)                                                                      \
    inline V operator OP(const V& a, const V& b) { V r; for (int i = 0; i < N; i++) r.v[i] = a.v[i] OP b.v[i]; return r; } \
    inline V operator OP(const V& a, S s) { V r; for (int i = 0; i < N; i++) r.v[i] = a.v[i] OP s; return r; }
GLX_IBIT(uvec2, uint, 2, >>) GLX_IBIT(uvec2, uint, 2, <<) GLX_IBIT(uvec2, uint, 2, ^) GLX_IBIT(uvec2, uint, 2, &)
GLX_IBIT(uvec2, uint, 2, |)
GLX_IBIT(ivec2, int, 2, >>) GLX_IBIT(ivec2, int, 2, <<) GLX_IBIT(ivec2, int, 2, ^) GLX_IBIT(ivec2, int, 2, &)

// ---- matrices: columns
template <int N> struct tmat {
    tvec<float, N> c[N];
    tmat() {}
    explicit tmat(float d) { for (int i = 0; i < N; i++) c[i].v[i] = d; }
    tmat(const tvec<float, N>& a, const tvec<float, N>& b, const tvec<float, N>& e) requires(N == 3) { c[0] = a; c[1] = b; c[2] = e; }
    template <int M> explicit tmat(const tmat<M>& m) requires(M > N)   // mat3(mat4): upper-left block
    {
        for (int j = 0; j < N; j++) for (int i = 0; i < N; i++) c[j].v[i] = m.c[j].v[i];
    }
    tvec<float, N>& operator[](int i) { return c[i]; }
    const tvec<float, N>& operator[](int i) const { return c[i]; }
};
typedef tmat<3> mat3;
typedef tmat<4> mat4;
// M * v = sum of columns scaled by v's components, in column order
inline vec3 operator*(const mat3& m, const vec3& v) { return m.c[0] * v.x + m.c[1] * v.y + m.c[2] * v.z; }
inline vec4 operator*(const mat4& m, const vec4& v) { return m.c[0] * v.x + m.c[1] * v.y + m.c[2] * v.z + m.c[3] * v.w; }
inline mat3 transpose(const mat3& m)
{
    mat3 r;
    for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) r.c[j].v[i] = m.c[i].v[j];
    return r;
}

// ---- built-ins (GLSL ES 3.00 §8), pinned meaning
inline float radians(float d) { return d * 0.017453292519943295f; }
inline float sqrt(float x) { return ::sqrtf(x); }                  // correctly rounded
inline float inversesqrt(float x) { return 1.0f / ::sqrtf(x); }
inline float abs(float x) { return ::fabsf(x); }
inline int abs(int x) { return x < 0 ? -x : x; }
inline float sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
inline float floor(float x) { return ::floorf(x); }
inline float ceil(float x) { return ::ceilf(x); }
inline float fract(float x) { return x - ::floorf(x); }                       // x - floor(x)
inline float mod(float x, float y) { return x - y * ::floorf(x / y); }         // x - y * floor(x/y)
inline float min(float x, float y) { return y < x ? y : x; }
inline float max(float x, float y) { return x < y ? y : x; }
inline int min(int x, int y) { return y < x ? y : x; }
inline int max(int x, int y) { return x < y ? y : x; }
inline float clamp(float x, float a, float b) { return min(max(x, a), b); }
inline float mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
inline float step(float e, float x) { return x < e ? 0.0f : 1.0f; }
inline float smoothstep(float e0, float e1, float x)
{
    float t = clamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}
inline float exp2(float x) { return g_exp2(x); }
inline float log2(float x) { return g_log2(x); }
inline float exp(float x) { return g_exp(x); }
inline float log(float x) { return g_log(x); }
inline float pow(float x, float y) { return g_pow(x, y); }
inline float sin(float x) { return g_sin(x); }
inline float cos(float x) { return g_cos(x); }
inline float tan(float x) { return g_sin(x) / g_cos(x); }
inline float atan(float x) { return g_atan(x); }
inline float atan(float y, float x) { return g_atan2(y, x); }
inline float acos(float x) { return g_acos(x); }

#define GLX_UN(V, N, F)  inline V F(const V& a) { V r; for (int i = 0; i < N; i++) r.v[i] = F(a.v[i]); return r; }
#define GLX_BIN(V, N, F) inline V F(const V& a, const V& b) { V r; for (int i = 0; i < N; i++) r.v[i] = F(a.v[i], b.v[i]); return r; } \
                         inline V F(const V& a, float b) { V r; for (int i = 0; i < N; i++) r.v[i] = F(a.v[i], b); return r; }
#define GLX_FV(V, N)                                                                                          \
    GLX_UN(V, N, sqrt) GLX_UN(V, N, inversesqrt) GLX_UN(V, N, abs) GLX_UN(V, N, sign) GLX_UN(V, N, floor)      \
    GLX_UN(V, N, ceil) GLX_UN(V, N, fract) GLX_UN(V, N, exp2) GLX_UN(V, N, log2) GLX_UN(V, N, exp)             \
    GLX_UN(V, N, log) GLX_UN(V, N, sin) GLX_UN(V, N, cos) GLX_UN(V, N, acos) GLX_UN(V, N, atan)                \
    GLX_BIN(V, N, mod) GLX_BIN(V, N, min) GLX_BIN(V, N, max) GLX_BIN(V, N, step) GLX_BIN(V, N, atan)         \
    inline V pow(const V& a, const V& b) { V r; for (int i = 0; i < N; i++) r.v[i] = pow(a.v[i], b.v[i]); return r; } \
    inline V clamp(const V& x, float a, float b) { V r; for (int i = 0; i < N; i++) r.v[i] = clamp(x.v[i], a, b); return r; } \
    inline V clamp(const V& x, const V& a, const V& b) { V r; for (int i = 0; i < N; i++) r.v[i] = clamp(x.v[i], a.v[i], b.v[i]); return r; } \
    inline V mix(const V& x, const V& y, float a) { V r; for (int i = 0; i < N; i++) r.v[i] = mix(x.v[i], y.v[i], a); return r; } \
    inline V mix(const V& x, const V& y, const V& a) { V r; for (int i = 0; i < N; i++) r.v[i] = mix(x.v[i], y.v[i], a.v[i]); return r; } \
    inline V smoothstep(float e0, float e1, const V& x) { V r; for (int i = 0; i < N; i++) r.v[i] = smoothstep(e0, e1, x.v[i]); return r; } \
    inline float dot(const V& a, const V& b) { float s = a.v[0] * b.v[0]; for (int i = 1; i < N; i++) s = s + a.v[i] * b.v[i]; return s; } \
    inline float length(const V& a) { return sqrt(dot(a, a)); }                                             \
    inline float distance(const V& a, const V& b) { return length(a - b); }                                 \
    inline V normalize(const V& a) { return a * (1.0f / sqrt(dot(a, a))); }                                 \
    inline V reflect(const V& I, const V& n) { return I - n * (2.0f * dot(n, I)); }                          \
    inline V refract(const V& I, const V& n, float eta)                                                      \
    {                                                                                                        \
        float d = dot(n, I);                                                                                 \
        float k = 1.0f - eta * eta * (1.0f - d * d);                                                         \
        if (k < 0.0f) return V();                                                                            \
        return I * eta - n * (eta * d + sqrt(k));                                                            \
    }
GLX_FV(vec2, 2)
GLX_FV(vec3, 3)
GLX_FV(vec4, 4)
inline vec3 cross(const vec3& a, const vec3& b)
{
    return vec3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}

// ---- samplers: texels in GL row order (row 0 = t 0), as the oracle's textures are given
struct sampler2D {
    const void* data = nullptr;
    int w = 0, h = 0;
    int f32 = 0;   // 1: RGBA32F texels, 0: RGBA8 (unorm8 = b / 255)
    vec4 texel(int x, int y) const
    {
        if (!data || x < 0 || y < 0 || x >= w || y >= h) return vec4();   // outside the texture: 0
        const size_t i = 4 * ((size_t)y * w + x);
        if (f32) { const float* p = (const float*)data + i; return vec4(p[0], p[1], p[2], p[3]); }
        const uint8_t* p = (const uint8_t*)data + i;
        return vec4((float)p[0] / 255.0f, (float)p[1] / 255.0f, (float)p[2] / 255.0f, (float)p[3] / 255.0f);
    }
};
inline vec4 texelFetch(const sampler2D& s, const ivec2& c, int) { return s.texel(c.x, c.y); }
// implicit LOD of a non-mipmapped texture: level 0, bilinear, REPEAT
inline int glx_wrap(float f, int n)
{
    float r = ::fmodf(f, (float)n);
    if (!(r == r)) r = 0.0f;
    int i = (int)r;
    return i < 0 ? i + n : i;
}
inline vec4 texture(const sampler2D& s, const vec2& uv)
{
    if (!s.data || s.w <= 0 || s.h <= 0) return vec4();
    const float x = uv.x * (float)s.w - 0.5f, y = uv.y * (float)s.h - 0.5f;
    const float fx = ::floorf(x), fy = ::floorf(y);
    const float ax = x - fx, by = y - fy;
    const int x0 = glx_wrap(fx, s.w), y0 = glx_wrap(fy, s.h);
    const int x1 = x0 + 1 == s.w ? 0 : x0 + 1, y1 = y0 + 1 == s.h ? 0 : y0 + 1;
    return mix(mix(s.texel(x0, y0), s.texel(x1, y0), ax), mix(s.texel(x0, y1), s.texel(x1, y1), ax), by);
}

// ---- GLSL arrays: an index outside the array reads a sentinel and drops the write (pinned; for
// the BVH stack `stackLevels[28]` of (node, tNear) entries the sentinel's tNear = INFINITY, so a
// pop past the bottom is culled, as the oracle and the kernels pin it)
template <class T> inline T garr_sentinel() { return T(); }
template <> inline vec2 garr_sentinel<vec2>() { return vec2(0.0f, 1000000.0f); }
template <class T, int N> struct garr {
    T a[N];
    T dummy;
    T& operator[](int i)
    {
        if (i < 0 || i >= N) { dummy = garr_sentinel<T>(); return dummy; }
        return a[i];
    }
};

// ---- GLSL `out` / `inout` parameters: the callee works on a local copy (out: zero-initialised,
// the pinned meaning of an unwritten out) that is copied back when the function returns
template <class T> struct OutCopy {
    T& dst;
    const T& src;
    ~OutCopy() { dst = src; }
};

// ---- fragment-quad derivatives (the harness runs the four invocations of a 2x2 quad together)
float quad_dfdx(float v);
float quad_dfdy(float v);
inline float dFdx(float v) { return quad_dfdx(v); }
inline float dFdy(float v) { return quad_dfdy(v); }
inline float fwidth(float v) { return abs(dFdx(v)) + abs(dFdy(v)); }
inline vec3 dFdx(const vec3& v) { return vec3(dFdx(v.x), dFdx(v.y), dFdx(v.z)); }
inline vec3 dFdy(const vec3& v) { return vec3(dFdy(v.x), dFdy(v.y), dFdy(v.z)); }
inline vec3 fwidth(const vec3& v) { return vec3(fwidth(v.x), fwidth(v.y), fwidth(v.z)); }

}  // namespace glx
