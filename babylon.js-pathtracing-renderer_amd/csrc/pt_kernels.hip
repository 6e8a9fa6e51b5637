// pt_kernels.hip — gfx950 kernels behind libpt.so.
//
//   pt_trace<PROG,COUNT,CONT> the per-pixel path-tracing program (js/PathTracingCommon.js:1251-1358
//                         with the Cornell / glTF scene shaders' SetupScene, SceneIntersect and
//                         CalculateRadiance). One lane = one pixel = one path of <= 6 segments.
//   pt_copy               screenCopy (js/PathTracingCommon.js:1-16), band-aware.
//   pt_output             screenOutput (js/PathTracingCommon.js:19-309): 5x5 / 3x3 edge-aware
//                         filter, 1/N, Reinhard, gamma 0.4545, unorm8.
//   pt_math_probe_kernel  device self-test of the pinned built-ins.
//
// Mapping onto CDNA4:
//  * a 256-lane block shades a 16x16 tile as four 8x8 wave tiles; lane bits (x0,y0,x1,x2,y1,y2)
//    put every GL 2x2 fragment quad inside 4 consecutive lanes, so dFdx/dFdy/fwidth are two
//    DPP/ds_swizzle exchanges (__shfl_xor 1 and 2) instead of a G-buffer round trip through HBM;
//  * the scene constants (SetupScene) live in the kernarg segment -> SGPRs;
//  * the BVH short stack (stackLevels[28] of (node, tNear)) keeps its first kStackLds levels per
//    lane in LDS at [level][lane] (conflict-free); deeper levels (rare for the reference meshes'
//    rays, but legal for depth <= 28 trees) go to a global slab [level][grid lane], not to a
//    private array: scratch would be reserved for every resident wave;
//  * BVH nodes are read as the reference's 32-byte texel pairs (two dwordx4 loads per node) and
//    leaf triangles as three dwordx4 loads: the AoS texture layout is already the right one for
//    incoherent per-lane gathers (one 32/48-B segment per lane, vs 8-9 lines for SoA).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_device.h"
#include "pt_glsl.h"
#include "pt_program.h"
#include "pt_trace.h"
#ifdef PT_SECPROF
#define PT_SECPROF_ON 1
#else
#define PT_SECPROF_ON 0
#endif

using namespace ptg;

namespace pt {
// longest-first dispatch: wave durations (shader clock) in 8 log-scale buckets per octave
PT_D int costBucket(unsigned dur)
{
    const float l = __log2f((float)dur + 1.0f);   // scheduling only, never in the image
    return min(kCostBuckets - 1, max(0, (int)((l - 8.0f) * 8.0f)));
}

// Builds order[] (a permutation of the ntiles 16x16 tiles) for the next frame from the running
// cost[tile*4 + quadrant] (each wave halves the old value and adds half its duration: smooths the
// frame-to-frame noise of 64 random paths; measured 1-2 % better than the last frame alone) (one block): a tile weighs as its slowest quadrant wave; tiles are dealt
// bucket by bucket, slowest bucket first; within a bucket the order is whatever the LDS atomics
// give - any permutation renders the same bits, only the schedule changes.
// (one block of 1024 threads as its own kernel, or of 256 as the extra block of pt_output)
// near_arg: near_buckets (bits 0-7) | (flat + 1) << 8 (bits 8-15, 0 = no flattening) | the least tiles / 64 of a
// flattened frame << 16: with flat >= 0, every
// bucket more than `flat` below the slowest tile's is dealt as one bucket, in (about) row-major order - the
// slowest tiles still start first, the bulk of the frame sweeps down the screen, so the tiles in flight at
// once lie in one band (their BVH working set shared in each XCD's L2)
PT_D void orderBuild(unsigned ntiles, const unsigned* cost, unsigned* order, unsigned* split, unsigned split_cap,
                     unsigned dominance, int near_arg)
{
    __shared__ unsigned cnt[kCostBuckets];
    __shared__ unsigned long long total;
    __shared__ unsigned slowest;
    __shared__ unsigned floorB;
    const int near_buckets = near_arg & 255, flat = ((near_arg >> 8) & 255) - 1;
    const unsigned flat_min = (unsigned)(near_arg >> 16) * 64u;   // flattening from this many tiles up
    for (int b = threadIdx.x; b < kCostBuckets; b += blockDim.x) cnt[b] = 0;
    if (threadIdx.x == 0) { total = 0; slowest = 0; }
    __syncthreads();
    auto tileCost = [&](unsigned t) {
        const unsigned* c = cost + 4u * t;
        return max(max(c[0], c[1]), max(c[2], c[3]));
    };
    auto tileBucket = [&](unsigned t) { return costBucket(tileCost(t)); };
    unsigned long long part = 0;
    unsigned mx = 0;
    // up to kOrderHeld tiles per thread (128: a 4K frame with 256 threads) go through registers,
    // their buckets four to a register: all the cost loads of a chunk are issued before its LDS
    // atomics (a loop with the atomic inside waits one HBM round trip per iteration), and the
    // scatter reuses the buckets instead of reloading
    constexpr int kOrderChunk = 8;
    const bool held = ntiles <= kOrderHeld * blockDim.x;
    unsigned bk[(int)kOrderHeld / 4];
    if (held) {
#pragma unroll
        for (int c0 = 0; c0 < (int)kOrderHeld; c0 += kOrderChunk) {
            if (c0 * blockDim.x >= ntiles) continue;   // (no break: the loop must unroll, bk[] stays in registers)
            uint4 v[kOrderChunk];
#pragma unroll
            for (int j = 0; j < kOrderChunk; j++) {
                const unsigned t = threadIdx.x + (c0 + j) * blockDim.x;
                v[j] = t < ntiles ? *(const uint4*)(cost + 4u * t) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int j = 0; j < kOrderChunk; j++) {
                const unsigned t = threadIdx.x + (c0 + j) * blockDim.x;
                const unsigned m = max(max(v[j].x, v[j].y), max(v[j].z, v[j].w));
                const unsigned b = (unsigned)costBucket(m);
                const int k = c0 + j;
                bk[k >> 2] = (k & 3) ? (bk[k >> 2] | (b << (8 * (k & 3)))) : b;
                part += (unsigned long long)v[j].x + v[j].y + v[j].z + v[j].w;
                mx = max(mx, m);
                if (t < ntiles) atomicAdd(&cnt[b], 1u);
            }
        }
    } else {
        for (unsigned t = threadIdx.x; t < ntiles; t += blockDim.x) {
            atomicAdd(&cnt[tileBucket(t)], 1u);
            const unsigned* c = cost + 4u * t;
            part += (unsigned long long)c[0] + c[1] + c[2] + c[3];
            mx = max(mx, tileCost(t));
        }
    }
    for (int o = 32; o > 0; o >>= 1) {   // one LDS atomic per wave, not per thread
        part += __shfl_xor(part, o, 64);
        mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if ((threadIdx.x & 63u) == 0) { atomicAdd(&total, part); atomicMax(&slowest, mx); }
    __syncthreads();
    if (threadIdx.x < 64) {
        // tiles to split (pt_trace): when the slowest wave costs at least `dominance` (8) x the mean (a few tiles
        // bound the launch, as the helmet's do: ~10x; the dragon stand-in and the bunny, bound by
        // throughput, stay near 4x), those within near_buckets (3: ~0.77x) of the slowest, at most split_cap of them. Wave 0 does it, two buckets a lane (a serial loop over LDS is ~6 us).
        static_assert(kCostBuckets == 128, "two buckets per lane of one wave");
        const int l = threadIdx.x;
        const unsigned c0 = cnt[2 * l], c1 = cnt[2 * l + 1];
        const unsigned long long nz = __ballot((c0 | c1) != 0u);
        int top = 0;
        if (nz) {
            const int tl = 63 - __builtin_clzll(nz);
            top = 2 * tl + ((unsigned)__shfl((int)c1, tl, 64) != 0u ? 1 : 0);
        }
        unsigned near = (2 * l <= top && 2 * l > top - near_buckets ? c0 : 0u) +
                        (2 * l + 1 <= top && 2 * l + 1 > top - near_buckets ? c1 : 0u);
        for (int o = 1; o < 64; o <<= 1) near += (unsigned)__shfl_xor((int)near, o, 64);
        const bool dominated = (unsigned long long)slowest * 4ull * ntiles >= dominance * total && total > 0;
        if (l == 0) {
            const unsigned k = (near + 7u) & ~7u;   // split_cap: a multiple of 8, <= ntiles
            *split = dominated ? min(k, split_cap) : 0u;
        }
        // flattening: the buckets below fl dealt as bucket fl (their counts folded into it) - for frames of more
        // than 8192 tiles (4K); at 1080p it lost on the helmet and StanfordBunny (-1.4 %, -2.5 %)
        const int fl = flat >= 0 && ntiles > flat_min ? max(0, top - flat) : 0;
        unsigned below = (2 * l < fl ? c0 : 0u) + (2 * l + 1 < fl ? c1 : 0u);
        for (int o = 32; o > 0; o >>= 1) below += (unsigned)__shfl_xor((int)below, o, 64);
        unsigned f0 = 2 * l < fl ? 0u : c0, f1 = 2 * l + 1 < fl ? 0u : c1;
        if (2 * l == fl) f0 += below;
        if (2 * l + 1 == fl) f1 += below;
        unsigned suf = f0 + f1;   // inclusive suffix sum over lanes l..63 (descending bucket order)
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned t = (unsigned)__shfl_down((int)suf, o, 64);
            if (l + o < 64) suf += t;
        }
        const unsigned excl = suf - f0 - f1;   // tiles in buckets above 2l + 1
        cnt[2 * l + 1] = excl;
        cnt[2 * l] = excl + f1;
        if (l == 0) floorB = (unsigned)fl;
    }
    __syncthreads();
    const unsigned fb = floorB;
    if (held) {
#pragma unroll
        for (int j = 0; j < (int)kOrderHeld; j++) {
            const unsigned t = threadIdx.x + j * blockDim.x;
            if (t < ntiles) {
                const unsigned pos = atomicAdd(&cnt[max((bk[j >> 2] >> (8 * (j & 3))) & 255u, fb)], 1u);
                if (pos < ntiles) order[pos] = t;
            }
        }
        return;
    }
    for (unsigned t = threadIdx.x; t < ntiles; t += blockDim.x) {
        const unsigned pos = atomicAdd(&cnt[max((unsigned)tileBucket(t), fb)], 1u);
        if (pos < ntiles) order[pos] = t;
    }
}

__global__ __launch_bounds__(1024) void pt_order_build(unsigned ntiles, const unsigned* cost, unsigned* order,
                                                        unsigned* split, unsigned split_cap, unsigned dominance,
                                                        int near_buckets)
{
    orderBuild(ntiles, cost, order, split, split_cap, dominance, near_buckets);
}
// ------------------------------------------------------------------------------ screenCopy
__global__ __launch_bounds__(256) void pt_copy(CopyArgs a)
{
    // one block per (16-row band, 256-texel column chunk); shards copy only their own bands
    const int band = blockIdx.y * a.num_parts + a.part;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= a.width) return;
    for (int r = 0; r < kTile; r++) {
        int y = band * kTile + r;
        if (y >= a.height) return;
        long long i = (long long)y * a.width + x;
        a.dst[i] = a.src[i];
    }
}

// ------------------------------------------------------------------------------ accumulation
// The history half of main() (js/PathTracingCommon.js:1326-1357) for a megakernel draw: the pixel's
// history texel (previousBuffer = the screenCopy target), cleared at frame 1 and halved while the camera
// moves, plus the radiance pt_trace left in `rad`; alpha = the radiance's pre-history flag unless the
// history's says 1.01 (stays sharp) or -1 (0). Each pixel reads only its own texels, so `prev` may be
// `out` (in-place history). A block covers 64 columns x one 16-row band, each thread 4 rows, loads first.
PT_D void blendRows(const BlendArgs& a, int x, int r0)
{
    typedef float nt4 __attribute__((ext_vector_type(4)));
    nt4 rv[4], pv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int y = r0 + 4 * k;
        if (y < a.height) {
            const long long i = (long long)y * a.width + x;
            rv[k] = __builtin_nontemporal_load((const nt4*)&a.rad[i]);
            pv[k] = __builtin_nontemporal_load((const nt4*)&a.prev[i]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int y = r0 + 4 * k;
        if (y >= a.height) break;
        float4 prev = make_float4(pv[k].x, pv[k].y, pv[k].z, pv[k].w);
        float cr = rv[k].x, cg = rv[k].y, cb = rv[k].z, ca = rv[k].w;
        if (a.frame == 1.0f) prev = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        else if (a.moving) {
            prev.x *= 0.5f; prev.y *= 0.5f; prev.z *= 0.5f;
            cr *= 0.5f; cg *= 0.5f; cb *= 0.5f;
            prev.w = 0.0f;
        }
        if (prev.w == 1.01f) ca = 1.01f;
        if (prev.w == -1.0f) ca = 0.0f;
        a.out[(long long)y * a.width + x] = make_float4(prev.x + cr, prev.y + cg, prev.z + cb, ca);
    }
}
__global__ __launch_bounds__(256) void pt_blend(BlendArgs a)
{
    const int band = blockIdx.y * a.num_parts + a.part;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int r0 = band * kTile + (threadIdx.x >> 6);
    if (a.cont_count && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2) a.cont_count[threadIdx.x] = 0u;   // counter, queue head (pt_cont is done)
    if (a.cont_bins && blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < kSortBins; i += 256) a.cont_bins[i] = 0u;
    if (x >= a.width) return;
    blendRows(a, x, r0);
}
// The same as one-wave workgroups that stride over (64 columns x 4 rows of a band) units: beside the
// overlapped frames' path tracing a free wave slot comes one at a time, and a 4-wave workgroup waits
// for four on one CU (the main stream's small kernels then took 100-600 us)
__global__ __launch_bounds__(64) void pt_blend_w(BlendArgs a, int units_x, int units)
{
    if (a.cont_count && blockIdx.x == 0 && threadIdx.x < 2) a.cont_count[threadIdx.x] = 0u;
    if (a.cont_bins && blockIdx.x == 0)
        for (int i = threadIdx.x; i < kSortBins; i += 64) a.cont_bins[i] = 0u;
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        const int cx = u % units_x, rest = u / units_x;
        const int band = (rest >> 2) * a.num_parts + a.part;
        const int x = cx * 64 + threadIdx.x;
        if (x < a.width) blendRows(a, x, band * kTile + (rest & 3));
    }
}

// ------------------------------------------------------------------------------ screenOutput
// the texel texelFetch(accumulationBuffer, ivec2(gl_FragCoord.xy + vec2(dx, dy)), 0) reads for the
// tap at integer position (x, y) = pixel + (dx, dy) (js/PathTracingCommon.js:44-72): ivec2() of a
// float truncates toward zero, so position -1 (fragment coordinate -0.5) reads texel 0 and -2
// (-1.5) is outside the texture: 0 (pinned)
PT_D float4 accAt(const OutputArgs& a, int x, int y)
{
    x = (int)((float)x + 0.5f);
    y = (int)((float)y + 0.5f);
    if (x < 0 || y < 0 || x >= a.acc_w || y >= a.acc_h) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return a.acc[(long long)y * a.acc_w + x];
}

// screenOutput of pixel (x, y) from its tile's 20x20 neighbourhood staged in LDS (lx, ly: the
// pixel's place in the 16x16 tile)
PT_D void outputPixel(const OutputArgs& a, const float4* tile, int lx, int ly, int x, int y)
{
    float4 m25[25];
#pragma unroll
    for (int k = 0; k < 25; k++) m25[k] = tile[(ly + 2 + 2 - (k / 5)) * 20 + (lx + 2 + (k % 5) - 2)];
    // the frame's screenCopy (js/PathTracingCommon.js:1-16), deferred by the host to ride along:
    // the same texel of the same source, written to the copy target
    if (a.copy_dst) a.copy_dst[(long long)y * a.acc_w + x] = m25[12];
    const float th = 1.0f;
    float4 cp = m25[12];
    float fr = cp.x, fg = cp.y, fb = cp.z;
    int count = 1;
    // first-ring tap, then its two outer taps, in the reference's order (js/PathTracingCommon.js:82-209)
    constexpr int T5[8][3] = { { 11, 10, 5 }, { 13, 14, 19 }, { 7, 2, 3 }, { 17, 22, 21 },
                               { 6, 0, 1 }, { 8, 4, 9 }, { 16, 15, 20 }, { 18, 23, 24 } };
#pragma unroll
    for (int r = 0; r < 8; r++) {
        if (m25[T5[r][0]].w < th) {
            fr += m25[T5[r][0]].x; fg += m25[T5[r][0]].y; fb += m25[T5[r][0]].z; count++;
            if (m25[T5[r][1]].w < th) { fr += m25[T5[r][1]].x; fg += m25[T5[r][1]].y; fb += m25[T5[r][1]].z; count++; }
            if (m25[T5[r][2]].w < th) { fr += m25[T5[r][2]].x; fg += m25[T5[r][2]].y; fb += m25[T5[r][2]].z; count++; }
        }
    }
    fr /= (float)count; fg /= (float)count; fb /= (float)count;
    if (cp.w > 0.0f || cp.w == -1.0f) {
        constexpr int R3[8] = { 11, 13, 7, 17, 6, 8, 16, 18 };
        count = 1;
        fr = cp.x; fg = cp.y; fb = cp.z;
#pragma unroll
        for (int r = 0; r < 8; r++)
            if (m25[R3[r]].w < th) { fr += m25[R3[r]].x; fg += m25[R3[r]].y; fb += m25[R3[r]].z; count++; }
        fr /= (float)count; fg /= (float)count; fb /= (float)count;
        fr = gmix(fr, cp.x, 0.5f); fg = gmix(fg, cp.y, 0.5f); fb = gmix(fb, cp.z, 0.5f);
    }
    if ((cp.w == 1.01f && a.one_over_n < 0.005f) || a.one_over_n < 0.0002f) { fr = cp.x; fg = cp.y; fb = cp.z; }
    fr *= a.one_over_n; fg *= a.one_over_n; fb *= a.one_over_n;
    float c[3] = { fr * a.exposure, fg * a.exposure, fb * a.exposure };
    float o[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float v = gclamp(c[k] / (1.0f + c[k]), 0.0f, 1.0f);
        o[k] = gclamp(gpow(v, 0.4545f), 0.0f, 1.0f);
    }
    const long long i = (long long)y * a.width + x;
    if (a.canvas)
        a.canvas[i] = make_uchar4((unsigned char)floorf(o[0] * 255.0f + 0.5f), (unsigned char)floorf(o[1] * 255.0f + 0.5f),
                                  (unsigned char)floorf(o[2] * 255.0f + 0.5f), 255);
    else
        a.out_f[i] = make_float4(o[0], o[1], o[2], 1.0f);
}

// One 16x16 tile of an owned band at a time per 256-thread block; the tile's 20x20 neighbourhood
// (+-2 texels, texelFetch semantics: 0 outside the accumulation texture) is staged in LDS, so each
// texel is read from L2 once instead of by 25 taps. A fixed grid of blocks walks the tiles
// gridDim.x apart: the next tile's neighbourhood is loaded into registers while this tile is shaded
// from LDS, then stored into the other LDS buffer (one barrier per tile), so the loads' latency
// hides behind the shading (42.5 -> 38.8 us per 1080p frame against one block per tile).
__global__ __launch_bounds__(256) void pt_output(OutputArgs a, int tiles_x, int ntiles)
{
    __shared__ float4 tile[2][20 * 20];
    const int tid = threadIdx.x;
    const int lx = tid & 15, ly = tid >> 4;
    auto origin = [&](int t, int& x0, int& y0) {
        x0 = (t % tiles_x) * 16;
        y0 = ((t / tiles_x) * a.num_parts + a.part) * 16;
    };
    auto load = [&](int x0, int y0, float4& f0, float4& f1) {
        f0 = accAt(a, x0 + tid % 20 - 2, y0 + tid / 20 - 2);
        if (tid + 256 < 400) f1 = accAt(a, x0 + (tid + 256) % 20 - 2, y0 + (tid + 256) / 20 - 2);
    };
    int bid = (int)blockIdx.x, nblk = (int)gridDim.x;
    if (a.ob_cost) {   // block 0: the next megakernel draw's order (pt_order_build), beside the tiles
        if (bid == 0) {
            orderBuild(a.ob_ntiles, a.ob_cost, a.ob_order, a.ob_split, a.ob_cap, a.ob_dominance, a.ob_near);
            return;
        }
        bid--; nblk--;
    }
    int t = bid, x0, y0;
    if (t >= ntiles) return;
    origin(t, x0, y0);
    float4 f0, f1 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    load(x0, y0, f0, f1);
    tile[0][tid] = f0;
    if (tid + 256 < 400) tile[0][tid + 256] = f1;
    __syncthreads();
    for (int cur = 0; t < ntiles; cur ^= 1) {
        const int tn = t + nblk;
        int nx0 = 0, ny0 = 0;
        if (tn < ntiles) { origin(tn, nx0, ny0); load(nx0, ny0, f0, f1); }
        const int x = x0 + lx, y = y0 + ly;
        if (x < a.width && y < a.height) outputPixel(a, tile[cur], lx, ly, x, y);
        if (tn < ntiles) {
            tile[cur ^ 1][tid] = f0;
            if (tid + 256 < 400) tile[cur ^ 1][tid + 256] = f1;
        }
        __syncthreads();
        t = tn; x0 = nx0; y0 = ny0;
    }
}

// The same as one-wave workgroups (see pt_blend_w): 64 threads stage a tile's 20x20 neighbourhood (7
// texels each, the next tile's loaded into registers while this one is shaded) and shade 4 pixels each
__global__ __launch_bounds__(64) void pt_output_w(OutputArgs a, int tiles_x, int ntiles)
{
    __shared__ float4 tile[2][20 * 20];
    const int tid = threadIdx.x;
    const int lx = tid & 15, ly = tid >> 4;
    auto origin = [&](int t, int& x0, int& y0) {
        x0 = (t % tiles_x) * 16;
        y0 = ((t / tiles_x) * a.num_parts + a.part) * 16;
    };
    float4 f[7];
    auto load = [&](int x0, int y0) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int k = tid + 64 * i;
            if (k < 400) f[i] = accAt(a, x0 + k % 20 - 2, y0 + k / 20 - 2);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int k = tid + 64 * i;
            if (k < 400) tile[buf][k] = f[i];
        }
    };
    int bid = (int)blockIdx.x, nblk = (int)gridDim.x;
    if (a.ob_cost) {   // block 0: the next megakernel draw's order (pt_order_build), beside the tiles
        if (bid == 0) {
            orderBuild(a.ob_ntiles, a.ob_cost, a.ob_order, a.ob_split, a.ob_cap, a.ob_dominance, a.ob_near);
            return;
        }
        bid--; nblk--;
    }
    int t = bid, x0, y0;
    if (t >= ntiles) return;
    origin(t, x0, y0);
    load(x0, y0);
    store(0);
    __syncthreads();
    for (int cur = 0; t < ntiles; cur ^= 1) {
        const int tn = t + nblk;
        int nx0 = 0, ny0 = 0;
        if (tn < ntiles) { origin(tn, nx0, ny0); load(nx0, ny0); }
#pragma unroll 1
        for (int j = 0; j < 4; j++) {
            const int x = x0 + lx, y = y0 + ly + 4 * j;
            if (x < a.width && y < a.height) outputPixel(a, tile[cur], lx, ly + 4 * j, x, y);
        }
        if (tn < ntiles) store(cur ^ 1);
        __syncthreads();
        t = tn; x0 = nx0; y0 = ny0;
    }
}

// ------------------------------------------------------------------------------ child-pair BVH records
// Built once per (tAABBTexture, tTriangleTexture) upload; walked by bvhWalkPairs (pt_device.h).
// Every value is read from the reference textures with the same fetch32 / float index arithmetic
// the reference walk uses, so the boxes, codes and triangles equal what that walk would fetch.
//   pass 1  kinds: inner node (idObject < 0); leaf referenced as a child of an inner node (or the
//           root); `bad` flags links the records cannot express (right child not an exact integer
//           in [0, nrec), left child n+1 beyond the texture) -> the host keeps the reference walk
//   pass 2  per 1024-node block counts; the host scans them
//   pass 3  dense ranks -> rank codes: inner rank, or -1 - leaf rank
//   pass 4  inner records (64 B): A.min.xyz A.max.x | A.max.yz B.min.xy | B.min.z B.max.xyz |
//           codeA codeB (pairLineWrite; pairCode: record byte offsets, float bits); leaf records (48 B):
//           v0, e1 = v1 - v0, e2 = v2 - v0, idObject
constexpr int kPairsBlock = 1024;   // nodes per scan block (256 threads x 4)

__global__ __launch_bounds__(256) void pt_pairs_kinds(const float4* aabb, long long texels, unsigned nrec,
                                                      unsigned char* inner, unsigned char* leafref, unsigned* bad)
{
    const unsigned n = blockIdx.x * 256u + threadIdx.x;
    if (n >= nrec) return;
    const float fn = (float)n;   // exact: nrec <= 2^23
    const float4 c0 = fetch32(aabb, texels, fn * 2.0f), c1 = fetch32(aabb, texels, fn * 2.0f + 1.0f);
    const bool in = c0.x < 0.0f;
    inner[n] = in ? 1 : 0;
    // boxFast needs NaN-free boxes
    if (c0.y != c0.y || c0.z != c0.z || c0.w != c0.w || c1.y != c1.y || c1.z != c1.z || c1.w != c1.w) atomicOr(bad, 1u);
    if (n == 0 && !in) leafref[0] = 1;
    if (!in) return;
    const float idA = fn + 1.0f, idB = c1.x;
    const bool ok = idB >= 0.0f && idB < (float)nrec && floorf(idB) == idB && n + 1u < nrec;
    if (!ok) { atomicOr(bad, 1u); return; }
    const float4 a0 = fetch32(aabb, texels, idA * 2.0f), b0 = fetch32(aabb, texels, idB * 2.0f);
    if (!(a0.x < 0.0f)) leafref[n + 1u] = 1;
    if (!(b0.x < 0.0f)) leafref[(unsigned)idB] = 1;
}

__global__ __launch_bounds__(256) void pt_pairs_count(const unsigned char* inner, const unsigned char* leafref,
                                                      unsigned nrec, unsigned* counts)
{
    __shared__ unsigned si[256], sl[256];
    unsigned ci = 0, cl = 0;
    for (int k = 0; k < 4; k++) {
        const unsigned n = blockIdx.x * kPairsBlock + threadIdx.x * 4u + k;
        if (n < nrec) { ci += inner[n]; cl += leafref[n]; }
    }
    si[threadIdx.x] = ci; sl[threadIdx.x] = cl;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) { si[threadIdx.x] += si[threadIdx.x + o]; sl[threadIdx.x] += sl[threadIdx.x + o]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { counts[2 * blockIdx.x] = si[0]; counts[2 * blockIdx.x + 1] = sl[0]; }
}

__global__ __launch_bounds__(256) void pt_pairs_rank(const unsigned char* inner, const unsigned char* leafref,
                                                     unsigned nrec, const unsigned* offsets, float* code)
{
    __shared__ unsigned si[256], sl[256];
    unsigned fi[4], fl[4], ci = 0, cl = 0;
    for (int k = 0; k < 4; k++) {
        const unsigned n = blockIdx.x * kPairsBlock + threadIdx.x * 4u + k;
        fi[k] = n < nrec ? inner[n] : 0u;
        fl[k] = n < nrec ? leafref[n] : 0u;
        ci += fi[k]; cl += fl[k];
    }
    si[threadIdx.x] = ci; sl[threadIdx.x] = cl;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {   // inclusive Hillis-Steele scan
        unsigned vi = threadIdx.x >= (unsigned)o ? si[threadIdx.x - o] : 0u;
        unsigned vl = threadIdx.x >= (unsigned)o ? sl[threadIdx.x - o] : 0u;
        __syncthreads();
        si[threadIdx.x] += vi; sl[threadIdx.x] += vl;
        __syncthreads();
    }
    unsigned ri = offsets[2 * blockIdx.x] + si[threadIdx.x] - ci;
    unsigned rl = offsets[2 * blockIdx.x + 1] + sl[threadIdx.x] - cl;
    for (int k = 0; k < 4; k++) {
        const unsigned n = blockIdx.x * kPairsBlock + threadIdx.x * 4u + k;
        if (n >= nrec) break;
        float cd = 0.0f;
        if (fi[k]) cd = (float)ri;
        else if (fl[k]) cd = -1.0f - (float)rl;
        code[n] = cd;
        ri += fi[k]; rl += fl[k];
    }
}

__global__ __launch_bounds__(256) void pt_pairs_build(const float4* aabb, long long texels, const float4* tri,
                                                      long long tri_texels, unsigned nrec, const float* code,
                                                      float4* inner_rec, float4* leaf_rec,
                                                      const unsigned char* inner, const unsigned char* leafref,
                                                      unsigned leaf_base)
{
    const unsigned n = blockIdx.x * 256u + threadIdx.x;
    if (n >= nrec) return;
    const float fn = (float)n;
    if (inner[n]) {
        const float4 c1 = fetch32(aabb, texels, fn * 2.0f + 1.0f);
        const float idA = fn + 1.0f, idB = c1.x;
        const float4 a0 = fetch32(aabb, texels, idA * 2.0f), a1 = fetch32(aabb, texels, idA * 2.0f + 1.0f);
        const float4 b0 = fetch32(aabb, texels, idB * 2.0f), b1 = fetch32(aabb, texels, idB * 2.0f + 1.0f);
        float4* o = inner_rec + 4ull * (unsigned)code[n];
        pairLineWrite(o, a0, a1, b0, b1);
        o[3] = make_float4(__uint_as_float(pairCode(code[n + 1u], leaf_base)),
                           __uint_as_float(pairCode(code[(unsigned)idB], leaf_base)), 0.0f, 0.0f);
    } else if (leafref[n]) {
        const float hdr = fetch32(aabb, texels, fn * 2.0f).x;
        const float id = 8.0f * hdr;
        const float4 t0 = fetch32(tri, tri_texels, id), t1 = fetch32(tri, tri_texels, id + 1.0f),
                     t2 = fetch32(tri, tri_texels, id + 2.0f);
        // edges e1 = v1 - v0, e2 = v2 - v0 are the walk's first two IEEE subtractions, done here once
        const f3 v0 = mk(t0.x, t0.y, t0.z), e1 = mk(t0.w, t1.x, t1.y) - v0, e2 = mk(t1.z, t1.w, t2.x) - v0;
        float4* o = leaf_rec + 3ull * (unsigned)(-1.0f - code[n]);
        o[0] = make_float4(v0.x, v0.y, v0.z, e1.x);
        o[1] = make_float4(e1.y, e1.z, e2.x, e2.y);
        o[2] = make_float4(e2.z, hdr, 0.0f, 0.0f);
    }
}

// Restart-trail prerequisites (PROG_TRAIL, bvhWalkTrail in pt_device.h), after the records:
//   links  every child link of an inner node counted (refs) and its parent noted; a node linked twice,
//          or the root linked at all, is no tree -> *flag
//   depth  every linked node climbs its parents to the root within kTrailMaxDepth steps, else *flag
//          (the trail has one bit per depth; unreachable runs are skipped)
//   top    the jump table: for each depth p <= kTopLevels and path (p A/B bits, heap order) the
//          inner record the path reaches, copied (64 B); zero where the path meets a leaf first
__global__ __launch_bounds__(256) void pt_pairs_links(const float4* aabb, long long texels, unsigned nrec,
                                                      const unsigned char* inner, unsigned* parent, unsigned* refs,
                                                      unsigned* flag)
{
    const unsigned n = blockIdx.x * 256u + threadIdx.x;
    if (n >= nrec || !inner[n]) return;
    const unsigned c[2] = { n + 1u, (unsigned)fetch32(aabb, texels, (float)n * 2.0f + 1.0f).x };   // exact: checked by pass 1
    for (int k = 0; k < 2; k++) {
        const unsigned old = atomicAdd(&refs[c[k]], 1u);
        parent[c[k]] = n;
        if (old != 0u || c[k] == 0u) atomicOr(flag, 1u);
    }
}

__global__ __launch_bounds__(256) void pt_pairs_depth(unsigned nrec, const unsigned* parent, const unsigned* refs,
                                                      unsigned* flag)
{
    const unsigned n = blockIdx.x * 256u + threadIdx.x;
    if (n >= nrec || n == 0u || refs[n] == 0u) return;
    unsigned m = n;
    for (int d = 1; d <= kTrailMaxDepth; d++) {
        m = parent[m];
        if (m == 0u) return;
        if (refs[m] == 0u) return;   // a run that is not reached from the root
    }
    atomicOr(flag, 1u);
}

__global__ __launch_bounds__(256) void pt_pairs_top(const float4* rec, uint32_t root, float4* top)
{
    for (unsigned idx = threadIdx.x; idx < kTopEntries; idx += blockDim.x) {
        const int p = 31 - __builtin_clz(idx + 1u);
        const unsigned prefix = idx + 1u - (1u << p);
        uint32_t code = root;
        bool ok = true;
        for (int j = 0; j < p && ok; j++) {
            if (code & kLeafBit) { ok = false; break; }
            const float4 c = rec[code / 16u + 3u];
            code = __float_as_uint(((prefix >> (p - 1 - j)) & 1u) ? c.y : c.x);
        }
        if (code & kLeafBit) ok = false;
        for (int q = 0; q < 4; q++) top[4u * idx + q] = ok ? rec[code / 16u + q] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

// ------------------------------------------------------------------------------ self-test
// every binary32 pattern with bits 31..24 == hi: fast device sequence vs the IEEE operation it
// stands for (NaN == NaN); one atomic per wave with a mismatch
__global__ __launch_bounds__(256) void pt_exhaustive_kernel(int op, uint32_t hi, unsigned long long* bad)
{
    const uint32_t bits = (hi << 24) | (blockIdx.x * 256u + threadIdx.x);
    const float x = __uint_as_float(bits);
    float got = 0.0f, ref = 0.0f;
    if (op == 0) { got = grcp(x); ref = 1.0f / x; }
    else if (op == 1) { got = gsqrt(x); ref = sqrtf(x); }
    const bool ok = (ref != ref) ? (got != got) : (__float_as_uint(got) == __float_as_uint(ref));
    const unsigned long long m = __ballot(!ok);
    if (m && (threadIdx.x & 63u) == (unsigned)(__ffsll((long long)m) - 1)) atomicAdd(bad, (unsigned long long)__popcll(m));
}

__global__ void pt_math_probe_kernel(int op, const float* x, const float* y, float* out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = x[i], b = y ? y[i] : 0.0f;
    float r = 0.0f;
    switch (op) {
    case 0: r = gexp2(a); break;
    case 1: r = glog2(a); break;
    case 2: r = gsin(a); break;
    case 3: r = gcos(a); break;
    case 4: r = gatan(a); break;
    case 5: r = gatan2(a, b); break;
    case 6: r = gacos(a); break;
    case 7: r = gpow(a, b); break;
    case 8: r = gexp(a); break;
    case 9: r = glog(a); break;
    case 10: r = gsqrt(a); break;
    case 11: { Path p; p.s0 = (uint32_t)a; p.s1 = (uint32_t)b; r = rng(p); break; }
    case 12: r = a / b; break;
    case 13: r = grcp(gsqrt(a)); break;
    case 14: r = grcp(a); break;
    default: r = 0.0f;
    }
    out[i] = r;
}

// ------------------------------------------------------------------------------ pt_cont's record order
// (PT_CONT_SORT) between pt_trace and pt_cont on the draw's side stream: the records in the order of their
// ray keys (pt_trace.h contRank) - a counting sort whose counts and ranks pt_trace took as it stored the
// records, so what is left is the keys' first places (one wave: an exclusive scan of the totals, in place)
// and placing the records: perm[first place of the key + rank] = record. No LDS in either kernel: beside the
// path-tracing waves, which fill every CU's LDS, a workgroup that needs some waits for a wave to end.
__global__ __launch_bounds__(64) void pt_cont_offsets(SortArgs s)
{
    const unsigned lane = threadIdx.x, per = s.nbins / 64u;   // consecutive keys per lane
    unsigned* const bins = (unsigned*)s.bins;
    unsigned sum = 0;
#pragma unroll 16
    for (unsigned k = 0; k < per; k++) sum += bins[per * lane + k];
    unsigned inc = sum;   // inclusive scan over the lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(inc, d, 64);
        if (lane >= (unsigned)d) inc += o;
    }
    unsigned run = inc - sum;
    for (unsigned k = 0; k < per; k++) {
        const unsigned v = bins[per * lane + k];
        bins[per * lane + k] = run;
        run += v;
    }
}
__global__ __launch_bounds__(64) void pt_cont_scatter(SortArgs s)
{
    const unsigned n = *s.count;
    const unsigned begin = blockIdx.x * s.chunk, end = min(n, begin + s.chunk);
    // eight records per lane at a time, their loads issued together (each record is a chain of three:
    // key -> the key's first place -> the store)
    for (unsigned i0 = begin + threadIdx.x; i0 < end; i0 += 8u * 64u) {
        unsigned key[8], rank[8], at[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const unsigned i = i0 + 64u * k;
            key[k] = i < end ? (unsigned)s.key[i] : 0u;
            rank[k] = i < end ? s.rank[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) at[k] = s.bins[key[k]];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const unsigned i = i0 + 64u * k;
            if (i < end) s.perm[at[k] + rank[k]] = i;
        }
    }
}

} // namespace pt

// ------------------------------------------------------------------------------ launchers
#define PT_WALK_LAUNCHERS(W)                                                                                     \
    hipError_t pt_launch_trace_##W(int prog, int count, const pt::TraceArgs* a, dim3 grid, dim3 block, hipStream_t s); \
    hipError_t pt_launch_persist_##W(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x,   \
                                     unsigned n_wave_tiles, unsigned per_wave, unsigned refill, dim3 grid, dim3 block, \
                                     hipStream_t s);                                                                \
    hipError_t pt_launch_cont_##W(int prog, const pt::TraceArgs* a, dim3 grid, hipStream_t s);
PT_WALK_LAUNCHERS(ref)
PT_WALK_LAUNCHERS(pairs)
PT_WALK_LAUNCHERS(trail)
#undef PT_WALK_LAUNCHERS

extern "C" {

// the megakernel of a draw: the program variant's walk picks the translation unit that holds it
// (pt_trace_walk*.hip)
hipError_t pt_launch_trace(int prog, int count, const pt::TraceArgs* a, int grid_x, int grid_y, hipStream_t s)
{
    const dim3 grid(grid_x * pt::kTraceSub, grid_y), block(pt::kTraceBlock);
    // texture-free models (the bench's StanfordBunny) take the variant without PBR code
    prog = pt::resolveProgram(prog, a->uses_albedo || a->uses_bump, a->bvh_walk);
    switch (prog / pt::PROG_PAIRS) {
    case pt::WALK_REF: return pt_launch_trace_ref(prog, count, a, grid, block, s);
    case pt::WALK_PAIRS: return pt_launch_trace_pairs(prog, count, a, grid, block, s);
    case pt::WALK_TRAIL: return pt_launch_trace_trail(prog, count, a, grid, block, s);
    default: return hipErrorInvalidValue;
    }
}

// late-bounce compaction: pt_cont over the paths the draw's pt_trace stored (`waves` one-wave workgroups)
hipError_t pt_launch_cont(int prog, const pt::TraceArgs* a, int waves, hipStream_t s)
{
    prog = pt::resolveProgram(prog, a->uses_albedo || a->uses_bump, a->bvh_walk);
    const dim3 grid(waves);
    switch (prog / pt::PROG_PAIRS) {
    case pt::WALK_REF: return pt_launch_cont_ref(prog, a, grid, s);
    case pt::WALK_PAIRS: return pt_launch_cont_pairs(prog, a, grid, s);
    case pt::WALK_TRAIL: return pt_launch_cont_trail(prog, a, grid, s);
    default: return hipErrorInvalidValue;
    }
}

// (PT_CONT_SORT) the record order of a draw's pt_cont: up to `cap` records
hipError_t pt_launch_cont_sort(const pt::SortArgs* a, size_t cap, hipStream_t s)
{
    const unsigned blocks = (unsigned)((cap + a->chunk - 1) / a->chunk);
    hipLaunchKernelGGL(pt::pt_cont_offsets, dim3(1), dim3(64), 0, s, *a);
    hipLaunchKernelGGL(pt::pt_cont_scatter, dim3(blocks ? blocks : 1), dim3(64), 0, s, *a);
    return hipGetLastError();
}

hipError_t pt_launch_order_build(unsigned ntiles, const unsigned* cost, unsigned* order, unsigned* split,
                                 unsigned split_cap, unsigned dominance, int near_buckets, hipStream_t s, int threads)
{
    hipLaunchKernelGGL(pt::pt_order_build, dim3(1), dim3(threads), 0, s, ntiles, cost, order, split, split_cap, dominance,
                       near_buckets);
    return hipGetLastError();
}

hipError_t pt_launch_persist(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w, int tiles_x,
                             unsigned n_wave_tiles, unsigned per_wave, unsigned refill, hipStream_t s)
{
    prog = pt::resolveProgram(prog, a->uses_albedo || a->uses_bump, a->bvh_walk);
    const unsigned waves = (n_wave_tiles + per_wave - 1) / per_wave;
    const dim3 grid((waves + 3) / 4), block(pt::kBlock);
    switch (prog / pt::PROG_PAIRS) {
    case pt::WALK_REF: return pt_launch_persist_ref(prog, count, a, w, tiles_x, n_wave_tiles, per_wave, refill, grid, block, s);
    case pt::WALK_PAIRS: return pt_launch_persist_pairs(prog, count, a, w, tiles_x, n_wave_tiles, per_wave, refill, grid, block, s);
    case pt::WALK_TRAIL: return pt_launch_persist_trail(prog, count, a, w, tiles_x, n_wave_tiles, per_wave, refill, grid, block, s);
    default: return hipErrorInvalidValue;
    }
}

// the four passes of the child-pair build; `offsets` is filled by the host between pass 2 and 3
hipError_t pt_launch_pairs_pass(int pass, const float4* aabb, long long texels, const float4* tri, long long tri_texels,
                                unsigned nrec, unsigned char* inner, unsigned char* leafref, unsigned* counts,
                                float* code, float4* inner_rec, float4* leaf_rec, unsigned leaf_base, unsigned* bad,
                                hipStream_t s)
{
    const dim3 nodes((nrec + 255) / 256), blocks((nrec + pt::kPairsBlock - 1) / pt::kPairsBlock), b256(256);
    switch (pass) {
    case 1: hipLaunchKernelGGL(pt::pt_pairs_kinds, nodes, b256, 0, s, aabb, texels, nrec, inner, leafref, bad); break;
    case 2: hipLaunchKernelGGL(pt::pt_pairs_count, blocks, b256, 0, s, inner, leafref, nrec, counts); break;
    case 3: hipLaunchKernelGGL(pt::pt_pairs_rank, blocks, b256, 0, s, inner, leafref, nrec, counts, code); break;
    case 4:
        hipLaunchKernelGGL(pt::pt_pairs_build, nodes, b256, 0, s, aabb, texels, tri, tri_texels, nrec, code, inner_rec,
                           leaf_rec, inner, leafref, leaf_base);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the restart-trail passes: 1 links, 2 depth, 3 top (rec = the record array, top its jump table)
hipError_t pt_launch_trail_pass(int pass, const float4* aabb, long long texels, unsigned nrec, const unsigned char* inner,
                                unsigned* parent, unsigned* refs, unsigned* flag, const float4* rec, uint32_t root,
                                float4* top, hipStream_t s)
{
    const dim3 nodes((nrec + 255) / 256), b256(256);
    switch (pass) {
    case 1: hipLaunchKernelGGL(pt::pt_pairs_links, nodes, b256, 0, s, aabb, texels, nrec, inner, parent, refs, flag); break;
    case 2: hipLaunchKernelGGL(pt::pt_pairs_depth, nodes, b256, 0, s, nrec, parent, refs, flag); break;
    case 3: hipLaunchKernelGGL(pt::pt_pairs_top, dim3(1), b256, 0, s, rec, root, top); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t pt_launch_blend(const pt::BlendArgs* a, int bands, hipStream_t s, int waves)
{
    if (bands <= 0) return hipSuccess;
    if (waves > 0) {
        const int ux = (a->width + 63) / 64, units = ux * bands * 4;
        hipLaunchKernelGGL(pt::pt_blend_w, dim3(units < waves ? units : waves), dim3(64), 0, s, *a, ux, units);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(pt::pt_blend, dim3((a->width + 63) / 64, bands), dim3(256), 0, s, *a);
    return hipGetLastError();
}

hipError_t pt_launch_copy(const pt::CopyArgs* a, int grid_x, int grid_y, hipStream_t s)
{
    hipLaunchKernelGGL(pt::pt_copy, dim3(grid_x, grid_y), dim3(256), 0, s, *a);
    return hipGetLastError();
}

hipError_t pt_launch_output(const pt::OutputArgs* a, hipStream_t s, int waves)
{
    const int nb = (a->height + 15) / 16;
    dim3 grid((a->width + 15) / 16, a->part < nb ? (nb - a->part + a->num_parts - 1) / a->num_parts : 0);
    if (grid.y == 0) {   // no band of this part: a fused order build runs on its own
        if (a->ob_cost)
            hipLaunchKernelGGL(pt::pt_order_build, dim3(1), dim3(1024), 0, s, a->ob_ntiles, a->ob_cost, a->ob_order,
                               a->ob_split, a->ob_cap, a->ob_dominance, a->ob_near);
        return hipGetLastError();
    }
    // persistent screenOutput blocks: about four 16x16 tiles each, 4096..8192 (1080p 4096: 37.2 ->
    // 36.1 us; 4K 8192: 122 -> 109 us; profiles/r02i_ab_out_blocks.txt); PT_OUT_BLOCKS fixes the count
    const int ntiles = (int)(grid.x * grid.y);
    if (waves > 0) {
        hipLaunchKernelGGL(pt::pt_output_w, dim3((ntiles < waves ? ntiles : waves) + (a->ob_cost ? 1 : 0)), dim3(64), 0, s,
                           *a, (int)grid.x, ntiles);
        return hipGetLastError();
    }
#ifdef PT_OUT_BLOCKS
    const int blocks = PT_OUT_BLOCKS;
#else
    const int blocks = ntiles / 4 < 4096 ? 4096 : ntiles / 4 > 8192 ? 8192 : ntiles / 4;
#endif
    hipLaunchKernelGGL(pt::pt_output, dim3((ntiles < blocks ? ntiles : blocks) + (a->ob_cost ? 1 : 0)), dim3(256), 0, s, *a,
                       (int)grid.x, ntiles);
    return hipGetLastError();
}

hipError_t pt_launch_exhaustive(int op, unsigned long long* bad, hipStream_t s)
{
    for (uint32_t hi = 0; hi < 256u; hi++)
        hipLaunchKernelGGL(pt::pt_exhaustive_kernel, dim3(65536), dim3(256), 0, s, op, hi, bad);
    return hipGetLastError();
}

hipError_t pt_launch_math_probe(int op, const float* x, const float* y, float* out, int n, hipStream_t s)
{
    hipLaunchKernelGGL(pt::pt_math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, op, x, y, out, n);
    return hipGetLastError();
}

}
