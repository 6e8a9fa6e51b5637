// pt_bvh_gpu.hip — BVH_Build_Iterative (js/BVH_Fast_Builder.js:43-406) on the device: the same
// tree as pt_bvh_build (csrc/pt_bvh_build.cpp), bit for bit, built level by level.
//
// The reference builds depth-first with a work-list stack; the tree it emits is a function of the
// input only: a node is a run of the work list, split at the double (min + max) * 0.5 of its box
// on the first axis (longest extent first) whose centroid test separates the run, or dealt
// alternately when none does; children keep their parent's order; nodes are numbered depth-first,
// left subtree first. A subtree over k triangles has 2k - 1 nodes, so a node's id follows from its
// parent's: left = p + 1, right = p + 2 * nLeft. That makes every level of the tree independent
// work: all runs of one depth are split together.
//
// Device state, all n-sized: perm (the work list, runs contiguous), runb (each position's run
// start); per run, indexed by its start b: size, node id, box keys, split, axis counts. One level:
//   pt_bvh_box     per element: the run's box as order-preserving integer keys (atomicMin/Max,
//                  one atomic per wave when the wave's lanes share a run) + NaN flags
//   pt_bvh_split   per run: box -> doubles, split (double), axis order by extent
//   pt_bvh_count   per element: centroid < split on all three axes (ballot counts per wave)
//   pt_bvh_choose  per run: the first separating axis (or the alternate deal), the inner node
//   pt_bvh_flag    per element: goes left?
//   (exclusive scan of the flags, hipCUB)
//   pt_bvh_move    per element: stable partition into perm2 / runb2; leaf nodes of 1-runs
//   pt_bvh_next    per run: the two child runs (size, node id), reset their accumulators
// The host loops until a level leaves no run of 2 or more (one 4-byte read per level).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <vector>

#include "../../include/pt.h"

namespace ptb {

constexpr int kBlock = 256;
constexpr uint32_t kNaN = 0x7fc00000u;   // (float)NAN: what the host builder stores for a NaN bound

// float -> unsigned key whose unsigned order is the float order with -0 < +0 (NaN kept apart)
__device__ inline uint32_t fkey(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float fkeyInv(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// (float)(double)x of the host builder: a float -> double -> float round trip (quiets a signalling NaN)
__device__ inline float viaDouble(float x) { return (float)(double)x; }

struct Level {
    const float* aabb;       // 9 floats per triangle: min.xyz, max.xyz, centroid.xyz
    const uint32_t* perm;    // this level's work list
    const uint32_t* runb;    // run start of every position
    uint32_t* perm2;
    uint32_t* runb2;
    uint32_t* size;          // per run start: run length (0 = not a run start)
    uint32_t* node;          // per run start: node id
    uint32_t* kmin;          // [3][n] box keys
    uint32_t* kmax;
    uint32_t* knan;          // bit a: a NaN among the mins of axis a; bit 3 + a: among the maxes
    uint32_t* cnt;           // [3][n] centroid < split counts
    double* split;           // [3][n]
    int* order;              // per run start: the axis order, 3 bits each (a0 | a1 << 2 | a2 << 4)
    int* axis;               // per run start: the chosen axis, -1 = alternate deal
    uint32_t* nleft;         // per run start: elements going left
    uint32_t* flag;          // per element
    const uint32_t* scan;    // exclusive scan of flag
    float* out;              // 8 floats per node
    uint32_t* more;          // runs of >= 2 left for the next level
    uint32_t n;
};

__device__ inline bool activeRun(const Level& L, uint32_t b) { return L.size[b] >= 2u; }
__device__ inline float centroid(const Level& L, uint32_t k, int a) { return L.aabb[9ull * k + 6 + a]; }

__global__ __launch_bounds__(kBlock) void pt_bvh_box(Level L)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const bool in = i < L.n;
    const uint32_t b = in ? L.runb[i] : 0xffffffffu;
    const bool act = in && activeRun(L, b);
    const uint32_t k = act ? L.perm[i] : 0u;
    uint32_t mn[3], mx[3], nanbits = 0;
    for (int a = 0; a < 3; a++) {
        const float lo = act ? L.aabb[9ull * k + a] : 0.0f, hi = act ? L.aabb[9ull * k + 3 + a] : 0.0f;
        if (lo != lo) nanbits |= 1u << a;
        if (hi != hi) nanbits |= 8u << a;
        mn[a] = (act && lo == lo) ? fkey(lo) : 0xffffffffu;
        mx[a] = (act && hi == hi) ? fkey(hi) : 0u;
    }
    // one atomic per wave when every active lane is in the same run (the upper levels)
    const uint64_t actm = __ballot(act);
    if (!actm) return;
    const uint32_t b0 = __shfl(b, __ffsll((long long)actm) - 1, 64);
    if (__ballot(act && b != b0) == 0ull) {
        for (int o = 32; o > 0; o >>= 1) {
            for (int a = 0; a < 3; a++) {
                mn[a] = min(mn[a], (uint32_t)__shfl_xor((int)mn[a], o, 64));
                mx[a] = max(mx[a], (uint32_t)__shfl_xor((int)mx[a], o, 64));
            }
            nanbits |= (uint32_t)__shfl_xor((int)nanbits, o, 64);
        }
        if (i % 64u == (uint32_t)(__ffsll((long long)actm) - 1)) {
            for (int a = 0; a < 3; a++) {
                atomicMin(&L.kmin[a * L.n + b0], mn[a]);
                atomicMax(&L.kmax[a * L.n + b0], mx[a]);
            }
            if (nanbits) atomicOr(&L.knan[b0], nanbits);
        }
        return;
    }
    if (!act) return;
    for (int a = 0; a < 3; a++) {
        atomicMin(&L.kmin[a * L.n + b], mn[a]);
        atomicMax(&L.kmax[a * L.n + b], mx[a]);
    }
    if (nanbits) atomicOr(&L.knan[b], nanbits);
}

// the run's box as the host builder's doubles: Math.min / Math.max folds (NaN wins)
__device__ inline void runBox(const Level& L, uint32_t b, double mn[3], double mx[3])
{
    const uint32_t nb = L.knan[b];
    for (int a = 0; a < 3; a++) {
        mn[a] = (nb >> a) & 1u ? (double)__uint_as_float(kNaN) : (double)fkeyInv(L.kmin[a * L.n + b]);
        mx[a] = (nb >> (3 + a)) & 1u ? (double)__uint_as_float(kNaN) : (double)fkeyInv(L.kmax[a * L.n + b]);
    }
}

__global__ __launch_bounds__(kBlock) void pt_bvh_split(Level L)
{
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= L.n || L.runb[b] != b || !activeRun(L, b)) return;
    double mn[3], mx[3];
    runBox(L, b, mn, mx);
    for (int a = 0; a < 3; a++) L.split[a * L.n + b] = (mn[a] + mx[a]) * 0.5;   // spatial median
    // longest extent first, then the other two (js/BVH_Fast_Builder.js:120-186)
    const double s0 = mx[0] - mn[0], s1 = mx[1] - mn[1], s2 = mx[2] - mn[2];
    int ax[3] = { 0, 1, 2 };
    if (s0 >= s1 && s0 >= s2) { ax[0] = 0; ax[1] = s1 >= s2 ? 1 : 2; ax[2] = s1 >= s2 ? 2 : 1; }
    else if (s1 > s0 && s1 >= s2) { ax[0] = 1; ax[1] = s0 >= s2 ? 0 : 2; ax[2] = s0 >= s2 ? 2 : 0; }
    else if (s2 > s0 && s2 > s1) { ax[0] = 2; ax[1] = s0 >= s1 ? 0 : 1; ax[2] = s0 >= s1 ? 1 : 0; }
    L.order[b] = ax[0] | (ax[1] << 2) | (ax[2] << 4);
}

__global__ __launch_bounds__(kBlock) void pt_bvh_count(Level L)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const bool in = i < L.n;
    const uint32_t b = in ? L.runb[i] : 0xffffffffu;
    const bool act = in && activeRun(L, b);
    bool lt[3] = { false, false, false };
    if (act) {
        const uint32_t k = L.perm[i];
        for (int a = 0; a < 3; a++) lt[a] = (double)centroid(L, k, a) < L.split[a * L.n + b];
    }
    const uint64_t actm = __ballot(act);
    if (!actm) return;
    const int first = __ffsll((long long)actm) - 1;
    const uint32_t b0 = __shfl(b, first, 64);
    if (__ballot(act && b != b0) == 0ull) {
        const uint32_t c[3] = { (uint32_t)__popcll(__ballot(lt[0])), (uint32_t)__popcll(__ballot(lt[1])),
                                (uint32_t)__popcll(__ballot(lt[2])) };
        if ((int)(i % 64u) == first)
            for (int a = 0; a < 3; a++)
                if (c[a]) atomicAdd(&L.cnt[a * L.n + b0], c[a]);
        return;
    }
    if (!act) return;
    for (int a = 0; a < 3; a++)
        if (lt[a]) atomicAdd(&L.cnt[a * L.n + b], 1u);
}

__device__ inline void writeNode(float* out, uint32_t id, float idObject, const float mn[3], float idRight, const float mx[3])
{
    float* o = out + 8ull * id;
    o[0] = idObject; o[1] = mn[0]; o[2] = mn[1]; o[3] = mn[2];
    o[4] = idRight;  o[5] = mx[0]; o[6] = mx[1]; o[7] = mx[2];
}

__global__ __launch_bounds__(kBlock) void pt_bvh_choose(Level L)
{
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= L.n || L.runb[b] != b || !activeRun(L, b)) return;
    const uint32_t sz = L.size[b];
    const int ord = L.order[b];
    int axis = -1;
    uint32_t nl = 0;
    for (int j = 0; j < 3; j++) {
        const int a = (ord >> (2 * j)) & 3;
        const uint32_t c = L.cnt[a * L.n + b];
        if (c > 0u && c < sz) { axis = a; nl = c; break; }
    }
    if (axis < 0) nl = (sz + 1u) / 2u;   // even positions go left (js/BVH_Fast_Builder.js:281-313)
    L.axis[b] = axis;
    L.nleft[b] = nl;
    double mn[3], mx[3];
    runBox(L, b, mn, mx);
    const float fmn[3] = { (float)mn[0], (float)mn[1], (float)mn[2] }, fmx[3] = { (float)mx[0], (float)mx[1], (float)mx[2] };
    const uint32_t p = L.node[b];
    writeNode(L.out, p, -1.0f, fmn, (float)(p + 2u * nl), fmx);
}

__global__ __launch_bounds__(kBlock) void pt_bvh_flag(Level L)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t b = L.runb[i];
    uint32_t f = 0;
    if (activeRun(L, b)) {
        const int a = L.axis[b];
        f = a >= 0 ? ((double)centroid(L, L.perm[i], a) < L.split[a * L.n + b] ? 1u : 0u) : ((i - b) % 2u == 0u ? 1u : 0u);
    }
    L.flag[i] = f;
}

__global__ __launch_bounds__(kBlock) void pt_bvh_move(Level L)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t b = L.runb[i];
    const uint32_t k = L.perm[i];
    if (!activeRun(L, b)) { L.perm2[i] = k; L.runb2[i] = b; return; }   // a finished leaf keeps its place
    const uint32_t nl = L.nleft[b], sz = L.size[b], p = L.node[b];
    const uint32_t rankL = L.scan[i] - L.scan[b];
    const bool left = L.flag[i] != 0u;
    const uint32_t pos = left ? b + rankL : b + nl + (i - b - rankL);
    const uint32_t cb = left ? b : b + nl;
    L.perm2[pos] = k;
    L.runb2[pos] = cb;
    const uint32_t csz = left ? nl : sz - nl;
    if (csz == 1u) {   // a leaf: idObject, the triangle's own box (js/BVH_Fast_Builder.js:59-75)
        const float* t = L.aabb + 9ull * k;
        const float fmn[3] = { viaDouble(t[0]), viaDouble(t[1]), viaDouble(t[2]) };
        const float fmx[3] = { viaDouble(t[3]), viaDouble(t[4]), viaDouble(t[5]) };
        writeNode(L.out, left ? p + 1u : p + 2u * nl, (float)k, fmn, -1.0f, fmx);
    }
}

__device__ inline void resetRun(const Level& L, uint32_t b)
{
    for (int a = 0; a < 3; a++) { L.kmin[a * L.n + b] = 0xffffffffu; L.kmax[a * L.n + b] = 0u; L.cnt[a * L.n + b] = 0u; }
    L.knan[b] = 0u;
}

__global__ __launch_bounds__(kBlock) void pt_bvh_next(Level L)
{
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= L.n || L.runb[b] != b || !activeRun(L, b)) return;
    const uint32_t nl = L.nleft[b], sz = L.size[b], p = L.node[b];
    L.size[b] = nl;            L.node[b] = p + 1u;
    L.size[b + nl] = sz - nl;  L.node[b + nl] = p + 2u * nl;
    uint32_t runs = 0;
    if (nl >= 2u) { resetRun(L, b); runs++; }
    if (sz - nl >= 2u) { resetRun(L, b + nl); runs++; }
    if (runs) atomicAdd(L.more, runs);
}

__global__ __launch_bounds__(kBlock) void pt_bvh_init(Level L, const uint32_t* work)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= L.n) return;
    L.perm2[i] = work[i];   // (the host swaps: perm2 is the first level's perm)
    L.runb2[i] = 0u;
    L.size[i] = i == 0u ? L.n : 0u;
    L.node[i] = 0u;
    resetRun(L, i);
}

}  // namespace ptb

namespace {

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
};

}  // namespace

// pt_bvh_build_gpu: include/pt.h
extern "C" int pt_bvh_build_gpu(int device, const float* aabb_in, const uint32_t* work, int n, float* nodes_out,
                                int max_nodes, float* ms_out)
{
    using namespace ptb;
    if (!aabb_in || !work || !nodes_out || n < 1) return PT_ERR_ARG;
    const long long nodes = 2ll * n - 1;
    if (nodes > max_nodes || n > (1 << 24)) return PT_ERR_ARG;   // node ids are exact floats below 2^24
    uint32_t kmax = 0;
    for (int i = 0; i < n; i++) kmax = work[i] > kmax ? work[i] : kmax;
    if (hipSetDevice(device) != hipSuccess) return PT_ERR_DEVICE;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return PT_ERR_HIP;
    const size_t N = (size_t)n, tri = (size_t)kmax + 1;
    // one allocation, carved: aabb, work, perm x2, runb x2, size, node, kmin/kmax/cnt [3N],
    // knan, order, axis, nleft, flag, scan, split [3N] doubles, out, more, scan temp
    size_t scanTemp = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, scanTemp, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s);
    size_t off = 0;
    auto carve = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t oAabb = carve(tri * 9 * 4), oWork = carve(N * 4), oPerm = carve(N * 4), oPerm2 = carve(N * 4),
                 oRunb = carve(N * 4), oRunb2 = carve(N * 4), oSize = carve(N * 4), oNode = carve(N * 4),
                 oKmin = carve(3 * N * 4), oKmax = carve(3 * N * 4), oCnt = carve(3 * N * 4), oKnan = carve(N * 4),
                 oOrder = carve(N * 4), oAxis = carve(N * 4), oNleft = carve(N * 4), oFlag = carve(N * 4),
                 oScan = carve(N * 4), oSplit = carve(3 * N * 8), oOut = carve((size_t)nodes * 32), oMore = carve(4),
                 oTemp = carve(scanTemp);
    DevBuf mem;
    int rc = PT_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&mem.p, off) != hipSuccess) { (void)hipStreamDestroy(s); return PT_ERR_OOM; }
    char* base = (char*)mem.p;
    auto at = [&](size_t o) { return (void*)(base + o); };
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    Level L;
    L.aabb = (const float*)at(oAabb);
    L.size = (uint32_t*)at(oSize); L.node = (uint32_t*)at(oNode);
    L.kmin = (uint32_t*)at(oKmin); L.kmax = (uint32_t*)at(oKmax); L.knan = (uint32_t*)at(oKnan);
    L.cnt = (uint32_t*)at(oCnt); L.split = (double*)at(oSplit); L.order = (int*)at(oOrder); L.axis = (int*)at(oAxis);
    L.nleft = (uint32_t*)at(oNleft); L.flag = (uint32_t*)at(oFlag); L.scan = (const uint32_t*)at(oScan);
    L.out = (float*)at(oOut); L.more = (uint32_t*)at(oMore); L.n = (uint32_t)n;
    uint32_t* perm[2] = { (uint32_t*)at(oPerm), (uint32_t*)at(oPerm2) };
    uint32_t* runb[2] = { (uint32_t*)at(oRunb), (uint32_t*)at(oRunb2) };
    const dim3 grid((unsigned)((N + kBlock - 1) / kBlock)), block(kBlock);
    int cur = 0;
    uint32_t more = 1;
    bool ok = hipMemcpyAsync(at(oAabb), aabb_in, tri * 9 * 4, hipMemcpyHostToDevice, s) == hipSuccess &&
              hipMemcpyAsync(at(oWork), work, N * 4, hipMemcpyHostToDevice, s) == hipSuccess;
    (void)hipEventRecord(e0, s);
    if (ok) {
        L.perm = perm[1]; L.runb = runb[1]; L.perm2 = perm[0]; L.runb2 = runb[0];
        hipLaunchKernelGGL(pt_bvh_init, grid, block, 0, s, L, (const uint32_t*)at(oWork));
        if (n == 1) more = 0;   // a single leaf: written below
    }
    // levels until no run of two or more triangles is left
    for (int level = 0; ok && more; level++) {
        L.perm = perm[cur]; L.runb = runb[cur]; L.perm2 = perm[cur ^ 1]; L.runb2 = runb[cur ^ 1];
        ok = hipMemsetAsync(L.more, 0, 4, s) == hipSuccess;
        hipLaunchKernelGGL(pt_bvh_box, grid, block, 0, s, L);
        hipLaunchKernelGGL(pt_bvh_split, grid, block, 0, s, L);
        hipLaunchKernelGGL(pt_bvh_count, grid, block, 0, s, L);
        hipLaunchKernelGGL(pt_bvh_choose, grid, block, 0, s, L);
        hipLaunchKernelGGL(pt_bvh_flag, grid, block, 0, s, L);
        ok = ok && hipcub::DeviceScan::ExclusiveSum(at(oTemp), scanTemp, L.flag, (uint32_t*)at(oScan), n, s) == hipSuccess;
        hipLaunchKernelGGL(pt_bvh_move, grid, block, 0, s, L);
        hipLaunchKernelGGL(pt_bvh_next, grid, block, 0, s, L);
        ok = ok && hipGetLastError() == hipSuccess;
        ok = ok && hipMemcpyAsync(&more, L.more, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        cur ^= 1;
        if (level > n) ok = false;   // every level splits every run: cannot happen
    }
    (void)hipEventRecord(e1, s);
    if (n == 1 && ok) {   // the root is the leaf: write it from the host's view of the input
        const float* t = aabb_in + 9ull * work[0];
        float o[8] = { (float)work[0], (float)(double)t[0], (float)(double)t[1], (float)(double)t[2],
                       -1.0f, (float)(double)t[3], (float)(double)t[4], (float)(double)t[5] };
        ok = hipMemcpyAsync(L.out, o, 32, hipMemcpyHostToDevice, s) == hipSuccess;
    }
    ok = ok && hipMemcpyAsync(nodes_out, L.out, (size_t)nodes * 32, hipMemcpyDeviceToHost, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    if (ok && ms_out) { float ms = 0.0f; (void)hipEventElapsedTime(&ms, e0, e1); *ms_out = ms; }
    if (!ok) rc = PT_ERR_HIP;
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return rc == PT_OK ? (int)nodes : rc;
}
