// Microbenchmark: cost of one BVH-walk-like step in the vector memory pipeline (TA/TD/L1) as a
// function of the load mix per step: 3 x dwordx4 + 1 x dwordx2 (the child-pair walk today),
// 3 x dwordx4 + 1 x dword, 3 x dwordx4, 4 x dwordx4, 2 x dwordx4; for 64 / 16 / 4 active lanes
// and 8 waves per SIMD (the walk's occupancy). Dependent chain: the next record offset is a function
// of the loaded data, as in a walk. Table L2-resident (1 MiB) and MALL-resident (48 MiB).
// build: hipcc --offload-arch=gfx950 -O3 -o td_width td_width.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int vu4 __attribute__((ext_vector_type(4)));
typedef unsigned int vu2 __attribute__((ext_vector_type(2)));

template <int MIX>
__global__ __launch_bounds__(64) void step(const unsigned* tab, unsigned tab_bytes, int iters, int active, unsigned* out)
{
    const int lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)tab_bytes, 0x00020000);
    const unsigned nrec = tab_bytes / 64u;
    unsigned off = ((blockIdx.x * 977u + (unsigned)lane * 131u) % nrec) * 64u;
    unsigned acc = 0;
    if (lane < active) {
        for (int i = 0; i < iters; i++) {
            vu4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            unsigned x = v.x;
            if (MIX != 4) {
                const vu4 w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 16, 0, 0);
                x ^= w.y;
            }
            if (MIX <= 3) {
                const vu4 w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 32, 0, 0);
                x ^= w.z;
            }
            if (MIX == 0) {
                const vu2 c = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off + 48, 0, 0);
                x ^= c.x;
            } else if (MIX == 1) {
                x ^= __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 48, 0, 0);
            } else if (MIX == 3) {
                const vu4 w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 48, 0, 0);
                x ^= w.w;
            }
            off = ((x + (unsigned)i * 2654435761u + (unsigned)lane * 40503u) % nrec) * 64u;
            acc += v.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int MIX>
static void run(const unsigned* d, unsigned tab_bytes, unsigned* o, int active, const char* name, hipEvent_t a, hipEvent_t b)
{
    const int cus = 256, waves_per_cu = 32, iters = 200;
    const int blocks = cus * waves_per_cu;
    step<MIX><<<blocks, 64>>>(d, tab_bytes, iters, active, o);
    hipEventRecord(a);
    step<MIX><<<blocks, 64>>>(d, tab_bytes, iters, active, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double steps_per_cu = (double)waves_per_cu * iters;
    const double ns = ms * 1e6 / steps_per_cu;
    printf("table %8u B  %-22s active %2d: %.3f ms, %.2f ns per wave-step per CU (%.1f cyc @2.4GHz)\n", tab_bytes, name, active,
           ms, ns, ns * 2.4);
}

int main()
{
    for (unsigned tab_bytes : { 1u << 20, 48u << 20 }) {
        std::vector<unsigned> h(tab_bytes / 4);
        for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 3);
        unsigned *d, *o;
        hipMalloc(&d, tab_bytes);
        hipMalloc(&o, 4);
        hipMemcpy(d, h.data(), tab_bytes, hipMemcpyHostToDevice);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int active : { 64, 16, 4 }) {
            run<0>(d, tab_bytes, o, active, "3 x dwordx4 + dwordx2", a, b);
            run<1>(d, tab_bytes, o, active, "3 x dwordx4 + dword", a, b);
            run<2>(d, tab_bytes, o, active, "3 x dwordx4", a, b);
            run<3>(d, tab_bytes, o, active, "4 x dwordx4", a, b);
            run<4>(d, tab_bytes, o, active, "1 x dwordx4", a, b);
        }
        hipFree(d);
        hipFree(o);
    }
    return 0;
}
