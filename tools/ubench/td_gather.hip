// Microbenchmark: cost of a scattered buffer_load_dwordx4 in the vector memory pipeline (TA/TD/L1)
// as a function of active lanes per wave-instruction and distinct 64-B lines per instruction.
// Every wave loops over dependent loads (the loaded value feeds the next address, like a BVH walk)
// from an L1/L2-resident table; many waves per CU give the throughput regime.
// build: hipcc --offload-arch=gfx950 -O3 -o td_gather td_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int vu4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void gather(const unsigned* tab, unsigned tab_bytes, int iters, int active, int lines,
                                             int dwords, unsigned* out)
{
    const int lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)tab_bytes, 0x00020000);
    unsigned off = ((blockIdx.x * 977u + (unsigned)(lane % lines) * 131u) % (tab_bytes / 64u)) * 64u;
    unsigned acc = 0;
    if (lane < active) {
        for (int i = 0; i < iters; i++) {
            vu4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            if (dwords > 4) {
                vu4 w = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 16, 0, 0);
                vu4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 32, 0, 0);
                vu4 y = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 48, 0, 0);
                v = v ^ w ^ x ^ y;
            }
            // next line: a function of the data (dependent chain), same line for lanes sharing `lane % lines`
            off = ((v.x + (unsigned)i * 2654435761u + (unsigned)(lane % lines) * 40503u) % (tab_bytes / 64u)) * 64u;
            acc += v.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv)
{
    const unsigned tab_bytes = argc > 1 ? (unsigned)atoi(argv[1]) : (1u << 20);
    std::vector<unsigned> h(tab_bytes / 4);
    for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 3);
    unsigned *d, *o;
    hipMalloc(&d, tab_bytes); hipMalloc(&o, 4);
    hipMemcpy(d, h.data(), tab_bytes, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    int cus = 256;
    const int iters = 400;
    printf("table %u B\n", tab_bytes);
    for (int dwords : {4, 16})
    for (int waves_per_cu : {4, 24})
    for (int active : {64, 16, 4, 1})
    for (int lines : {64, 16, 4, 1}) {
        if (lines > active) continue;
        int blocks = cus * waves_per_cu;
        gather<<<blocks, 64>>>(d, tab_bytes, iters, active, lines, dwords, o);
        hipEventRecord(a);
        gather<<<blocks, 64>>>(d, tab_bytes, iters, active, lines, dwords, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double instr_per_cu = (double)waves_per_cu * iters * (dwords / 4);
        double ns_per_instr = ms * 1e6 / instr_per_cu;
        printf("dwords %2d waves/CU %2d active %2d lines %2d: %.3f ms, %.2f ns per wave-load per CU (%.1f cyc @2.1GHz)\n",
               dwords, waves_per_cu, active, lines, ms, ns_per_instr, ns_per_instr * 2.1);
    }
    return 0;
}
