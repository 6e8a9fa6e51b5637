"""Variant edit: screenOutput over 32x16 tiles (36x20 staged texels, 1.41 reads per pixel instead of
1.56), two pixels per thread (x and x + 16). argv[1] = csrc dir."""
import os
import sys

p = os.path.join(sys.argv[1], "pt_kernels.hip")
s = open(p).read()


def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)


sub("PT_D void outputPixel(const OutputArgs& a, const float4* tile, int lx, int ly, int x, int y)",
    "template <int TW>\nPT_D void outputPixel(const OutputArgs& a, const float4* tile, int lx, int ly, int x, int y)")
sub("m25[k] = tile[(ly + 2 + 2 - (k / 5)) * 20 + (lx + 2 + (k % 5) - 2)];",
    "m25[k] = tile[(ly + 2 + 2 - (k / 5)) * TW + (lx + 2 + (k % 5) - 2)];")
old_kernel_start = s.index("__global__ __launch_bounds__(256) void pt_output(OutputArgs a, int tiles_x, int ntiles)")
old_kernel_end = s.index("// ------------------------------------------------------------------------------ child-pair BVH records")
s = s[:old_kernel_start] + """__global__ __launch_bounds__(256) void pt_output(OutputArgs a, int tiles_x, int ntiles)
{
    constexpr int TW = 36, TN = 36 * 20;   // 32x16 tile + the +-2 border
    __shared__ float4 tile[2][TN];
    const int tid = threadIdx.x;
    const int lx = tid & 15, ly = tid >> 4;
    auto origin = [&](int t, int& x0, int& y0) {
        x0 = (t % tiles_x) * 32;
        y0 = ((t / tiles_x) * a.num_parts + a.part) * 16;
    };
    auto load = [&](int x0, int y0, float4& f0, float4& f1, float4& f2) {
        f0 = accAt(a, x0 + tid % TW - 2, y0 + tid / TW - 2);
        f1 = accAt(a, x0 + (tid + 256) % TW - 2, y0 + (tid + 256) / TW - 2);
        if (tid + 512 < TN) f2 = accAt(a, x0 + (tid + 512) % TW - 2, y0 + (tid + 512) / TW - 2);
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
    float4 f0, f1, f2 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    load(x0, y0, f0, f1, f2);
    tile[0][tid] = f0;
    tile[0][tid + 256] = f1;
    if (tid + 512 < TN) tile[0][tid + 512] = f2;
    __syncthreads();
    for (int cur = 0; t < ntiles; cur ^= 1) {
        const int tn = t + nblk;
        int nx0 = 0, ny0 = 0;
        if (tn < ntiles) { origin(tn, nx0, ny0); load(nx0, ny0, f0, f1, f2); }
        const int y = y0 + ly;
        if (x0 + lx < a.width && y < a.height) outputPixel<TW>(a, tile[cur], lx, ly, x0 + lx, y);
        if (x0 + lx + 16 < a.width && y < a.height) outputPixel<TW>(a, tile[cur], lx + 16, ly, x0 + lx + 16, y);
        if (tn < ntiles) {
            tile[cur ^ 1][tid] = f0;
            tile[cur ^ 1][tid + 256] = f1;
            if (tid + 512 < TN) tile[cur ^ 1][tid + 512] = f2;
        }
        __syncthreads();
        t = tn; x0 = nx0; y0 = ny0;
    }
}

""" + s[old_kernel_end:]
sub("    dim3 grid((a->width + 15) / 16, a->part < nb ? (nb - a->part + a->num_parts - 1) / a->num_parts : 0);",
    "    dim3 grid((a->width + 31) / 32, a->part < nb ? (nb - a->part + a->num_parts - 1) / a->num_parts : 0);")
sub("    const int blocks = ntiles / 4 < 4096 ? 4096 : ntiles / 4 > 8192 ? 8192 : ntiles / 4;",
    "    const int blocks = ntiles / 2 < 4096 ? 4096 : ntiles / 2 > 8192 ? 8192 : ntiles / 2;")
open(p, "w").write(s)
