// pt_output.h — screenOutput's per-pixel program (js/PathTracingCommon.js:19-309), shared by the
// pt_output kernel (pt_kernels.hip) and the riding workgroups of pt_trace (pt_trace.h), which run the
// previous frame's screenOutput in the launch's tail.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_args.h"
#include "pt_glsl.h"

namespace pt {
using namespace ptg;

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

// screenOutput of pixel (x, y) from its tile's neighbourhood staged in LDS, W texels wide (a 16x16
// tile's 20x20 in pt_output, an 8x8 quadrant's 12x12 in pt_trace's riding workgroups; lx, ly: the
// pixel's place in the tile)
template <int W>
PT_D void outputPixel(const OutputArgs& a, const float4* tile, int lx, int ly, int x, int y)
{
    float4 m25[25];
#pragma unroll
    for (int k = 0; k < 25; k++) m25[k] = tile[(ly + 2 + 2 - (k / 5)) * W + (lx + 2 + (k % 5) - 2)];
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

} // namespace pt
