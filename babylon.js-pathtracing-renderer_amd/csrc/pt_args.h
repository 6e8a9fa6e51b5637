// pt_args.h — kernel-argument layouts shared by the C-ABI host code (pt_capi.cpp) and the gfx950
// kernels (pt_kernels.hip). Passed by value as kernarg segments (scalar-loaded, wave-uniform).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_glsl.h"

namespace pt {

constexpr int kBlock = 256;          // 4 waves; a block shades a 16x16 pixel tile
constexpr int kTile = 16;            // tile edge == row-band height used for sharding
constexpr int kWaveLogSlots = 13;   // experiment builds (PT_SECPROF): u64 per workgroup in TraceArgs::wave_log
// split tiles (pt_trace, longest-first): each 8x8 quadrant of a split 16x16 tile is shaded by this
// many waves of 64 / kSplitParts lanes (4x4-pixel waves of 16 lanes; one 2x2 quad per wave measured
// slower)
constexpr unsigned kSplitParts = 4;
constexpr int kStackLevels = 28;     // stackLevels[28], js/GLTFModelPathTracing_FragmentShader.js:95
// BVH stack levels kept in LDS per lane (deeper levels go to a global slab): 7 for the 4-wave variants;
// the child-pair walk of the texture-free mesh programs runs at 8 waves/SIMD (pt_device.h kMinWaves),
// where 6 LDS levels and the G-buffer fill the 160 KB of a CU (pt_trace.h MegaStack::push)
constexpr int kStackLds = 7;
constexpr int kStackLdsPairs = 6;
constexpr int kStackLdsMin = kStackLdsPairs < kStackLds ? kStackLdsPairs : kStackLds;   // sizes the slab

// child-pair record codes: a node's rank code from the build's rank pass (rank >= 0 of an inner
// node, -1 - rank of a leaf) -> the 32-bit code the walk carries: the record's byte offset in the
// one record array (inner records first, the leaf records from byte leafBase on), with kLeafBit set
// for a leaf
constexpr uint32_t kLeafBit = 0x80000000u;
__host__ __device__ inline uint32_t pairCode(float rankCode, uint32_t leafBase)
{
    return rankCode >= 0.0f ? (uint32_t)rankCode * 64u : kLeafBit | (leafBase + (uint32_t)(-1.0f - rankCode) * 48u);
}

// restart-trail walk (pt_device.h bvhWalkTrail): one trail bit per depth 1..31 of a register; trees of
// depth <= 28 (stackLevels[28] then never overflows); a jump table of the inner records at depths
// 0..kTopLevels, by path, after the leaf records
constexpr int kTrailMaxDepth = 28;
constexpr int kTopLevels = 11;
constexpr unsigned kTopEntries = (2u << kTopLevels) - 1u;   // 4095 record copies (64 B, 256 KB), heap order

// the BVH walk of a mesh draw (TraceArgs::bvh_walk; the program variant's thousands digit, pt_device.h)
enum { WALK_REF = 0, WALK_PAIRS = 1, WALK_TRAIL = 2 };

enum Counter { C_PATHS, C_SEGMENTS, C_NODE, C_LEAF, C_HIT, C_RGBA8, C_OVERFLOW, C_HDR, C_NUM };
enum ErrBits { E_STACK = 1u };

// material enum of js/PathTracingCommon.js:330-350 (the subset the implemented scenes use)
enum Mat { LIGHT = 0, DIFFUSE = 1, TRANSPARENT = 2, METAL = 3, CLEARCOAT_DIFFUSE = 4, PBR_MATERIAL = 10 };

struct QuadArg {            // struct Quad of the scene shaders (js/GLTFModelPathTracing_FragmentShader.js:39)
    ptg::f3 normal, v0, v1, v2, v3, color;
    int type;
};

// the two triangles of quad i (QuadIntersect = TriangleIntersect(v0,v1,v2) min (v0,v2,v3)) with
// the edge vectors v1-v0, v2-v0 evaluated once on the host (same IEEE subtraction as the GLSL)
struct TriArg {
    ptg::f3 v0, e1, e2;
};

struct SphereArg {          // UnitSphere + its inverse transform uniform
    ptg::m4 inv;
    ptg::f3 color;
    int type;
};

struct Tex8 {               // RGBA8 sampler: texels row-major from row 0 (invertY applied at upload)
    const uchar4* p;
    int w, h;
};

struct TexF {               // RGBA32F sampler (tHDRTexture), same row convention
    const float4* p;
    int w, h;
};

// Uniform-only terms of Get_Sky_Color (js/PathTracingCommon.js:416-475), evaluated once per draw
// on the host with the pinned sequences
struct SkyArgs {
    ptg::f3 sun;            // uSunDirection
    ptg::f3 rayleigh, mie;  // rayleighAtX, mieAtX
    ptg::f3 rm;             // rayleighAtX + mieAtX
    float sunE, sunE19000;  // SunIntensity(dot(UP, sun)), sunE * 19000
    float fade;             // clamp(pow(1 - cosSunUpAngle, 5), 0, 1)
    float retExp;           // 1 / (1.2 + 1.2 * sunfade)
};

// Per-draw kernel arguments. Wave-uniform: read with scalar loads from the kernarg segment; the
// per-object loops index them dynamically so they are re-read from the scalar cache instead of
// being hoisted into (vector) registers.
struct TraceArgs {
    int width, height;      // render target
    int num_parts, part;    // row-band sharding (pt_set_row_partition)
    // common uniforms (js/PathTracingCommon.js:357-368)
    float res[2], rnd[2];
    float ulen, vlen, frame, eps, aperture, focus;
    int moving;
    ptg::m4 cam, model;
    // SetupScene() hoisted to the host: identical IEEE ops, evaluated once per frame
    SphereArg sph[2];
    TriArg qtri[12];
    ptg::f3 qnormal[6], qcolor[6];
    int qtype[6];
    int nquads;             // N_QUADS: 6 (Cornell, glTF, quadric), 4 (sky, HDRI: no ceiling, no quad light)
    // transformed-quadric program (js/TransformedQuadricGeometry_FragmentShader.js:9-24): the twelve
    // unit shapes' inverse matrices in SceneIntersect order, uShapeK, uAllShapesMatType
    ptg::m4 shape_inv[12];
    float shape_k;
    int shape_mat;
    SkyArgs sky;            // sky.sun is uSunDirection for the HDRI program too
    // HDRI environment (js/HDRIEnvironmentPathTracing_FragmentShader.js:15-22)
    TexF hdr;
    float hdr_exposure;     // uHDRExposure
    float sun_weight;       // uSunPower * uSunPower * 0.0000001
    QuadArg light;          // quads[5], sampled by sampleAxisAlignedQuadLight
    float light_r2;         // distance(v0,v1)*distance(v0,v3) of quads[5]
    // glTF material switches (js/GLTFModelPathTracing_FragmentShader.js:21-25)
    int model_mat, uses_albedo, uses_bump, uses_metal, uses_emissive;
    // samplers
    const float4* prev;     // the wavefront / persistent schedules' finish pass: history in,
    float4* out;            // accumulation out
    // the megakernel: per pixel (py * width + px) CalculateRadiance()'s result and the pre-history
    // alpha flag (0, 1.01 or -1: the G-buffer sharpness and the 2x2 edge test); pt_blend folds in the
    // history (js/PathTracingCommon.js:1326-1357), so the kernel never reads it and consecutive frames'
    // path tracing may overlap
    float4* rad;
    // late-bounce compaction (megakernel mesh draws; pt_cont): after a bounce >= cont_bounce,
    // a wave with at most cont_lanes live paths stores them as 64-B records and ends; pt_cont runs them
    // packed into full waves (cont_rec NULL: off)
    float4* cont_rec;
    unsigned* cont_aux;     // per record: the pixel (py * width + px) | the 2x2 edge flag << 31
    unsigned* cont_count;   // [0] records stored by this draw, [1] pt_cont's queue head (both zeroed by the draw's pt_blend)
    unsigned cont_bounce, cont_lanes, cont_refill;
    // (PT_CONT_SORT) pt_cont takes the records ordered by a ray key (pt_trace.h contRank): per record its key and
    // its rank among the key's records (pt_trace), the keys' totals (NULL: no sort), the order (pt_cont_scatter)
    unsigned short* cont_key;
    unsigned* cont_rank;
    unsigned* cont_bins;
    const unsigned* cont_perm;
    float cont_cell[3];          // the key's origin cells: (o - model box min) * cont_cell, 0..2^cont_grid_bits - 1 per axis
    unsigned cont_grid_bits, cont_key_mode;
    Tex8 bluenoise;
    const float4* aabb;
    long long aabb_texels;
    const float4* tri;
    long long tri_texels;
    const float4* bvh_pairs;   // child-pair records of tAABBTexture (PROG_PAIRS variants only): inner, then leaf
    uint32_t bvh_root_code;    // pairCode of node 0
    float bvh_root_box[6];     // node 0's box (texels 0.yzw, 1.yzw as uploaded; PROG_PAIRS only): the root test of
                               // every segment reads SGPRs instead of waiting on a load
    uint32_t bvh_pairs_bytes;  // size of the record array (its buffer descriptor)
    uint32_t bvh_top_base;     // PROG_TRAIL: byte offset of the restart jump table (inner-record copies) in it
    int bvh_walk;              // WALK_REF / _PAIRS / _TRAIL (pt_device.h): the variant the draw takes
    float2* spill;             // megakernel BVH stack levels >= kStackLds: [level][grid lane]
    unsigned spill_stride;
    // longest-first dispatch (megakernel): order[slot] = the 16x16 tile dealt to tile slot `slot`
    // (NULL: row-major); each wave records its duration in cost[tile * 4 + quadrant]
    const unsigned* order;
    unsigned* cost;
    unsigned prio_tiles;   // the first prio_tiles tiles of `order` (the slowest last frame) run at s_setprio 3
    unsigned order_zig;    // 1: after the split tiles, runs of 8 slots (a tile per XCD) take `order` from both
                           // ends in turn (8 slowest, 8 cheapest, ...): the slowest still start first, cheap
                           // tiles mix in
    // *split (written by the previous pt_order_build; a multiple of 8): the first *split tiles of
    // `order` are shaded by 16 waves of 16 lanes (4x4 pixels) instead of 4 waves of 64 (pt_trace);
    // the grid carries padding rows for up to split_cap of them
    const unsigned* split;
    unsigned ntiles;       // 16x16 tiles of the draw
    Tex8 albedo, bump, metal, emissive;
    // diagnostics
    unsigned long long* counters;   // C_NUM entries, only with counting builds
    unsigned* err;                  // ErrBits
#ifdef PT_SECPROF
    unsigned long long* wave_log;   // experiment builds: per workgroup (start, end) wall clock, walk iterations, longest lane's steps, 8 section cycle sums
    unsigned long long* walk_stat;  // experiment builds: per bounce 0..7, the child-pair walk's load coherence (WalkStat, pt_device.h)
#endif
};

// wavefront buffers (pt_wavefront.hip). Path queues are split into kShards shards of `shard_cap`
// slots: shard s holds the paths of tiles t with t % kShards == s, and is produced and consumed by
// blocks b with b % kShards == s, so a path never changes shard and each queue append is one
// atomic per block-iteration on that shard's counter (no single hot word). Path state travels with
// the queue as 4 x 16-byte SoA records, double-buffered between bounces; per-pixel outputs are
// indexed py * wq + px.
constexpr int kShards = 16;
constexpr unsigned kHole = 0xFFFFFFFFu;   // queue-0 slot of a tile lane outside the frame

struct WfBufs {
    float4* qA[2];          // ro.xyz, pixel index (bits; kHole = empty slot)
    float4* qB[2];          // rd.xyz, blueNoise counter
    float4* qC[2];          // mask.xyz, metallicRoughness.g
    float4* qD[2];          // seed.xy (bits), flags (bits), blue-noise bytes (bits)
    float4* hit0;           // per slot of the current bounce: t, object id (bits), u, v
    float4* hit1;           // hitNormal.xyz
    unsigned* bvhq;         // per shard: slots whose ray enters the model's root box this bounce
    float4* gb0;            // per pixel: objectNormal.xyz, objectID
    float4* gb1;            // per pixel: objectColor.xyz, pixelSharpness
    float4* rad;
    // late-bounce compaction (megakernel mesh draws; pt_cont): after a bounce >= cont_bounce,
    // a wave with at most cont_lanes live paths stores them as 64-B records and ends; pt_cont runs them
    // packed into full waves (cont_rec NULL: off)
    float4* cont_rec;
    unsigned* cont_aux;     // per record: the pixel (py * width + px) | the 2x2 edge flag << 31
    unsigned* cont_count;   // [0] records stored by this draw, [1] pt_cont's queue head (both zeroed by the draw's pt_blend)
    unsigned cont_bounce, cont_lanes, cont_refill;            // per pixel: CalculateRadiance() result
    float2* spill;          // BVH stack levels >= kStackLds: [level][persistent lane]
    unsigned* cnt;          // [b * kShards + s]: live paths of shard s entering bounce b (b = 0..6)
    unsigned* bcnt;         // [b * kShards + s]: BVH queue of shard s at bounce b
    unsigned shard_cap;     // slots per shard
    int wq, hq;             // quad-rounded frame size
};

constexpr unsigned kOrderHeld = 128;   // pt_order_build: tiles per thread kept in registers (a byte each)
struct OutputArgs {
    int width, height;      // output (canvas or render target) size
    int num_parts, part;    // with an output partition: only 16-row bands b % num_parts == part
    int acc_w, acc_h;       // accumulation texture size (texelFetch bounds)
    float one_over_n, exposure;
    const float4* acc;
    uchar4* canvas;         // RGBA8 target (NULL when writing float)
    float4* out_f;          // RGBA32F target (NULL when writing the canvas)
    float4* copy_dst;       // a deferred screenCopy of `acc` fused into this pass (NULL: none)
    // the longest-first order build of the last megakernel draw (pt_order_build) fused into this
    // pass as one extra block that runs beside the output tiles (NULL ob_cost: none)
    // (fused only while each of its 256 threads holds its tiles in registers: ntiles <= kOrderHeld * 256)
    const unsigned* ob_cost;
    unsigned* ob_order;
    unsigned* ob_split;
    unsigned ob_ntiles, ob_cap, ob_dominance;
    int ob_near;
};

// pt_blend: the progressive accumulation of a megakernel draw (js/PathTracingCommon.js:1326-1357) over
// the owned 16-row bands: out = history (x 0.5 when the camera moved, 0 at frame 1) + radiance, alpha
// from the radiance's pre-history flag and the history's
struct BlendArgs {
    int width, height;
    int num_parts, part;
    float frame;
    int moving;
    const float4* rad;
    const float4* prev;
    float4* out;
    unsigned* cont_count;   // late-bounce compaction: the draw's record counter, zeroed here (NULL: none)
    unsigned* cont_bins;    // (PT_CONT_SORT) the record sort's kSortBins totals, zeroed here (NULL: none)
};

// (PT_CONT_SORT) pt_cont's records ordered by a ray key (pt_kernels.hip pt_cont_hist / pt_cont_scatter)
constexpr int kSortBins = 8192;   // at most: light flag x 8 octants x 8^3 cells
struct SortArgs {
    const unsigned* count;        // [0] records stored by the draw
    const unsigned short* key;    // per record (pt_trace)
    const unsigned* rank;         // per record: its place among its key's records (pt_trace)
    const unsigned* bins;         // the keys' totals
    unsigned* perm;
    unsigned chunk;               // pt_cont_scatter: records per workgroup
    unsigned nbins;               // keys in use (a multiple of 64, <= kSortBins)
};

struct CopyArgs {
    int width, height;
    int num_parts, part;
    const float4* src;
    float4* dst;
};

} // namespace pt
