/* include/pt.h — C ABI of libpt.so, the MI355X (gfx950) backend behind the Babylon.js effect API.
 *
 * The reference drives its hot path only through Babylon's effect API (js/babylon.js, vendored
 * 5.0.0-alpha.43). Each entry point below is what a binding of that API needs; the comment on
 * each names the reference call it replaces (file:line in the reference repository). A Node
 * N-API addon (babylon.js-pathtracing-renderer_amd/napi/pt_napi.c) binds these for the
 * unmodified setup scripts; ctypes binds them for tests and bench.py.
 *
 * Conventions: plain pointers and sizes; every call returns PT_OK (0) or a negative pt_status
 * and never throws. Device memory is owned by the context. Host arrays are copied at the call.
 * All work of a context is ordered on one HIP stream (the context's own, or the caller's: pt_set_stream);
 * pt_render is asynchronous and pt_read_pixels / pt_sync synchronise. The megakernel's path tracing of a
 * frame runs on one of the context's internal side streams (two or three, PT_OVERLAP_DEPTH) beside the
 * previous frames' (frame overlap: it never reads the history), gated by events recorded on the
 * context's stream, and the history blend that follows it runs on that one stream, so every observable
 * result is in call order. Not re-entrant (single JS thread, like the reference).
 * Image rows are stored bottom-up (row 0 = gl_FragCoord.y 0.5), as GL render targets are.
 */
#ifndef PT_H
#define PT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_ctx pt_ctx;
typedef struct pt_effect pt_effect;
typedef struct pt_texture pt_texture;

enum pt_status {
    PT_OK = 0,
    PT_ERR_ARG = -1,         /* bad handle, size or name */
    PT_ERR_HIP = -2,         /* HIP runtime error (message in pt_last_error) */
    PT_ERR_SHADER = -3,      /* fragment source not recognised as a supported program */
    PT_ERR_STATE = -4,       /* e.g. render with a required sampler unbound */
    PT_ERR_OOM = -5,
    PT_ERR_DEVICE = -6,      /* no usable gfx950 device */
    PT_ERR_UNSUPPORTED = -7, /* recognised program that this build does not implement yet */
    PT_ERR_DATA = -8         /* scene data outside the reference's limits (e.g. BVH deeper than stackLevels[28]) */
};

/* Programs recognised from the fragment source registered in Effect.ShadersStore. */
enum pt_program {
    PT_PROG_UNKNOWN = 0,
    PT_PROG_SCREEN_COPY = 1,    /* js/PathTracingCommon.js:1-16 */
    PT_PROG_SCREEN_OUTPUT = 2,  /* js/PathTracingCommon.js:19-309 */
    PT_PROG_CORNELL = 3,        /* js/BabylonPathTracing_FragmentShader.js */
    PT_PROG_GLTF = 4,           /* js/GLTFModelPathTracing_FragmentShader.js */
    PT_PROG_HDRI = 5,           /* js/HDRIEnvironmentPathTracing_FragmentShader.js */
    PT_PROG_SKY = 6,            /* js/PhysicalSkyModel_FragmentShader.js */
    PT_PROG_QUADRIC = 7,        /* js/TransformedQuadricGeometry_FragmentShader.js */
    /* BASELINE configs[4]: js/PhysicalSkyModel_FragmentShader.js with the glTF model block of
     * js/GLTFModelPathTracing_FragmentShader.js:201-346 appended to its SceneIntersect (the sky shader
     * text plus `uniform sampler2D tAABBTexture`); the reference has no such page */
    PT_PROG_SKY_MESH = 8
};

/* Babylon sampling-mode constants (BABYLON.Constants.TEXTURE_*_SAMPLINGMODE) */
enum pt_sampling { PT_SAMPLING_NEAREST = 1, PT_SAMPLING_BILINEAR = 2, PT_SAMPLING_TRILINEAR = 3 };

/* ---- context: replaces `new BABYLON.Engine(canvas, true)` (js/GLTF_Model_Path_Tracing.js:189).
 * A context has one or more parts, each one HIP stream on one gfx950 device. With several parts
 * every draw fans out inside pt_render: part k shades the 16-row bands b % N == k, screenOutput
 * pulls the +-2 halo rows from the band neighbours and part 0 gathers the RGBA8 bands into the
 * canvas (device-to-device copies over xGMI, ordered by HIP events). Render targets
 * stay distributed by bands; pt_read_pixels assembles them. Results are bit-identical to one part.
 * pt_ctx_create(device): one part on `device`. */
pt_ctx* pt_ctx_create(int device, int* err);
/* one part per set bit of device_mask (bit d = HIP device d), in increasing device order */
pt_ctx* pt_ctx_create_mask(uint32_t device_mask, int* err);
/* part k on devices[k]; a device may appear more than once (several parts on one GPU: the same
 * split, halo and gather path on a one-GPU host) */
pt_ctx* pt_ctx_create_devices(const int* devices, int n, int* err);
int pt_ctx_parts(const pt_ctx* ctx);
/* 1 when the halo pulls and the canvas gather between the context's distinct devices run as strided 2D
 * copies over peer access (xGMI), 0 when some pair has no peer access (hipDeviceCanAccessPeer false or
 * hipDeviceEnablePeerAccess failing; PT_PEER=0 forces it): they then run band by band through
 * hipMemcpyPeerAsync, same results. One-device contexts report 1. */
int pt_ctx_peer_copies(const pt_ctx* ctx);
void pt_ctx_destroy(pt_ctx* ctx);
const char* pt_last_error(pt_ctx* ctx);
int pt_sync(pt_ctx* ctx);
/* the default framebuffer ("canvas", RGBA8) that pt_render(effect, NULL) draws into;
 * replaces engine.resize()/getRenderWidth() (js/GLTF_Model_Path_Tracing.js:521-537) */
int pt_canvas_resize(pt_ctx* ctx, int width, int height);

/* ---- effects: replaces `new BABYLON.EffectWrapper({engine, fragmentShader, uniformNames,
 * samplerNames, name})` (js/GLTF_Model_Path_Tracing.js:773-811). The program is recognised from
 * the GLSL text; unknown text -> NULL with *err = PT_ERR_SHADER. Uniform/sampler names not in the
 * lists are ignored by the setters, as Babylon ignores undeclared uniforms. */
pt_effect* pt_effect_create(pt_ctx* ctx, const char* fragment_source,
                            const char* const* uniform_names, int n_uniforms,
                            const char* const* sampler_names, int n_samplers, int* err);
/* Same, with the program named directly (hosts that do not carry the reference's GLSL text,
 * e.g. the Python binding replaying a recorded uniform stream on the GPU box). */
pt_effect* pt_effect_create_program(pt_ctx* ctx, int program,
                                    const char* const* uniform_names, int n_uniforms,
                                    const char* const* sampler_names, int n_samplers, int* err);
void pt_effect_destroy(pt_effect* fx);
int pt_effect_program(const pt_effect* fx);

/* ---- uniforms: replaces effect.setFloat / setFloat2 / setFloat3 / setVector3 / setMatrix /
 * setInt / setBool (js/GLTF_Model_Path_Tracing.js:826-847). n = component count (1,2,3,4,16).
 * setBool is setInt(0|1), as in Babylon. Returns PT_OK also for ignored (undeclared) names. */
int pt_set_float(pt_effect* fx, const char* name, const float* v, int n);
int pt_set_int(pt_effect* fx, const char* name, int v);
/* effect.setTexture(sampler, texture) (js/GLTF_Model_Path_Tracing.js:818-825); tex NULL binds
 * nothing (an unloaded Babylon texture) */
int pt_set_texture(pt_effect* fx, const char* sampler, pt_texture* tex);

/* ---- textures -------------------------------------------------------------------------------
 * BABYLON.RawTexture.CreateRGBATexture(data, w, h, scene, mips, invertY, sampling, FLOAT)
 * (js/GLTF_Model_Path_Tracing.js:466-487): RGBA32F, data copied. */
pt_texture* pt_texture_create_rgba32f(pt_ctx* ctx, int width, int height, const float* data,
                                      int sampling, int invert_y, int* err);
/* new BABYLON.Texture(url, scene, noMipmap, invertY, sampling) of 8-bit images, decoded by the
 * host (js/GLTF_Model_Path_Tracing.js:749-758): RGBA8, data copied. */
pt_texture* pt_texture_create_rgba8(pt_ctx* ctx, int width, int height, const uint8_t* data,
                                    int sampling, int invert_y, int* err);
/* new BABYLON.RenderTargetTexture(name, {width,height}, scene, false, false, TEXTURETYPE_FLOAT,
 * false, NEAREST, ...) (js/GLTF_Model_Path_Tracing.js:762-768): RGBA32F, zero-filled. */
pt_texture* pt_render_target_create(pt_ctx* ctx, int width, int height, int* err);
/* MI355X extension: an RGBA32F render target over caller-owned device memory (w*h*16 bytes on
 * this context's device, e.g. a torch tensor that RCCL collectives also use). Not freed by
 * pt_texture_destroy; not resizable. */
pt_texture* pt_render_target_wrap(pt_ctx* ctx, int width, int height, void* device_ptr, int* err);
/* renderTarget.resize({width,height}) (js/GLTF_Model_Path_Tracing.js:529-530) */
int pt_render_target_resize(pt_texture* tex, int width, int height);
/* renderTarget.getSize() (js/GLTF_Model_Path_Tracing.js:826) */
int pt_texture_size(const pt_texture* tex, int* width, int* height);
void pt_texture_destroy(pt_texture* tex);

/* ---- draw: replaces eRenderer.render(effectWrapper, renderTargetOrNull)
 * (js/GLTF_Model_Path_Tracing.js:1230-1235). target NULL = the canvas. */
int pt_render(pt_effect* fx, pt_texture* target);
/* (A screenCopy draw may be deferred until the next draw: when that draw is the screenOutput of
 * the same source it writes the copy in the same pass. Every pt_* call that could observe the copy
 * target - another draw, read/write pixels, resize, destroy, pt_sync, pt_set_stream - runs it
 * first; code reading a wrapped render target's memory directly calls pt_sync before.) */

/* readPixels of a render target (RGBA32F, 16 B/texel) or of the canvas (tex NULL, RGBA8),
 * rows bottom-up; synchronises. */
int pt_read_pixels(pt_ctx* ctx, const pt_texture* tex, void* dst, size_t bytes);
/* Upload rows of a render target (RGBA32F), used to seed the history buffer in tests and to
 * land gathered bands on the root in multi-GPU runs. */
int pt_write_pixels(pt_ctx* ctx, pt_texture* tex, const void* src, size_t bytes);

/* ---- MI355X extensions (no reference counterpart) -------------------------------------------
 * Row-band sharding for one-part contexts driven by one process per GPU (bench.py, torch.distributed;
 * a multi-part context shards itself and refuses these four: PT_ERR_ARG; pt_canvas_wrap then wraps
 * the gathered canvas): this context's path-tracing and screenCopy passes
 * shade only the 16-row bands b with b % num_parts == part (bands are whole 2x2 quads, so
 * derivatives are unchanged). num_parts = 1 restores full frames. */
int pt_set_row_partition(pt_ctx* ctx, int num_parts, int part);
/* screenOutput under the row partition too (enable = 1): only the owned bands of the output are
 * written. Its 5x5 filter reads the accumulation 2 rows beyond each band, so those halo rows must
 * hold the neighbouring ranks' values (babylon_pt.exchange_halos) before the draw. Default 0:
 * screenOutput shades the whole frame. */
int pt_set_output_partition(pt_ctx* ctx, int enable);
/* The canvas over caller-owned device memory: width*height RGBA8 texels, rows bottom-up (e.g. a
 * torch tensor that RCCL gathers from). Not freed by the context; pt_canvas_resize replaces it
 * with context-owned memory again. Re-wrapping another caller buffer is a host-side switch (no
 * synchronisation), so a caller can alternate between two canvases frame by frame. */
int pt_canvas_wrap(pt_ctx* ctx, int width, int height, void* device_ptr);
/* Path-tracing backend of this context: PT_BACKEND_MEGAKERNEL (default: one kernel, one lane per
 * path), PT_BACKEND_WAVEFRONT (per-segment kernels over compacted path queues) or
 * PT_BACKEND_PERSISTENT (waves regenerate finished lanes with new pixels; G-buffer + finish pass).
 * Results are bit-identical; the choice only changes speed. */
enum pt_backend { PT_BACKEND_MEGAKERNEL = 0, PT_BACKEND_WAVEFRONT = 1, PT_BACKEND_PERSISTENT = 2 };
int pt_set_backend(pt_ctx* ctx, int backend);
/* BVH walk of the glTF program. PT_BVH_PAIRS (default) re-packs tAABBTexture once per upload into
 * 64-byte child-pair records (both children's boxes in one line, pops without a fetch) and walks
 * those with the reference's short stack (LDS levels, deeper ones in a global slab); PT_BVH_TRAIL
 * walks the same records stacklessly: a restart trail of one bit per tree level plus a per-lane LDS
 * ring of the deepest pending entries, re-descending from a jump table of the top levels when the
 * ring runs dry (no stack memory beyond LDS; trees deeper than 28 levels - the reference's
 * stackLevels[28] - or whose nodes have more than one parent, keep PT_BVH_PAIRS). A texture whose
 * links are not exact in-range integers keeps PT_BVH_REFERENCE, the walk over the reference's own
 * texel pairs. Same nodes, same order, same results every way
 * (js/GLTFModelPathTracing_FragmentShader.js:211-298). Other values: PT_ERR_ARG.
 * pt_bvh_layout_used reports what the last glTF draw of the context walked (-1: none yet).
 * API change (round 4): the two-level layout PT_BVH_QUADS (3) was removed - it was slower on every
 * workload; pt_set_bvh_layout(ctx, 3) now returns PT_ERR_ARG and the Python
 * set_bvh_layout("quads") raises KeyError. */
enum pt_bvh_layout { PT_BVH_REFERENCE = 0, PT_BVH_PAIRS = 1, PT_BVH_TRAIL = 2 };
int pt_set_bvh_layout(pt_ctx* ctx, int layout);
int pt_bvh_layout_used(pt_ctx* ctx);
/* Enqueue this context's work on a caller-owned HIP stream (e.g. torch.cuda.current_stream(), so
 * that draws and RCCL collectives are ordered without host syncs); NULL restores the context's own
 * stream. The caller keeps the stream alive while the context uses it. */
int pt_set_stream(pt_ctx* ctx, void* hip_stream);
/* Device pointer of a render target's RGBA32F storage (for RCCL collectives from the host). */
void* pt_texture_device_ptr(pt_texture* tex);
/* Device time of the last pt_render of each program kind, in ms (HIP events on the context
 * stream; requires pt_sync first). Draws are bracketed by events only once this has been called
 * (or with PT_DRAW_EVENTS=1): an event record costs ~5 us of stream time between kernels, so the
 * first call turns them on and returns PT_ERR_ARG; the draws after it are reported. */
int pt_last_render_ms(pt_ctx* ctx, int program, float* ms);
/* Timing window: between pt_timing_begin and pt_timing_end every draw is bracketed by its own
 * HIP event pair (no host sync inside the window); pt_timing_end closes the window, synchronises
 * and returns the summed device time and launch count of one program kind (further pt_timing_end
 * calls report other kinds from the same window). PT_TIMING_EVERY=k (read at pt_timing_begin)
 * brackets only every k-th draw of each program kind, so the events barely disturb the timed
 * stream; the launch count returned is then the bracketed draws'. */
int pt_timing_begin(pt_ctx* ctx);
int pt_timing_end(pt_ctx* ctx, int program, double* total_ms, int* launches);
/* Frame latency from the same timing window (closes it and synchronises, like pt_timing_end): for each
 * bracketed path-tracing draw of `program`, the device time from its begin event (recorded on the stream
 * its path tracing runs on, after the waits that order it: the moment its frame's path tracing may start)
 * to the end event of the next bracketed screenOutput draw (its canvas complete, main stream). Writes up
 * to `cap` values in window order and their count; with several parts, the slowest part's per frame. The
 * reference displays every frame it draws (js/GLTF_Model_Path_Tracing.js:1228-1237): with frames in
 * flight this is the draw-to-display delay the overlap adds. */
int pt_timing_latency(pt_ctx* ctx, int program, float* ms, int cap, int* n);
/* Algorithmic-byte counters: when enabled, path-tracing passes also accumulate
 * {paths, segments, node_fetches, leaf_tests, hit_lookups, rgba8_taps, stack_overflow, hdr_taps}. */
#define PT_NUM_COUNTERS 8
int pt_set_counting(pt_ctx* ctx, int enable);
int pt_read_counters(pt_ctx* ctx, uint64_t out[PT_NUM_COUNTERS]);
int pt_reset_counters(pt_ctx* ctx);
/* Wavefront queue statistics of the last path-tracing draw (synchronises): out[b] = paths entering
 * bounce b (b = 0..6), out[8 + b] = rays handed to the BVH walk at bounce b (b = 0..5); megakernel:
 * out[7] = the slowest tiles the next draw of the same target and program shades as 16-lane waves;
 * out[14] = late-bounce compaction of the last megakernel draw (PT_CONT: 0 off, 1 on, 2 auto = default):
 * bits 0-7: 0 off, 1 auto decided off, 2 auto decided on, 3 forced on, 4 auto trial running, 5 / 6 auto
 * before the trial, default on / off; bits 8-15: the frames that draw kept in flight (PT_OVERLAP_DEPTH, or 2
 * when the auto trial found two faster without compaction); bits 16-31: the path-tracing draws that
 * launched the late-bounce continuation (pt_cont) since the context was created, mod 2^16;
 * out[15] = the auto trial's time with
 * compaction per time without (at the faster depth), x 1000 (0 before the decision). */
int pt_queue_stats(pt_ctx* ctx, uint32_t out[16]);
/* Device self-test of the pinned GLSL built-ins (ops as the oracle's pto_math_probe). */
int pt_math_probe(pt_ctx* ctx, int op, const float* x, const float* y, float* out, int n);
/* Exhaustive device self-test of a fast built-in sequence against the IEEE operation it replaces,
 * over all 2^32 binary32 inputs: op 0 = the reciprocal (grcp vs 1.0f/x), op 1 = the square root
 * (gsqrt vs sqrtf). Writes the mismatch count. */
int pt_math_exhaustive(pt_ctx* ctx, int op, uint64_t* mismatches);
/* BVH_Build_Iterative(workList, aabb_array) (js/BVH_Fast_Builder.js:320-406) as native host code:
 * aabb_in = the per-triangle AABBs the setup script fills (9 floats: min.xyz, max.xyz,
 * centroid.xyz; js/GLTF_Model_Path_Tracing.js:421-454), work = the triangle ids to build over
 * (n of them). Writes 8 floats per node, depth-first, exactly the reference's tAABBTexture layout
 * and bits, and returns the node count (2n-1), or a negative pt_status (max_nodes too small). No
 * context or device needed. */
int pt_bvh_build(const float* aabb_in, const uint32_t* work, int n, float* nodes_out, int max_nodes);
/* The same build on a gfx950 device (csrc/pt_bvh_gpu.hip): level by level, every node of a depth
 * split together, the same tree and bits as pt_bvh_build (js/BVH_Fast_Builder.js:43-406; the page
 * runs it at js/GLTF_Model_Path_Tracing.js:456-462). aabb_in holds 9 floats for every triangle id
 * up to the largest in work; n <= 2^24. Synchronous. Returns the node count (2n-1) or a negative
 * pt_status; *ms_out (may be NULL) = device time of the build, uploads and read-back excluded. */
int pt_bvh_build_gpu(int device, const float* aabb_in, const uint32_t* work, int n, float* nodes_out,
                     int max_nodes, float* ms_out);
/* JPEG decode for the hosts' texture loading: replaces the browser's decode of the glTF models'
 * map images, which the glTF loader hands to `new BABYLON.Texture` (js/GLTF_Model_Path_Tracing.js:
 * 252-274) and the page binds with effect.setTexture (:822-825). libjpeg-turbo's default
 * decompression reproduced bit for bit (csrc/pt_jpeg.cpp: baseline and progressive, accurate
 * integer IDCT, fancy upsampling, RGB output); RGBA8 rows top first, alpha 255. pt_jpeg_size reads
 * the frame header; pt_jpeg_decode_rgba8 needs capacity >= 4 * width * height. Host code: no
 * context or device. PT_ERR_UNSUPPORTED for arithmetic-coded, 12-bit, CMYK or stored-RGB files. */
int pt_jpeg_size(const uint8_t* data, size_t size, int* width, int* height);
int pt_jpeg_decode_rgba8(const uint8_t* data, size_t size, uint8_t* rgba, size_t capacity);
/* Library identity: "libpt <version> gfx950" */
const char* pt_version(void);

#ifdef __cplusplus
}
#endif
#endif
