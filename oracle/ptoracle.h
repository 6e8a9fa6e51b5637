/* oracle/ptoracle.h — TEST INFRASTRUCTURE: the CPU restatement of the reference's per-pixel
 * path-tracing fragment program (js/PathTracingCommon.js pathtracing_default_main + the scene
 * shaders' SetupScene / SceneIntersect / CalculateRadiance) and of the screenOutput pass.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product (libpt.so) never links or calls it.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PTO_SCENE_SKYMESH: BASELINE configs[4], the physical-sky scene (js/PhysicalSkyModel_FragmentShader.js)
 * with the glTF model block of js/GLTFModelPathTracing_FragmentShader.js:201-346 appended to its
 * SceneIntersect (hitObjectID = objectCount = 6); the reference has no such page. */
enum { PTO_SCENE_CORNELL = 0, PTO_SCENE_GLTF = 1, PTO_SCENE_SKY = 2, PTO_SCENE_HDRI = 3, PTO_SCENE_QUADRIC = 4,
       PTO_SCENE_SKYMESH = 5 };

/* One frame's uniforms, by the names the setup scripts push (js/GLTF_Model_Path_Tracing.js:813-848,
 * js/Babylon_Path_Tracing.js:339-363). Matrices are Babylon Matrix.m (GLSL column-major). */
typedef struct pto_frame {
    int32_t scene;
    int32_t width, height;              /* framebuffer size (render target) */
    float uResolution[2];
    float uRandomVec2[2];
    float uULen, uVLen, uTime;
    float uFrameCounter, uSampleCounter;
    float uEPS_intersect, uApertureSize, uFocusDistance;
    int32_t uCameraIsMoving;
    float uCameraMatrix[16];
    float uLeftSphereInvMatrix[16];
    float uRightSphereInvMatrix[16];
    float uGLTF_Model_InvMatrix[16];
    float uQuadLightPlaneSelectionNumber, uQuadLightRadius;
    int32_t uRightSphereMatType;         /* cornell */
    int32_t uModelMaterialType;          /* gltf */
    int32_t uModelUsesAlbedoTexture, uModelUsesBumpTexture, uModelUsesMetallicTexture, uModelUsesEmissiveTexture;
    /* samplers */
    const uint8_t* blueNoise;            /* 256x256 RGBA8, texel (x,y) at 4*(y*256+x) */
    const float* aabb;                   /* tAABBTexture texels (RGBA32F), linear texel index */
    int64_t aabbTexels;
    const float* tri;                    /* tTriangleTexture texels (RGBA32F) */
    int64_t triTexels;
    const uint8_t* albedo; int32_t albedoW, albedoH;     /* RGBA8, LOD0 bilinear, REPEAT */
    const uint8_t* bump; int32_t bumpW, bumpH;
    const uint8_t* metallic; int32_t metallicW, metallicH;
    const uint8_t* emissive; int32_t emissiveW, emissiveH;
    float uSunDirection[3];              /* sky, hdri */
    float uHDRExposure, uSunPower;       /* hdri */
    const float* hdr; int32_t hdrW, hdrH; /* tHDRTexture: RGBA32F, GL row order (invertY applied), bilinear, REPEAT */
    /* quadric: uSphere/Cylinder/Cone/Paraboloid/Hyperboloid/Capsule/FlattenedRing/Box/
     * PyramidFrustum/Disk/Rectangle/TorusInvMatrix, in SceneIntersect order */
    float uShapeInvMatrix[12][16];
    float uShapeK;
    int32_t uAllShapesMatType;
} pto_frame;

typedef struct pto_counters {
    uint64_t paths;          /* pixels shaded (incl. quad helpers outside the target) */
    uint64_t segments;       /* SceneIntersect calls */
    uint64_t node_fetches;   /* GetBoxNodeData calls: 2 RGBA32F texels = 32 B each */
    uint64_t leaf_tests;     /* leaf triangle fetches: 3 texels = 48 B each */
    uint64_t hit_lookups;    /* triangle attribute lookups: 8 texels = 128 B each */
    uint64_t rgba8_taps;     /* blue noise + PBR texel taps, 4 B each */
    uint64_t stack_overflow; /* pushes beyond stackLevels[28] (undefined in the reference) */
    uint64_t hdr_taps;       /* tHDRTexture texel taps (RGBA32F), 16 B each */
} pto_counters;

/* Render rows [row0,row1) of one pathTracing pass: prev -> out (RGBA32F, row 0 = bottom, GL
 * order). Rows are expanded to whole 2x2 quads internally (derivatives). Returns 0 on success. */
int pto_path_trace(const pto_frame* f, const float* prev, float* out, int row0, int row1,
                   int nthreads, pto_counters* counters);

/* Optional G-buffer dump of the same pass (bounce-0 objectNormal/objectColor/objectID,
 * pixelSharpness and radiance), 11 floats per pixel, rows [row0,row1). */
int pto_gbuffer(const pto_frame* f, float* gbuf, int row0, int row1, int nthreads);

/* Get_Sky_Color (js/PathTracingCommon.js:416-475) for n directions (xyz triples) -> rgb triples. */
int pto_sky_color(const float sun[3], const float* dirs, float* out, int n);

/* One transformed-quadric intersector (shape = SceneIntersect order 0..11) on n object-space rays:
 * t (INFINITY = 1e6 on a miss) and the unnormalised object-space normal. */
int pto_quadric_probe(int shape, float k, const float* ro, const float* rd, float* t, float* nrm, int n);

/* screenOutput pass (js/PathTracingCommon.js:19-309): RGBA32F accumulation -> RGBA8 canvas. */
int pto_screen_output(int width, int height, const float* acc, float uOneOverSampleCounter,
                      float uToneMappingExposure, uint8_t* out, int nthreads);
/* The same pass into an RGBA32F target: the tone-mapped floats before the canvas's unorm8. */
int pto_screen_output_f32(int width, int height, const float* acc, float uOneOverSampleCounter,
                          float uToneMappingExposure, float* out);

/* Pinned-math probes (KATs shared with the HIP self-test): op 0 exp2, 1 log2, 2 sin, 3 cos,
 * 4 atan, 5 atan2(x, y2), 6 acos, 7 pow(x, y2), 8 exp, 9 log, 10 sqrt, 11 rng stream. */
int pto_math_probe(int op, const float* x, const float* y2, float* out, int n);

#ifdef __cplusplus
}
#endif
#endif
