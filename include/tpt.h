/*
 * tpt.h -- C ABI of the MI355X-native path-tracing hot path (libtpt.so).
 *
 * This is the drop-in boundary for the reference's per-pixel / per-sample
 * integration loop.  The reference has no C ABI; the interfaces each entry point
 * replaces are cited below (paths relative to the reference repository root):
 *
 *   Renderer::Render(std::string out, const Scene&, int spp, int j, bool bdpt)
 *                                               Renderer.hpp:11, Renderer.cpp:68-127
 *     -> tpt_create + tpt_upload_scene + tpt_render (+ host JPEG/float dump)
 *   FillBufferThread(j, off, spp, fb, bdpt)     Renderer.cpp:32-63
 *     -> tpt_render's pixel shard {pixel_begin, pixel_stride} (i = off; i += j)
 *   PathTrace(const Scene*, const Ray&, int&)   PathTracer.hpp:3 / PathTracer.cpp:44-134
 *   BDPT(const Scene*, const Ray&, int&, Vector3f* emissionBuffer)
 *                                               BDPT.hpp:172 / BDPT.cpp:282-315
 *     -> tpt_render_params.mode (TPT_MODE_PT / TPT_MODE_BDPT)
 *   Scene::BuildBVH / BVHAccel ctor / MeshTriangle ctor
 *                                               Scene.cpp:11-19, BVH.cpp:5-99, Triangle.cpp:32-75
 *     -> tpt_upload_scene (BVH built on the host, flattened, copied to HBM)
 *   Renderer::Render's std::async workers + splat merge   Renderer.cpp:86-114
 *     -> tpt_multi_* / tpt_render_multi (pixel shards per GPU + one RCCL reduce)
 *
 * Conventions: every call is synchronous and returns 0 on
 * success or a negative TPT_E* code; no C++ exception crosses the ABI; the
 * last error text is available from tpt_last_error(ctx).  Input arrays are
 * caller-owned and copied; device buffers are owned by the context.  One
 * context per device.  Output buffers are caller-owned host fp32 arrays.
 * No torch / HIP types appear in any signature.
 */
#ifndef TPT_H
#define TPT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: tpt_stats gained nonfinite / nonfinite_splat (round 3) */
#define TPT_ABI_VERSION 2

/* error codes */
#define TPT_OK 0
#define TPT_E_INVALID (-1)   /* bad argument */
#define TPT_E_DEVICE (-2)    /* HIP runtime error */
#define TPT_E_NOSCENE (-3)   /* tpt_render before tpt_upload_scene */
#define TPT_E_ALLOC (-4)     /* device allocation failed */
#define TPT_E_UNSUPPORTED (-5)

/* Material.hpp:11-13 (enum MaterialType) */
#define TPT_DIELETRIC 0
#define TPT_METAL 1
#define TPT_TRANSPARENT 2

/* Object.hpp:14-18 (enum FaceCulling) */
#define TPT_CULL_BACK 0
#define TPT_CULL_FRONT 1
#define TPT_NO_CULL 2

/* object kinds */
#define TPT_OBJ_MESH 0   /* MeshTriangle (Triangle.hpp:53-92) */
#define TPT_OBJ_SPHERE 1 /* Sphere (Sphere.hpp) */

/* render modes */
#define TPT_MODE_PT 0    /* PathTrace, PathTracer.cpp:44 */
#define TPT_MODE_BDPT 1  /* BDPT, BDPT.cpp:282 */
/* PathTrace with the indirect bounce enabled: PathTracer.cpp:44-134 without the
 * `break` at :109 (dead code at HEAD).  Off by default: no
 * reference entry point selects it, and it changes results against HEAD. */
#define TPT_MODE_PT_INDIRECT 2

/* tpt_render_params.flags.
 * TPT_FLAG_SAMPLE_SEED: per-sample seeding, a throughput mode that does NOT reproduce
 * the reference ("per-sample seeding for spp-parallel
 * throughput"; off by default).  The reference runs one XorShift32 stream per pixel
 * through all its samples (ResetRandom(i + 1), Renderer.cpp:42); with this flag
 * sample j of pixel i starts its own stream at tpt_sample_seed(i, j) instead, so the
 * samples are independent: the estimator is the reference's, the random numbers are
 * not.  A pixel's samples are then spread over lanes with no stream replay: PT drops
 * the skip-ahead, PT-indirect runs TPT_PT_LANES lanes per pixel.  The pixel still sums
 * (1/spp) * L in sample order for PT; PT-indirect sums per lane, then over lanes.
 * PT and PT-indirect only (BDPT returns TPT_E_UNSUPPORTED). */
#define TPT_FLAG_SAMPLE_SEED 1

/* Material (Material.hpp:15-44).  `rough` is the already-converted roughness
 * (Material::SetSmoothness -> SmoothnessToRoughenss, GGX.hpp:38-40). */
typedef struct tpt_material {
    int32_t type;
    float emission[3];
    float ior_d;
    float ior_m[3];
    float ior_m_k[3];
    float kd[3];
    float rough;
} tpt_material;

/* One scene object, in Scene::Add order (main.cpp:95-102).
 * Mesh: triangles are vertices[3*first_triangle .. 3*(first_triangle+num_triangles))
 *       as a triangle soup in OBJ face order (Triangle.cpp:46-65).
 * Sphere: center / radius (Sphere.hpp:16). */
typedef struct tpt_object {
    int32_t kind;
    int32_t material;
    int32_t first_triangle;
    int32_t num_triangles;
    float center[3];
    float radius;
} tpt_object;

typedef struct tpt_scene_desc {
    int32_t width, height;        /* Scene(int w, int h), Scene.hpp:29 */
    float eye[3];                 /* Scene::eyePos */
    float background[3];          /* Scene::backgroundColor */
    double fov;                   /* Scene::fov (degrees, double), Scene.hpp:21 */
    int32_t num_materials;
    const tpt_material* materials;
    int32_t num_objects;
    const tpt_object* objects;
    int64_t num_vertices;         /* 3 * total triangles */
    const float* vertices;        /* xyz per vertex */
} tpt_scene_desc;

typedef struct tpt_render_params {
    int32_t spp;                  /* samples per pixel (Renderer.cpp:43) */
    int32_t mode;                 /* TPT_MODE_PT | TPT_MODE_BDPT | TPT_MODE_PT_INDIRECT */
    int64_t pixel_begin;          /* first pixel of this shard (Renderer.cpp:38 `i = off`) */
    int64_t pixel_stride;         /* shard stride (Renderer.cpp:38 `i += j`); 1 = all pixels */
    int32_t flags;                /* 0, or TPT_FLAG_SAMPLE_SEED */
    int32_t reserved;
} tpt_render_params;

/* tpt_stats grew in ABI 2 (nonfinite, nonfinite_splat: 56 bytes, was 40), and every
 * render entry writes the whole struct.  A caller must check
 * tpt_abi_version() == TPT_ABI_VERSION before its first render call (a binary built
 * against ABI 1 would be overwritten past its 40-byte stats object); the in-reference
 * binding and pytpt do. */
typedef struct tpt_stats {
    int64_t pixels;               /* pixels rendered by this call */
    int64_t samples;              /* pixels * spp */
    int64_t bounces;              /* sum of outBounces (Renderer.cpp:52, 64-bit) */
    double kernel_ms;             /* device time of the integration kernel(s) */
    double total_ms;              /* wall time of tpt_render incl. copies */
    /* Pixels of this call's output whose radiance (rgb) / splat has a non-finite
     * component.  The reference's only NaN guard is an MSVC _DEBUG trap
     * (Vector.hpp:19-22): in a release build a NaN sample poisons its pixel silently
     * (config 5's frame has one, pixel 485594).  Counted on the device after the
     * render, outside kernel_ms. */
    int64_t nonfinite;
    int64_t nonfinite_splat;
} tpt_stats;

typedef struct tpt_ctx tpt_ctx;

/* Create a context on HIP device `device`. */
int tpt_create(int device, tpt_ctx** out);
void tpt_destroy(tpt_ctx* ctx);
const char* tpt_last_error(const tpt_ctx* ctx);
int tpt_abi_version(void);
/* The HIP version libtpt was compiled against (HIP_VERSION) and the one of the HIP
 * runtime the process has loaded (hipRuntimeGetVersion; -1 if it cannot be read).  A
 * process that loaded another libamdhip64 first (torch bundles its own) binds libtpt
 * to that one: pytpt warns when the major versions differ. */
void tpt_hip_versions(int* compiled, int* runtime);

/* Build the two-level BVH exactly as the reference does (median split, BVH.cpp:30-99;
 * top level over objects, one BVH per mesh), flatten it and copy it to HBM. */
int tpt_upload_scene(tpt_ctx* ctx, const tpt_scene_desc* desc);

/* Render one shard.  rgb: W*H*3 floats, pixel radiance accumulated as the
 * reference does ((1.0f/spp) * L per sample, Renderer.cpp:49/51); pixels outside
 * the shard are written as 0.  splat (BDPT only, may be NULL for PT): W*H*3
 * floats, the t=1 light-tracing splat buffer already scaled by 1/spp
 * (Renderer.cpp:58-60).  The caller adds splat to rgb (Renderer.cpp:98-114).
 * stats may be NULL. */
int tpt_render(tpt_ctx* ctx, const tpt_render_params* params, float* rgb, float* splat, tpt_stats* stats);

/* Same as tpt_render for an explicit pixel list (replay of arbitrary pixels).
 * rgb: n*3 floats (one row per listed pixel); splat as in tpt_render. */
int tpt_render_pixels(tpt_ctx* ctx, int32_t spp, int32_t mode, const int64_t* pixels, int64_t n,
                      float* rgb, float* splat, tpt_stats* stats);

/* Device-resident variants for callers that keep buffers in HBM (bench, multi-GPU
 * reduce): rgb_dev / splat_dev are device pointers of W*H*3 floats, written on the
 * context's stream; the call returns after the kernels complete. */
int tpt_render_device(tpt_ctx* ctx, const tpt_render_params* params, float* rgb_dev, float* splat_dev,
                      tpt_stats* stats);

/* Closest-hit queries through the device BVH (Scene::Intersect, Scene.cpp:21-35).
 * rays: n*6 floats {origin, direction}; out: n*8 floats
 * {hit, x.xyz, N.xyz, primitive ordinal} (ordinal = position of the hit Triangle /
 * Sphere in the scene's object order: each mesh's triangles in file order, a sphere
 * at its Scene::Add position; -1 on miss). */
int tpt_intersect(tpt_ctx* ctx, const float* rays, int64_t n, int32_t cull, float* out);

/* Camera scale (SceneRenderingHelper.cpp:12-14), computed on the host. */
float tpt_camera_scale(double fov);

/* The XorShift32 seed of sample j of pixel i under TPT_FLAG_SAMPLE_SEED: the
 * SplitMix64 finalizer of ((i + 1) << 32 | j), folded to 32 bits (never 0). */
uint32_t tpt_sample_seed(int64_t pixel, int32_t sample);

/* ---- multi-GPU (one process, the GPUs of one node) ---------------------------
 * Replaces Renderer::Render's worker split and splat merge (Renderer.cpp:86-114)
 * across devices instead of threads: device r of n renders the pixel shard
 * i = r, r + n, ... (Renderer.cpp:38's interleave) with its own context, then ONE
 * RCCL reduce (sum, fp32, over xGMI) of every device's [rgb; splat] buffer onto the
 * first device.  Radiance shards are disjoint, so the frame is bit-identical to one
 * GPU; splats (already scaled by 1/spp per device, Renderer.cpp:59) are summed as the
 * reference sums its per-thread buffers (:98-114).  RCCL is loaded when the group is
 * created; TPT_E_UNSUPPORTED if it cannot be. */
typedef struct tpt_multi tpt_multi;

/* devices: ngpu HIP device ids (NULL: 0 .. ngpu-1); one tpt_ctx per device. */
int tpt_multi_create(int ngpu, const int* devices, tpt_multi** out);
void tpt_multi_destroy(tpt_multi* m);
const char* tpt_multi_last_error(const tpt_multi* m);
/* tpt_upload_scene on every device. */
int tpt_multi_upload_scene(tpt_multi* m, const tpt_scene_desc* desc);
/* As tpt_render for the whole frame (params->pixel_begin 0, pixel_stride 1: the group
 * shards it).  stats sums pixels / samples / bounces over devices; kernel_ms is the
 * slowest device's. */
int tpt_render_multi(tpt_multi* m, const tpt_render_params* params, float* rgb, float* splat, tpt_stats* stats);

#ifdef __cplusplus
}
#endif

#endif /* TPT_H */
