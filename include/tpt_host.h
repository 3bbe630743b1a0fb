/*
 * tpt_host.h -- C entry points of the host-side caller surface (libtpt.so).
 *
 * The reference hard-codes its scenes in main.cpp:49-103; these build the same
 * scenes through the C++ mirror (tpt_scene_api.hpp: Scene, Material, MeshTriangle,
 * Sphere) and hand out the flattened tpt_scene_desc, so non-C++ callers (the Python
 * tests / bench, a ctypes or cgo binding) can render the reference's scenes.
 */
#ifndef TPT_HOST_H
#define TPT_HOST_H

#include "tpt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tpt_preset tpt_preset;

/* name: "silver" | "standard" | "refractive_ball" | "occlusion" | "multi_light" |
 *       "emissive_sphere" | "background" |
 *       "smooth_dielectric" | "bunny".  Returns 0 or TPT_E_INVALID. */
int tpt_preset_load(const char* models_dir, const char* name, int32_t width, int32_t height, tpt_preset** out);
const tpt_scene_desc* tpt_preset_desc(const tpt_preset* p);
void tpt_preset_free(tpt_preset* p);

/* Film output (SceneRenderingHelper.cpp:57-70): .jpg (baseline, q100), .ppm, .pfm */
int tpt_save_image(const float* rgb, int32_t width, int32_t height, const char* path);

#ifdef __cplusplus
}
#endif

#endif
