/*
 * spray_scene.h -- C ABI of the host-side scene layer (scene files, PLY
 * meshes, domain cache) that sits above spray_rt.h, mirroring the
 * reference's Scene<CacheT, TriMeshBuffer> surface for bindings:
 *   spray_scene_create      Scene::init (src/render/scene.inl:30-100):
 *                           SceneLoader::load (src/io/scene_loader.cc:315-358),
 *                           mergeDomainBounds (scene.inl:295-349), cache init
 *                           and warm-up (scene.inl:79-93), WbvhEmbree::init.
 *   spray_scene_load        Scene::load(id, SceneInfo*) (scene.inl:161-187)
 *                           with InfiniteCache/LruCache block assignment
 *                           (src/render/infinite_cache.cc:47-60,
 *                           src/render/lru_cache.cc:65-171).
 *   spray_scene_intersect1  Scene::intersect(rtc_scene, cache_block, org, dir,
 *                           isect) (src/render/scene.h:157-161).
 *   spray_scene_occluded1   Scene::occluded(rtc_scene, org, dir, ray)
 *                           (src/render/scene.h:191-195).
 *   spray_camera_init       Camera::init (src/render/camera.h:128-166).
 */
#ifndef SPRAY_SCENE_H_
#define SPRAY_SCENE_H_

#include <stddef.h>
#include <stdint.h>

#include "spray_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spray_scene* spray_scene_t;

/* cache_size < 0 (or >= #domains): every domain resident (InfiniteCache),
 * otherwise an LRU of cache_size slots.  err receives a message on failure. */
int spray_scene_create(const char* desc, const char* ply_path, int cache_size,
                       int hip_device, spray_scene_t* out, char* err,
                       size_t errlen);
int spray_scene_destroy(spray_scene_t scene);
const char* spray_scene_last_error(spray_scene_t scene);
spray_rt_ctx_t spray_scene_rt(spray_scene_t scene);
int spray_scene_num_domains(spray_scene_t scene);
int spray_scene_cache_capacity(spray_scene_t scene);
int spray_scene_bounds(spray_scene_t scene, float* boxes, float* bound);
int spray_scene_num_lights(spray_scene_t scene);
int spray_scene_light(spray_scene_t scene, int i, float* out7);
int spray_scene_load(spray_scene_t scene, int id, int* cache_block);
/* return 1 on hit / occlusion, 0 otherwise */
int spray_scene_intersect1(spray_scene_t scene, int cache_block,
                           const float* org, const float* dir,
                           spray_rt_ray_intersection* isect);
int spray_scene_occluded1(spray_scene_t scene, int cache_block,
                          const float* org, const float* dir,
                          spray_rt_ray_intersection* ray);
int spray_camera_init(const float* pos, const float* lookat, const float* up,
                      float vfov, int w, int h, float* cam14);
int spray_scene_domain_mesh(spray_scene_t scene, int id, size_t* nverts,
                            size_t* nfaces, float* verts, uint32_t* faces,
                            uint32_t* colors, float* normals);

/* Host-only (no GPU): parse a .spray file.  Call with NULL outputs for the
 * counts.  boxes[n][6] world bounds, transforms[n][16] (column-major),
 * lights[nl][7] = type, position[3], radiance[3]. */
int spray_host_parse_scene(const char* desc, const char* ply_path,
                           int* ndomains, int* nlights, float* boxes,
                           float* transforms, float* lights, char* err,
                           size_t errlen);
/* Host-only: the domains' materials (SceneLoader::parseMaterial,
 * src/io/scene_loader.cc:88-130) as spray_rt_bsdf records (diffuse/mirror:
 * p = albedo/reflectance; glass/transmission: p = eta_a, eta_b).  NULL
 * bsdfs -> count only. */
int spray_host_scene_bsdfs(const char* desc, int* ndomains, spray_rt_bsdf* bsdfs, char* err,
                           size_t errlen);
/* Host-only: TriMeshBuffer::load for domain `id` (PLY, transform, normals).
 * NULL arrays -> sizes only. */
int spray_host_domain_mesh(const char* desc, const char* ply_path, int id,
                           size_t* nverts, size_t* nfaces, float* verts,
                           uint32_t* faces, uint32_t* colors, float* normals);

#ifdef __cplusplus
}
#endif
#endif
