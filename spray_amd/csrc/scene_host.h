// scene_host.h -- host side above the C ABI, mirroring the reference's scene
// surface for the hot path:
//   SceneLoader / PlyLoader        src/io/scene_loader.cc, src/io/ply_loader.cc
//   TriMeshBuffer::load            src/render/trimesh_buffer.cc:117-169
//   InfiniteCache / LruCache       src/render/infinite_cache.cc, lru_cache.cc
//   Scene<CacheT, TriMeshBuffer>   src/render/scene.h:62-251, scene.inl
//   Camera::init                   src/render/camera.h:128-166
// GpuScene keeps the reference's method names and argument meaning
// (load / intersect / occluded / intersectDomains / getNumDomains / ...);
// the per-ray calls forward to the engine's 1M streams, and batched
// variants expose the streams directly.
#pragma once

#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <string>
#include <vector>

#include "spray_rt.h"

namespace spray_rt {
namespace detail {
struct SlotImage;
}
}  // namespace spray_rt

namespace spray_host {

struct Domain {  // src/render/domain.h:32-44
  int id = 0;
  size_t num_vertices = 0;
  size_t num_faces = 0;
  std::string filename;
  float object_aabb[6] = {0, 0, 0, 0, 0, 0};
  float world_aabb[6] = {0, 0, 0, 0, 0, 0};
  float transform[16];  // glm column-major
  std::vector<std::string> material;
};

struct Light {
  int type = 0;  // 0 point, 1 diffuse hemisphere
  float position[3] = {0, 0, 0};
  float radiance[3] = {0, 0, 0};
};

struct Mesh {
  std::vector<float> vertices;   // [nv][3]
  std::vector<uint32_t> faces;   // [nf][3]
  std::vector<uint32_t> colors;  // [nv] 0xRRGGBB
  std::vector<float> normals;    // [nv][3] unnormalised
};

// SceneLoader::load (scene_loader.cc:315-358).  Returns false + message.
bool load_scene_file(const std::string& desc, const std::string& ply_path,
                     std::vector<Domain>* domains, std::vector<Light>* lights,
                     std::string* err);
// PlyLoader::load (ply_loader.cc:179-324).
bool load_ply(const std::string& filename, Mesh* mesh, std::string* err);
// mat4 * vec4(v, 1) per vertex (trimesh_buffer.cc:141-157).
void transform_vertices(const float m[16], float* v, size_t nverts);
// computeNormals (trimesh_buffer.cc:267-326).
void compute_normals(Mesh* mesh);
// Camera::init -> cam[14] = pos, lowerleft, wvec, hvec, w, h.
void camera_init(const float pos[3], const float lookat[3], const float up[3],
                 float vfov, int image_w, int image_h, float cam[14]);

// domain -> cache block (InfiniteCache / LruCache semantics)
class DomainCache {
 public:
  void init(int num_domains, int cache_size);
  // true on hit; *block = cache block
  bool load(int domid, int* block);
  int capacity() const { return capacity_; }
  bool lru() const { return lru_; }

 private:
  struct Block {
    int block, domain;
  };
  bool lru_ = false;
  int capacity_ = 0, size_ = 0;
  std::vector<int> status_;  // 1 loaded
  std::list<Block> blocks_;  // front = LRU, back = MRU
  std::map<int, std::list<Block>::iterator> where_;
};

struct SceneInfo {  // scene.h:57-60 (rtc_scene -> engine slot)
  int cache_block = -1;
};

class GpuScene {
 public:
  GpuScene() = default;
  ~GpuScene();
  GpuScene(const GpuScene&) = delete;
  GpuScene& operator=(const GpuScene&) = delete;

  // Scene::init (scene.inl:30-100): parse, merge bounds, init cache, warm
  // up (every domain when cache_size < 0), domain bounds to the engine.
  int init(const std::string& desc, const std::string& ply_path,
           int cache_size, int hip_device);

  // Scene::load(id, SceneInfo*) (scene.inl:161-187)
  int load(int id, SceneInfo* sinfo);

  // per-ray surface (scene.h:157-195)
  bool intersect(const SceneInfo& s, const float org[3], const float dir[3],
                 spray_rt_ray_intersection* isect);
  bool occluded(const SceneInfo& s, const float org[3], const float dir[3],
                spray_rt_ray_intersection* ray);
  // sorted (id, tmin) list of the domains a ray overlaps (scene.h:197)
  int intersectDomains(const float org[3], const float dir[3], int* ids,
                       float* ts, int maxhits);

  // batched streams
  int intersect1M(int cache_block, spray_rt_ray_intersection* rays, size_t n);
  int occluded1M(int cache_block, spray_rt_ray_intersection* rays, size_t n);

  size_t getNumDomains() const { return domains_.size(); }
  const std::vector<Domain>& getDomains() const { return domains_; }
  const std::vector<Light>& getLights() const { return lights_; }
  const float* getBound() const { return bound_; }
  spray_rt_ctx_t rt() const { return rt_; }
  const std::string& error() const { return err_; }
  int cacheCapacity() const { return cache_.capacity(); }

 private:
  int upload(int id, int block);
  // the device image of domain id in pinned host memory (images_, pinned_);
  // thread-safe for distinct ids once the domain's PLY is in ply_cache_
  int build_image(int id, std::string* err);
  // every image built up front, in parallel, when they fit the host budget
  // (SPRAY_SCENE_PREBUILD_MB of pinned memory, default 4096; 0 = each on
  // its first miss); an all-resident cache frees them after its warm-up
  int prebuild_images();
  int fail(int code, const std::string& msg);

  std::vector<Domain> domains_;
  std::vector<Light> lights_;
  float bound_[6];
  DomainCache cache_;
  std::vector<int> block_domain_;  // cache block -> resident domain
  std::map<std::string, Mesh> ply_cache_;  // parsed PLY by filename
  // per-domain device images, built on the first load (upload())
  std::vector<spray_rt::detail::SlotImage> images_;
  std::vector<void*> pinned_;  // their bytes in pinned host memory
  spray_rt_ctx_t rt_ = nullptr;
  std::string err_;
};

}  // namespace spray_host
