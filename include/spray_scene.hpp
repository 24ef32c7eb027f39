// spray_scene.hpp -- header-only C++ drop-in for the reference's SceneT
// concept (spray::Scene<CacheT, TriMeshBuffer>, src/render/scene.h:62-251),
// over the C ABI of spray_scene.h / spray_rt.h.
//
// A tracer template (ooc::Tracer, insitu::MultiThreadTracer, the shaders)
// takes its scene type as ShaderT::SceneType (src/ooc/ooc_tracer.h:55); with
// spray_amd::Scene<> there the per-domain drains keep their call shapes:
//
//   scene->load(id, &sinfo);                                  // omp single
//   scene->intersect(sinfo.rtc_scene, sinfo.cache_block, r->org, r->dir,
//                    &rtc_isect_);                            // every thread
//   scene->occluded(sinfo.rtc_scene, r->org, r->dir, &rtc_ray_);
//   scene->intersectDomains(ray_ext);                         // Isector
//
// (ooc_tcontext.inl:28-100, insitu_tcontext.inl:125-186,
// ooc_isector.h:116-174).  The const queries are safe from any number of
// host threads at once: each calling thread gets its own submission lane
// (spray_rt_lane_*: stream + staging), created on first use.  load() must
// not run concurrently with queries -- the reference calls it inside omp
// single between barriers (ooc_pcontext.h:144-157).
//
// Record types are the caller's: RTCRayIntersection (96 B), Embree 2's
// RTCRay (96 B) and RTCRayExt (org / dir at the same offsets, a DomainList*
// with reset / push).  Only the byte offsets of spray_rt_ray_intersection
// are read or written.  Failures throw std::runtime_error (the reference
// CHECK-aborts).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "spray_rt.h"
#include "spray_scene.h"

namespace spray_amd {

// Scene::SceneInfo (scene.h:57-60): rtc_scene names the loaded domain's
// engine slot (the cache block), so occluded() -- which gets no cache block
// in the reference -- finds it.
typedef struct spray_rtc_scene_tag* RTCScene;
struct SceneInfo {
  RTCScene rtc_scene = nullptr;
  int cache_block = -1;
};
inline RTCScene slot_handle(int block) {
  return reinterpret_cast<RTCScene>(static_cast<uintptr_t>(block) + 1);
}
inline int handle_slot(RTCScene s) { return int(reinterpret_cast<uintptr_t>(s)) - 1; }

// Domain (src/render/domain.h:32-44), the fields the tracers read.
struct Domain {
  int id = 0;
  size_t num_vertices = 0, num_faces = 0;
  float world_aabb[6] = {0, 0, 0, 0, 0, 0};
};

// InsituPartition (src/render/data_partition.h:31-156): rank(domain).
class InsituPartition {
 public:
  void partition(const std::vector<Domain>& domains, const float bound[6], int nranks) {
    std::vector<float> boxes(6 * domains.size());
    for (size_t i = 0; i < domains.size(); ++i)
      std::memcpy(&boxes[6 * i], domains[i].world_aabb, 6 * sizeof(float));
    rank_.assign(domains.size(), 0);
    if (!domains.empty() &&
        spray_rt_insitu_partition(boxes.data(), int(domains.size()), bound, nranks, rank_.data()))
      throw std::runtime_error("spray_amd::InsituPartition: partition failed");
  }
  int rank(int id) const { return rank_[size_t(id)]; }
  size_t getNumDomains() const { return rank_.size(); }

 private:
  std::vector<int> rank_;
};

struct Light {  // PointLight / DiffuseHemisphereLight (src/render/light.h:31-89)
  int type = 0;  // 0 point, 1 diffuse hemisphere
  float position[3] = {0, 0, 0};
  float radiance[3] = {0, 0, 0};
};

template <typename Unused = void>
class Scene {
 public:
  Scene() = default;
  Scene(const Scene&) = delete;
  Scene& operator=(const Scene&) = delete;
  ~Scene() {
    for (auto& kv : lanes_) spray_rt_lane_destroy(kv.second);
    if (scene_) spray_scene_destroy(scene_);
  }

  // Scene::init (scene.inl:30-100).  storage_basepath and view_mode are
  // accepted for the signature; every domain is staged from ply_path, and
  // the cache warms up as the reference's film mode does (all domains when
  // cache_size < 0).  num_virtual_ranks: the in-situ partition's rank count.
  void init(const std::string& desc_filename, const std::string& ply_path,
            const std::string& storage_basepath, int cache_size, int view_mode,
            bool insitu_mode, int num_virtual_ranks, int hip_device = 0) {
    (void)storage_basepath;
    (void)view_mode;
    char err[512] = {0};
    if (spray_scene_create(desc_filename.c_str(), ply_path.c_str(), cache_size, hip_device,
                           &scene_, err, sizeof(err)))
      throw std::runtime_error(std::string("spray_amd::Scene::init: ") + err);
    rt_ = spray_scene_rt(scene_);
    const int n = spray_scene_num_domains(scene_);
    std::vector<float> boxes(6 * size_t(n));
    spray_scene_bounds(scene_, boxes.data(), bound_);
    domains_.resize(size_t(n));
    for (int i = 0; i < n; ++i) {
      Domain& d = domains_[size_t(i)];
      d.id = i;
      std::memcpy(d.world_aabb, &boxes[6 * size_t(i)], sizeof(d.world_aabb));
      spray_scene_domain_mesh(scene_, i, &d.num_vertices, &d.num_faces, nullptr, nullptr,
                              nullptr, nullptr);
    }
    for (int l = 0; l < spray_scene_num_lights(scene_); ++l) {
      float v[7];
      spray_scene_light(scene_, l, v);
      Light L;
      L.type = int(v[0]);
      std::memcpy(L.position, v + 1, 12);
      std::memcpy(L.radiance, v + 4, 12);
      lights_.push_back(L);
    }
    int nb = 0;
    spray_host_scene_bsdfs(desc_filename.c_str(), &nb, nullptr, err, sizeof(err));
    bsdfs_.resize(size_t(nb));
    if (nb && spray_host_scene_bsdfs(desc_filename.c_str(), &nb, bsdfs_.data(), err,
                                     sizeof(err)))
      throw std::runtime_error(std::string("spray_amd::Scene::init: ") + err);
    insitu_ = insitu_mode;
    partition_.partition(domains_, bound_, num_virtual_ranks > 0 ? num_virtual_ranks : 1);
  }

  // Scene::load(id, SceneInfo*) (scene.inl:161-187): not concurrent with
  // queries (omp single in the reference).
  void load(int id, SceneInfo* sinfo) {
    int block = -1;
    if (spray_scene_load(scene_, id, &block))
      throw std::runtime_error(std::string("spray_amd::Scene::load: ") +
                               spray_scene_last_error(scene_));
    sinfo->cache_block = block;
    sinfo->rtc_scene = slot_handle(block);
    cache_block_ = block;
  }
  // Scene::load(int id) (scene.h:154, scene.inl:161-187): the loaded domain
  // becomes the scene's current one (the reference's scene_ / cache_block_),
  // which the scene-less queries below use -- the baseline tracers' form
  // (baseline_shader_ao.h:90, baseline_shader_pt.h:110, 139,
  // baseline_insitu_tracer.inl:653, 695, 700).
  void load(int id) {
    SceneInfo s;
    load(id, &s);
  }

  // Scene::intersect (scene.h:157-173): makeRadianceRay (rays.h:345-363),
  // closest hit in the cache block's domain, updateIntersection.
  template <typename IsectT>
  bool intersect(RTCScene rtc_scene, int cache_block, const float org[3], const float dir[3],
                 IsectT* isect) const {
    static_assert(sizeof(IsectT) >= sizeof(spray_rt_ray_intersection),
                  "RTCRayIntersection layout (96 B) expected");
    (void)rtc_scene;
    make_ray(org, dir, isect);
    lane_call(spray_rt_lane_intersect1M(lane(), cache_block, isect, 1, sizeof(IsectT)));
    return geom_id(isect) != SPRAY_RT_INVALID_ID;
  }
  template <typename V, typename IsectT>
  bool intersect(RTCScene rtc_scene, int cache_block, const V& org, const float dir[3],
                 IsectT* isect) const {  // the glm::vec3 origin overload
    const float o[3] = {org[0], org[1], org[2]};
    return intersect(rtc_scene, cache_block, o, dir, isect);
  }

  // Scene::intersect(org, dir, isect) (scene.h:169-173): the current domain.
  template <typename IsectT>
  bool intersect(const float org[3], const float dir[3], IsectT* isect) const {
    return intersect(slot_handle(current()), current(), org, dir, isect);
  }

  // Scene::occluded (scene.h:175-195): makeShadowRay (rays.h:389-423), any
  // hit in the domain rtc_scene names; geomID = 0 when occluded.
  template <typename RayT>
  bool occluded(RTCScene rtc_scene, const float org[3], const float dir[3], RayT* ray) const {
    static_assert(sizeof(RayT) >= 84, "Embree 2 RTCRay layout expected");
    make_ray(org, dir, ray);
    lane_call(spray_rt_lane_occluded1M(lane(), handle_slot(rtc_scene), ray, 1, sizeof(RayT)));
    return geom_id(ray) != SPRAY_RT_INVALID_ID;
  }
  template <typename V, typename RayT>
  bool occluded(RTCScene rtc_scene, const V& org, const V& dir, RayT* ray) const {
    const float o[3] = {org[0], org[1], org[2]}, d[3] = {dir[0], dir[1], dir[2]};
    return occluded(rtc_scene, o, d, ray);
  }
  // Scene::occluded(org, dir, ray) (scene.h:175-178, 185-188): the current
  // domain (float[3] and glm::vec3 forms).
  template <typename RayT>
  bool occluded(const float org[3], const float dir[3], RayT* ray) const {
    return occluded(slot_handle(current()), org, dir, ray);
  }
  template <typename V, typename RayT,
            typename = decltype(std::declval<const V&>()[0] + 0.0f)>
  bool occluded(const V& org, const V& dir, RayT* ray) const {
    const float o[3] = {org[0], org[1], org[2]}, d[3] = {dir[0], dir[1], dir[2]};
    return occluded(slot_handle(current()), o, d, ray);
  }

  // Scene::updateIntersection (scene.h:203-205, TriMeshBuffer::
  // updateIntersection trimesh_buffer.cc:328-360): color and Ns of a hit
  // record from its primID, u, v and the current domain's mesh.
  template <typename IsectT>
  void updateIntersection(IsectT* isect) const {
    static_assert(sizeof(IsectT) >= sizeof(spray_rt_ray_intersection),
                  "RTCRayIntersection layout (96 B) expected");
    lane_call(spray_rt_lane_update_intersection1M(lane(), current(), isect, 1, sizeof(IsectT)));
  }

  // Scene::intersectDomains (scene.h:197, WbvhEmbree::intersect +
  // DomainList::sort): the ray's domain list, (t, id) ascending.
  template <typename RayExtT>
  void intersectDomains(RayExtT& ray) const {
    const int n = int(domains_.size());
    std::vector<int> ids(size_t(n > 0 ? n : 1));
    std::vector<float> ts(ids.size());
    int cnt = 0;
    lane_call(spray_rt_lane_domains1M(lane(), ray.org, ray.dir, 1, ids.data(), ts.data(), &cnt,
                                      n > 0 ? n : 1));
    ray.domains->reset();
    for (int k = 0; k < cnt; ++k) ray.domains->push(ids[size_t(k)], ts[size_t(k)]);
  }

  // ---- batched drains ----------------------------------------------------
  // The per-domain drains of the schedulers (ooc_tcontext.inl:28-100,
  // insitu_tcontext.inl:125-186) as gather -> one stream call -> scatter:
  // a thread copies its queue's rays into a record array (makeRay: the
  // fields makeRadianceRay / makeShadowRay set), submits it in one call on
  // its lane, and then runs its update / shade loop over the results in the
  // original queue order -- the results are pure functions of the rays, so
  // the VBuf / shading order of the reference is unchanged ("hard
  // parts").  M records of sizeof(RecordT) bytes, host or device memory.
  template <typename IsectT>
  void intersect1M(const SceneInfo& sinfo, IsectT* isects, size_t M) const {
    static_assert(sizeof(IsectT) >= sizeof(spray_rt_ray_intersection),
                  "RTCRayIntersection layout (96 B) expected");
    lane_call(spray_rt_lane_intersect1M(lane(), sinfo.cache_block, isects, M, sizeof(IsectT)));
  }
  template <typename RayT>
  void occluded1M(const SceneInfo& sinfo, RayT* rays, size_t M) const {
    static_assert(sizeof(RayT) >= 84, "Embree 2 RTCRay layout expected");
    lane_call(spray_rt_lane_occluded1M(lane(), handle_slot(sinfo.rtc_scene), rays, M,
                                       sizeof(RayT)));
  }
  // Isector::isectDomains over a queue (ooc_isector.h:116-124): ids / ts
  // [M][maxhits], counts[M], each list sorted by (t, id).
  void intersectDomains1M(const float* org, const float* dir, size_t M, int* ids, float* ts,
                          int* counts, int maxhits) const {
    lane_call(spray_rt_lane_domains1M(lane(), org, dir, M, ids, ts, counts, maxhits));
  }
  // RTCRayUtil::makeRadianceRay / makeShadowRay (rays.h:345-363, 389-423):
  // the same fields (tnear 0.001, tfar +inf, ids invalid, mask ~0, time 0).
  template <typename R>
  static void makeRay(const float org[3], const float dir[3], R* r) {
    make_ray(org, dir, r);
  }

  // Scene::getBsdf (scene.h:211): the domain's material record.
  const spray_rt_bsdf* getBsdf(int id) const { return &bsdfs_[size_t(id)]; }
  const InsituPartition& getInsituPartition() const { return partition_; }
  bool insitu() const { return insitu_; }
  size_t getNumDomains() const { return domains_.size(); }
  const std::vector<Domain>& getDomains() const { return domains_; }
  const std::vector<Light>& getLights() const { return lights_; }
  size_t getNumLights() const { return lights_.size(); }
  const float* getBound() const { return bound_; }
  spray_rt_ctx_t rt() const { return rt_; }

 private:
  template <typename R>
  static void make_ray(const float org[3], const float dir[3], R* r) {
    spray_rt_ray_intersection h;  // makeRadianceRay / makeShadowRay fields
    std::memcpy(&h, r, 84);
    for (int k = 0; k < 3; ++k) {
      h.org[k] = org[k];
      h.dir[k] = dir[k];
    }
    h.tnear = 0.001f;  // SPRAY_RAY_EPSILON
    h.tfar = std::numeric_limits<float>::infinity();
    h.time = 0.0f;
    h.mask = 0xFFFFFFFFu;
    h.geomID = h.primID = h.instID = SPRAY_RT_INVALID_ID;
    std::memcpy(r, &h, 84);
  }
  template <typename R>
  static uint32_t geom_id(const R* r) {
    uint32_t g;
    std::memcpy(&g, reinterpret_cast<const char*>(r) + 72, 4);
    return g;
  }
  // this thread's lane (created on first use)
  spray_rt_lane_t lane() const {
    const std::thread::id me = std::this_thread::get_id();
    {
      std::shared_lock<std::shared_mutex> lk(mu_);
      auto it = lanes_.find(me);
      if (it != lanes_.end()) return it->second;
    }
    std::unique_lock<std::shared_mutex> lk(mu_);
    spray_rt_lane_t l = nullptr;
    if (spray_rt_lane_create(rt_, &l))
      throw std::runtime_error(std::string("spray_amd::Scene: lane: ") +
                               spray_rt_lane_create_error());
    lanes_[me] = l;
    return l;
  }
  int current() const {
    if (cache_block_ < 0)
      throw std::runtime_error("spray_amd::Scene: no domain loaded (call load(id) first)");
    return cache_block_;
  }
  void lane_call(int rc) const {
    if (rc) throw std::runtime_error(std::string("spray_amd::Scene: ") +
                                     spray_rt_lane_last_error(lane()));
  }

  spray_scene_t scene_ = nullptr;
  spray_rt_ctx_t rt_ = nullptr;
  std::vector<Domain> domains_;
  std::vector<Light> lights_;
  std::vector<spray_rt_bsdf> bsdfs_;
  float bound_[6] = {0, 0, 0, 0, 0, 0};
  InsituPartition partition_;
  bool insitu_ = false;
  int cache_block_ = -1;  // the last loaded domain's cache block (scene_ / cache_block_)
  mutable std::shared_mutex mu_;
  mutable std::map<std::thread::id, spray_rt_lane_t> lanes_;
};

}  // namespace spray_amd
