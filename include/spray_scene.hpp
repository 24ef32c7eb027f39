// spray_scene.hpp -- header-only C++ drop-in for the reference's SceneT
// concept (spray::Scene<CacheT, TriMeshBuffer>, src/render/scene.h:62-251),
// over the C ABI of spray_scene.h / spray_rt.h.
//
// A tracer template (ooc::Tracer, insitu::MultiThreadTracer, the shaders)
// takes its scene type as ShaderT::SceneType (src/ooc/ooc_tracer.h:55); with
// spray_amd::Scene<AppTypes> there the tracers and shaders compile unchanged:
//
//   scene->load(id, &sinfo);                                  // omp single
//   scene->intersect(sinfo.rtc_scene, sinfo.cache_block, r->org, r->dir,
//                    &rtc_isect_);                            // every thread
//   scene->occluded(sinfo.rtc_scene, r->org, r->dir, &rtc_ray_);
//   scene->intersectDomains(ray_ext);                         // Isector
//   lights_ = scene->getLights();          // std::vector<Light*> (ooc_shader_pt.h:51)
//   const Bsdf* bsdf = scene_->getBsdf(domain_id);            // (:118)
//   const auto& ids = partition_->getDomains(rank);   // (insitu_tcontext.inl:98)
//   Aabb aabb = scene_.getBound(); scene_.buildWbvh();  // (spray_renderer.inl:47,96)
//
// (ooc_tcontext.inl:28-100, insitu_tcontext.inl:125-186,
// ooc_isector.h:116-174).  The const queries are safe from any number of
// host threads at once: each calling thread gets its own submission lane
// (spray_rt_lane_*: stream + staging), created on first use.  load() must
// not run concurrently with queries -- the reference calls it inside omp
// single between barriers (ooc_pcontext.h:144-157).
//
// Application types.  The shaders hold the scene's lights and materials as
// the application's own polymorphic classes (spray::Light with sample /
// sampleArea / isAreaLight, spray::Bsdf with isDelta / sampleDelta /
// sampleRandom, spray::Aabb with bounds[2]).  Scene<Types> builds them from
// the scene file through a policy:
//
//   struct SprayTypes {                       // what the reference would add
//     typedef spray::Light Light;  typedef spray::Bsdf Bsdf;  typedef spray::Aabb Aabb;
//     static Light* makeLight(const spray_amd::LightDesc& d);   // new PointLight(...)
//     static Bsdf* makeBsdf(const spray_rt_bsdf& b);            // new DiffuseBsdf(...)
//     static Aabb makeAabb(const float lo_hi[6]);
//   };
//   typedef spray_amd::Scene<SprayTypes> SceneType;
//
// DefaultTypes (below) are plain records with the same query methods for
// callers that bring no types of their own.  Lights are owned and deleted
// by the scene (as Scene::~Scene does, scene.h:66-71), BSDFs likewise (the
// reference's Domain owns its Bsdf, domain.h:33).
//
// Record types are the caller's: RTCRayIntersection (96 B), Embree 2's
// RTCRay (96 B) and RTCRayExt (org / dir at the same offsets, a DomainList*
// with reset / push).  Only the byte offsets of spray_rt_ray_intersection
// are read or written.  Failures throw std::runtime_error (the reference
// CHECK-aborts).
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <limits>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "spray_rt.h"
#include "spray_scene.h"

namespace spray_amd {

// Scene::SceneInfo (scene.h:57-60): rtc_scene names the loaded domain's
// engine slot (the cache block), so occluded() -- which gets no cache block
// in the reference -- finds it.
//
// The tracers declare the reference's own record, `spray::SceneInfo
// sinfo_` (ooc_pcontext.h:83, insitu_tcontext.h:186), whose rtc_scene is
// Embree 2's opaque handle (`typedef struct __RTCScene* RTCScene`).  load(),
// intersect(), occluded() and the batched drains are therefore templates on
// the caller's types: any record with members rtc_scene (a pointer type)
// and cache_block (an int), and any pointer-typed scene handle.  The slot
// travels inside the handle's bits (slot + 1; a null handle is no slot), so
// the caller's handle type never has to be a real Embree scene.
// spray_amd::SceneInfo / RTCScene below are the same shapes for callers
// that bring none.
typedef struct spray_rtc_scene_tag* RTCScene;
struct SceneInfo {
  RTCScene rtc_scene = nullptr;
  int cache_block = -1;
};
template <typename HandleT = RTCScene>
inline HandleT slot_handle(int block) {
  static_assert(std::is_pointer<HandleT>::value, "scene handles are pointer types");
  return reinterpret_cast<HandleT>(static_cast<uintptr_t>(block) + 1);
}
template <typename HandleT>
inline int handle_slot(HandleT s) {
  static_assert(std::is_pointer<HandleT>::value, "scene handles are pointer types");
  return int(reinterpret_cast<uintptr_t>(s)) - 1;
}

// A light of the scene file (SceneLoader, scene_loader.cc:262-313):
// type = SPRAY_RT_LIGHT_POINT (position, radiance) or
// SPRAY_RT_LIGHT_HEMISPHERE (radiance).
struct LightDesc {
  int type = SPRAY_RT_LIGHT_POINT;
  float position[3] = {0, 0, 0};
  float radiance[3] = {0, 0, 0};
};

// ---- default application types ---------------------------------------------
struct vec3 {
  float x = 0, y = 0, z = 0;
  vec3() = default;
  vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  const float& operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

// Aabb (src/render/aabb.h:32-80): the members the tracers read.
struct Aabb {
  vec3 bounds[2];
  const vec3& getMin() const { return bounds[0]; }
  const vec3& getMax() const { return bounds[1]; }
  const vec3& getBound(std::uint8_t i) const { return bounds[i]; }
  vec3 getCenter() const {  // (min + max) * 0.5
    return vec3((bounds[0].x + bounds[1].x) * 0.5f, (bounds[0].y + bounds[1].y) * 0.5f,
                (bounds[0].z + bounds[1].z) * 0.5f);
  }
  bool isValid() const {
    return bounds[0].x <= bounds[1].x && bounds[0].y <= bounds[1].y && bounds[0].z <= bounds[1].z;
  }
};

// Light / PointLight / DiffuseHemisphereLight (src/render/light.h:31-89):
// the parameters and the point light's sample(); area-light sampling is the
// shading layer's (spray_rt_shade on the device).
class Light {
 public:
  virtual ~Light() = default;
  virtual bool isAreaLight() const = 0;
  virtual int type() const = 0;
  const vec3& radiance() const { return radiance_; }

 protected:
  explicit Light(const vec3& r) : radiance_(r) {}
  vec3 radiance_;
};
class PointLight : public Light {
 public:
  PointLight(const vec3& position, const vec3& radiance) : Light(radiance), position_(position) {}
  bool isAreaLight() const override { return false; }
  int type() const override { return SPRAY_RT_LIGHT_POINT; }
  const vec3& position() const { return position_; }
  // PointLight::sample (light.h:47-53): wi = normalize(position - p), pdf 1
  vec3 sample(const vec3& p, vec3* wi, float* pdf) const {
    vec3 d(position_.x - p.x, position_.y - p.y, position_.z - p.z);
    const float inv = 1.0f / std::sqrt((d.x * d.x + d.y * d.y) + d.z * d.z);
    *wi = vec3(d.x * inv, d.y * inv, d.z * inv);
    *pdf = 1.0f;
    return radiance_;
  }

 private:
  vec3 position_;
};
class DiffuseHemisphereLight : public Light {
 public:
  explicit DiffuseHemisphereLight(const vec3& radiance) : Light(radiance) {}
  bool isAreaLight() const override { return true; }
  int type() const override { return SPRAY_RT_LIGHT_HEMISPHERE; }
};

// Bsdf (src/render/reflection.h:219-239): the material record of a domain.
class Bsdf {
 public:
  explicit Bsdf(const spray_rt_bsdf& r) : rec_(r) {}
  virtual ~Bsdf() = default;
  bool isDelta() const { return rec_.type != SPRAY_RT_BSDF_DIFFUSE; }
  int type() const { return rec_.type; }
  const spray_rt_bsdf& record() const { return rec_; }

 private:
  spray_rt_bsdf rec_;
};

struct DefaultTypes {
  typedef spray_amd::Light Light;
  typedef spray_amd::Bsdf Bsdf;
  typedef spray_amd::Aabb Aabb;
  static Light* makeLight(const LightDesc& d) {
    const vec3 r(d.radiance[0], d.radiance[1], d.radiance[2]);
    if (d.type == SPRAY_RT_LIGHT_HEMISPHERE) return new DiffuseHemisphereLight(r);
    return new PointLight(vec3(d.position[0], d.position[1], d.position[2]), r);
  }
  static Bsdf* makeBsdf(const spray_rt_bsdf& b) { return new Bsdf(b); }
  static Aabb makeAabb(const float b[6]) {
    Aabb a;
    a.bounds[0] = vec3(b[0], b[1], b[2]);
    a.bounds[1] = vec3(b[3], b[4], b[5]);
    return a;
  }
};

// Domain (src/render/domain.h:32-44), the fields the tracers read; bsdf is
// owned by the scene.
template <typename Types>
struct BasicDomain {
  unsigned id = 0;
  std::size_t num_vertices = 0, num_faces = 0;
  typename Types::Aabb world_aabb{};
  typename Types::Bsdf* bsdf = nullptr;
};

// InsituPartition (src/render/data_partition.h:31-243): rank(domain),
// getDomains(rank), computePartition(n).  The Morton codes and their
// dealing are the engine's (spray_rt_insitu_partition_mode).
class InsituPartition {
 public:
  enum Mode {
    GROUP_CLOSE_DOMAINS = SPRAY_RT_PARTITION_GROUP_CLOSE,  // the reference's compiled mode
    ROUND_ROBIN = SPRAY_RT_PARTITION_ROUND_ROBIN,          // :139-155, "scatter close domains"
  };

  // partition(ndomains, domains, scene_aabb, num_ranks) (:59-156)
  template <typename DomainT, typename AabbT>
  void partition(int ndomains, const std::vector<DomainT>& domains, const AabbT& scene_aabb,
                 int num_ranks, Mode mode = GROUP_CLOSE_DOMAINS) {
    if (ndomains != int(domains.size()) || num_ranks <= 0)
      throw std::runtime_error("spray_amd::InsituPartition: bad arguments");
    boxes_.assign(6 * domains.size(), 0.f);
    for (size_t i = 0; i < domains.size(); ++i)
      for (int k = 0; k < 3; ++k) {
        boxes_[6 * size_t(domains[i].id) + size_t(k)] = domains[i].world_aabb.bounds[0][k];
        boxes_[6 * size_t(domains[i].id) + 3 + size_t(k)] = domains[i].world_aabb.bounds[1][k];
      }
    for (int k = 0; k < 3; ++k) {
      bound_[k] = scene_aabb.bounds[0][k];
      bound_[3 + k] = scene_aabb.bounds[1][k];
    }
    mode_ = mode;
    domain_to_rank_ = deal(num_ranks);
    rank_to_domains_.assign(size_t(num_ranks), std::list<int>());
    for (size_t id = 0; id < domain_to_rank_.size(); ++id)  // mapDomains (:226-240)
      rank_to_domains_[size_t(domain_to_rank_[id])].push_back(int(id));
  }
  int rank(int id) const { return domain_to_rank_[size_t(id)]; }
  const std::list<int>& getDomains(int rank) const { return rank_to_domains_[size_t(rank)]; }
  std::size_t getNumDomains(int rank) const { return rank_to_domains_[size_t(rank)].size(); }
  int getNumDomains() const { return int(domain_to_rank_.size()); }
  // computePartition (:157-213): the same dealing over num_partitions
  std::vector<int> computePartition(int num_partitions) const { return deal(num_partitions); }
  Mode mode() const { return mode_; }

 private:
  std::vector<int> deal(int nranks) const {
    const int n = int(boxes_.size() / 6);
    std::vector<int> owner(size_t(n), 0);
    if (n && spray_rt_insitu_partition_mode(boxes_.data(), n, bound_, nranks, int(mode_),
                                            owner.data()))
      throw std::runtime_error("spray_amd::InsituPartition: partition failed");
    return owner;
  }
  std::vector<float> boxes_;
  float bound_[6] = {0, 0, 0, 0, 0, 0};
  Mode mode_ = GROUP_CLOSE_DOMAINS;
  std::vector<int> domain_to_rank_;
  std::vector<std::list<int>> rank_to_domains_;
};

template <typename Types = DefaultTypes>
class Scene {
 public:
  typedef typename Types::Light Light;
  typedef typename Types::Bsdf Bsdf;
  typedef typename Types::Aabb Aabb;
  typedef BasicDomain<Types> Domain;

  Scene() = default;
  Scene(const Scene&) = delete;
  Scene& operator=(const Scene&) = delete;
  ~Scene() {
    for (auto& kv : lanes_) spray_rt_lane_destroy(kv.second);
    for (Light* l : lights_) delete l;
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
    boxes_.assign(6 * size_t(n), 0.f);
    spray_scene_bounds(scene_, boxes_.data(), bound_);
    int nb = 0;
    spray_host_scene_bsdfs(desc_filename.c_str(), &nb, nullptr, err, sizeof(err));
    std::vector<spray_rt_bsdf> recs(static_cast<size_t>(nb));
    if (nb && spray_host_scene_bsdfs(desc_filename.c_str(), &nb, recs.data(), err, sizeof(err)))
      throw std::runtime_error(std::string("spray_amd::Scene::init: ") + err);
    domains_.resize(size_t(n));
    for (int i = 0; i < n; ++i) {
      Domain& d = domains_[size_t(i)];
      d.id = unsigned(i);
      d.world_aabb = Types::makeAabb(&boxes_[6 * size_t(i)]);
      spray_scene_domain_mesh(scene_, i, &d.num_vertices, &d.num_faces, nullptr, nullptr,
                              nullptr, nullptr);
      if (i < nb) {
        bsdfs_.emplace_back(Types::makeBsdf(recs[size_t(i)]));
        d.bsdf = bsdfs_.back().get();
      }
    }
    for (int l = 0; l < spray_scene_num_lights(scene_); ++l) {
      float v[7];
      spray_scene_light(scene_, l, v);
      LightDesc L;
      L.type = int(v[0]);
      std::memcpy(L.position, v + 1, 12);
      std::memcpy(L.radiance, v + 4, 12);
      lights_.push_back(Types::makeLight(L));
    }
    insitu_ = insitu_mode;
    partition_.partition(n, domains_, getBound(), num_virtual_ranks > 0 ? num_virtual_ranks : 1);
  }

  // Scene::buildWbvh (scene.inl:103-105): the domain-level BVH.  The engine
  // builds its top-level tree over the domain boxes when they are set; this
  // sets them (again), so a caller that edited nothing gets the same tree.
  void buildWbvh() {
    if (spray_rt_domain_bounds(rt_, int(domains_.size()), boxes_.data()))
      throw std::runtime_error(std::string("spray_amd::Scene::buildWbvh: ") +
                               spray_rt_last_error(rt_));
  }

  // Scene::load(id, SceneInfo*) (scene.inl:161-187): not concurrent with
  // queries (omp single in the reference).  SceneInfoT: the caller's record
  // (spray::SceneInfo in the reference's tracers, ooc_pcontext.h:83, 150).
  template <typename SceneInfoT>
  void load(int id, SceneInfoT* sinfo) {
    int block = -1;
    if (spray_scene_load(scene_, id, &block))
      throw std::runtime_error(std::string("spray_amd::Scene::load: ") +
                               spray_scene_last_error(scene_));
    sinfo->cache_block = block;
    sinfo->rtc_scene = slot_handle<typename std::decay<decltype(sinfo->rtc_scene)>::type>(block);
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
  template <typename HandleT, typename IsectT,
            typename = typename std::enable_if<std::is_pointer<HandleT>::value>::type>
  bool intersect(HandleT rtc_scene, int cache_block, const float org[3], const float dir[3],
                 IsectT* isect) const {
    static_assert(sizeof(IsectT) >= sizeof(spray_rt_ray_intersection),
                  "RTCRayIntersection layout (96 B) expected");
    (void)rtc_scene;
    make_ray(org, dir, isect);
    lane_call(spray_rt_lane_intersect1M(lane(), cache_block, isect, 1, sizeof(IsectT)));
    return geom_id(isect) != SPRAY_RT_INVALID_ID;
  }
  template <typename HandleT, typename V, typename IsectT,
            typename = typename std::enable_if<std::is_pointer<HandleT>::value>::type>
  bool intersect(HandleT rtc_scene, int cache_block, const V& org, const float dir[3],
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
  template <typename HandleT, typename RayT,
            typename = typename std::enable_if<std::is_pointer<HandleT>::value>::type>
  bool occluded(HandleT rtc_scene, const float org[3], const float dir[3], RayT* ray) const {
    static_assert(sizeof(RayT) >= 84, "Embree 2 RTCRay layout expected");
    make_ray(org, dir, ray);
    lane_call(spray_rt_lane_occluded1M(lane(), handle_slot(rtc_scene), ray, 1, sizeof(RayT)));
    return geom_id(ray) != SPRAY_RT_INVALID_ID;
  }
  template <typename HandleT, typename V, typename RayT,
            typename = typename std::enable_if<std::is_pointer<HandleT>::value>::type>
  bool occluded(HandleT rtc_scene, const V& org, const V& dir, RayT* ray) const {
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
  template <typename SceneInfoT, typename IsectT>
  void intersect1M(const SceneInfoT& sinfo, IsectT* isects, size_t M) const {
    static_assert(sizeof(IsectT) >= sizeof(spray_rt_ray_intersection),
                  "RTCRayIntersection layout (96 B) expected");
    lane_call(spray_rt_lane_intersect1M(lane(), sinfo.cache_block, isects, M, sizeof(IsectT)));
  }
  template <typename SceneInfoT, typename RayT>
  void occluded1M(const SceneInfoT& sinfo, RayT* rays, size_t M) const {
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

  // Scene::getBsdf (scene.h:213): the domain's material (null when the
  // scene file gives it none, as the reference's Domain::bsdf).
  const Bsdf* getBsdf(int id) const { return domains_[size_t(id)].bsdf; }
  const InsituPartition& getInsituPartition() const { return partition_; }
  bool insitu() const { return insitu_; }
  std::size_t getNumDomains() const { return domains_.size(); }
  const std::vector<Domain>& getDomains() const { return domains_; }
  // Scene::getLights (scene.h:219): the shaders copy it into their own
  // std::vector<Light*> (ooc_shader_pt.h:51)
  const std::vector<Light*>& getLights() const { return lights_; }
  std::size_t getNumLights() const { return lights_.size(); }
  // Scene::getBound (scene.h:82-85): the scene's world bound
  Aabb getBound() const { return Types::makeAabb(bound_); }
  const float* getBoundArray() const { return bound_; }
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
  std::vector<float> boxes_;
  std::vector<Light*> lights_;
  std::vector<std::unique_ptr<Bsdf>> bsdfs_;
  float bound_[6] = {0, 0, 0, 0, 0, 0};
  InsituPartition partition_;
  bool insitu_ = false;
  int cache_block_ = -1;  // the last loaded domain's cache block (scene_ / cache_block_)
  mutable std::shared_mutex mu_;
  mutable std::map<std::thread::id, spray_rt_lane_t> lanes_;
};

}  // namespace spray_amd
