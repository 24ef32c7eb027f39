// Mock drains over the SceneT drop-in (include/spray_scene.hpp) from N
// OpenMP threads, with the reference's call shapes.  Test infrastructure:
// built by __graft_entry__.build(), run by tests/test_gpu_adapter.py.
//
//   scene_adapter_test <scene.spray> <ply_path> <threads> <cache_size> [mode] [image]
//
// mode "single" (default; ooc_tcontext.inl:28-100, ooc_pcontext.h:144-157,
// ooc_isector.h:116-124): one ray per call, as the reference calls Scene:
//   #pragma omp single   scene.load(id, &sinfo);
//   every thread:        scene.intersect(sinfo.rtc_scene, sinfo.cache_block,
//                                        r->org, r->dir, &rtc_isect_);
//                        scene.occluded(sinfo.rtc_scene, pos, wi, &rtc_ray_);
//                        scene.intersectDomains(ray_ext);
// every result checked against brute force over the domain's triangles.
//
// mode "current": the baseline tracers' scene-less forms (load(id), then
// intersect(org, dir, isect) / occluded(org, dir, ray) on the current
// domain, updateIntersection(isect); baseline_shader_pt.h:110, 139,
// baseline_shader_ao.h:90, baseline_insitu_tracer.inl:653-700).
//
// mode "batched": the same drain as gather -> one stream call -> scatter per
// thread and domain (Scene::intersect1M / occluded1M /
// intersectDomains1M): each thread copies its share of the domain's queue
// into RTCRayIntersection records, makes one call, and checks the results
// in queue order; its shadow rays likewise.  image x image camera rays at
// 1 spp; every result checked against the oracle's canonical BVH of the
// domain (bit-equal to brute force, tests/test_oracle.py).  Prints the
// drain's rate (ray-domain pairs + shadow rays per second, timed apart from
// the checks) and, for comparison, the per-ray form's rate over the first
// queues.
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "ref_mock.h"
#include "spray_scene.hpp"

extern "C" {
#include "oracle.h"
}

namespace {

// the reference's record types (src/render/rays.h; Embree 2 RTCRay)
struct alignas(16) RTCRay {
  float org[3], align0, dir[3], align1, tnear, tfar, time;
  uint32_t mask;
  float Ng[3], align2, u, v;
  uint32_t geomID, primID, instID;
};
static_assert(sizeof(RTCRay) == 96, "RTCRay");
using RTCRayIntersection = spray_rt_ray_intersection;

class DomainList {  // rays.h:57-93
 public:
  void resize(size_t n) { hits_.resize(n); num_ = 0; }
  void reset() { num_ = 0; }
  void push(int id, float t) { hits_.at(num_) = {id, t}; ++num_; }
  size_t getNumHits() const { return num_; }
  int getId(size_t i) const { return hits_[i].id; }
  float getTnear(size_t i) const { return hits_[i].t; }
 private:
  struct Hit { int id; float t; };
  size_t num_ = 0;
  std::vector<Hit> hits_;
};
struct RTCRayExt {  // rays.h:117-170
  float org[3], align0, dir[3], align1, tnear, tfar;
  DomainList* domains;
  void reset(const float* o, const float* d, DomainList* dl) {
    std::memcpy(org, o, 12);
    std::memcpy(dir, d, 12);
    tnear = 0.001f;
    tfar = INFINITY;
    domains = dl;
  }
};

bool same(float a, float b) { return std::memcmp(&a, &b, 4) == 0; }
double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

const float kLight[3] = {0.f, 500.f, 1000.f};

// the point-light shadow ray of a hit (the test's own, same on both sides)
void shadow_ray(const float* o, const float* d, float t, float ps[3], float wi[3]) {
  for (int k = 0; k < 3; ++k) ps[k] = o[k] + t * d[k];
  float len = 0.f;
  for (int k = 0; k < 3; ++k) {
    wi[k] = kLight[k] - ps[k];
    len += wi[k] * wi[k];
  }
  len = std::sqrt(len);
  for (int k = 0; k < 3; ++k) wi[k] /= len;
}

struct Meshes {  // per-domain oracle data (TriMeshBuffer::load through the host layer)
  std::vector<std::vector<float>> tri, normals, verts;
  std::vector<std::vector<uint32_t>> faces, colors;
  std::vector<or_bvh*> bvh;
  std::vector<float> boxes;
  ~Meshes() {
    for (or_bvh* b : bvh)
      if (b) or_bvh_free(b);
  }
};

template <typename SceneT>
void load_meshes(const char* desc, const char* ply, const SceneT& scene, Meshes* m, bool bvh) {
  const int nd = int(scene.getNumDomains());
  m->tri.resize(nd);
  m->verts.resize(nd);
  m->faces.resize(nd);
  m->colors.resize(nd);
  m->normals.resize(nd);
  m->bvh.assign(nd, nullptr);
  m->boxes.resize(6 * size_t(nd));
  for (int d = 0; d < nd; ++d) {
    size_t nv = 0, nf = 0;
    spray_host_domain_mesh(desc, ply, d, &nv, &nf, nullptr, nullptr, nullptr, nullptr);
    m->verts[d].resize(3 * nv);
    m->faces[d].resize(3 * nf);
    m->colors[d].resize(nv);
    m->normals[d].resize(3 * nv);
    spray_host_domain_mesh(desc, ply, d, &nv, &nf, m->verts[d].data(), m->faces[d].data(),
                           m->colors[d].data(), m->normals[d].data());
    m->tri[d].resize(12 * nf);
    or_prep_tris(m->verts[d].data(), m->faces[d].data(), nf, m->tri[d].data());
    if (bvh) m->bvh[d] = or_bvh_build(m->verts[d].data(), m->faces[d].data(), nf);
    const auto& a = scene.getDomains()[size_t(d)].world_aabb;
    for (int k = 0; k < 3; ++k) {
      m->boxes[6 * size_t(d) + size_t(k)] = a.bounds[0][k];
      m->boxes[6 * size_t(d) + 3 + size_t(k)] = a.bounds[1][k];
    }
  }
}

// the closest-hit record of one ray in domain id against the oracle's
// (t, u, v, prim); p == 0xFFFFFFFF: a miss (the record must say so)
bool check_hit(const Meshes& m, int id, const RTCRayIntersection& r, bool hit, float t, float u,
               float v, uint32_t p) {
  bool ok = hit == (p != 0xFFFFFFFFu);
  if (ok && hit) {
    uint32_t col;
    float ns[3];
    or_epilogue(m.faces[id].data(), m.colors[id].data(), m.normals[id].data(), &p, &u, &v, 1,
                &col, ns);
    const float* ng = &m.tri[id][12 * size_t(p) + 9];
    ok = r.primID == p && same(r.tfar, t) && same(r.u, u) && same(r.v, v) && r.geomID == 0 &&
         r.color == col;
    for (int k = 0; k < 3; ++k) ok = ok && same(r.Ns[k], ns[k]) && same(r.Ng[k], ng[k]);
  }
  if (!hit) ok = ok && std::isinf(r.tfar) && r.geomID == SPRAY_RT_INVALID_ID;
  return ok;
}

// mode "single" / "current": one ray per call, brute-force checks
int run_single(const char* desc, const char* ply, int T, int cache, bool current) {
  spray_amd::Scene<> scene;
  scene.init(desc, ply, "", cache, 0, false, 1);
  const int nd = int(scene.getNumDomains());
  const int W = 96, H = 96;
  const float pos[3] = {90.172180f, 84.141418f, 82.480225f}, at[3] = {30.f, 28.649426f, 30.f},
              up[3] = {0.f, 1.f, 0.f};
  float cam[14];
  or_camera_init(pos, at, up, 90.f, W, H, cam);
  const size_t n = size_t(W) * H;
  std::vector<float> org(3 * n), dir(3 * n);
  std::vector<int32_t> pix(n), sam(n);
  or_eye_rays_ooc(cam, W, 1, 0, 0, W, H, org.data(), dir.data(), pix.data(), sam.data());
  Meshes m;
  load_meshes(desc, ply, scene, &m, false);

  std::atomic<long> bad{0}, nhit{0}, nocc{0}, ncalls{0};
  // domain lists from every thread at once (Isector::isectDomains)
  std::vector<std::vector<int>> lists(n);
  std::vector<int32_t> oids(n * size_t(nd)), ocnt(n);
  std::vector<float> ots(n * size_t(nd));
  or_domain_query(org.data(), dir.data(), n, m.boxes.data(), nd, nd, oids.data(), ots.data(),
                  ocnt.data());
#pragma omp parallel for num_threads(T) schedule(dynamic, 32)
  for (long i = 0; i < long(n); ++i) {
    DomainList dl;
    dl.resize(size_t(nd));
    RTCRayExt ext;
    ext.reset(&org[3 * i], &dir[3 * i], &dl);
    scene.intersectDomains(ext);
    bool ok = int(dl.getNumHits()) == ocnt[i];
    for (size_t k = 0; ok && k < dl.getNumHits(); ++k)
      ok = dl.getId(k) == oids[i * nd + k] && same(dl.getTnear(k), ots[i * nd + k]);
    if (!ok) ++bad;
    for (size_t k = 0; k < dl.getNumHits(); ++k) lists[i].push_back(dl.getId(k));
  }
  const long bad_lists = bad.load();
  std::vector<std::vector<long>> queue(nd);
  for (size_t i = 0; i < n; ++i)
    for (int d : lists[i]) queue[d].push_back(long(i));

  // the drains: load in omp single, every thread intersects / occludes
  spray::SceneInfo sinfo;  // the reference's own record (ooc_pcontext.h:83)
#pragma omp parallel num_threads(T)
  {
    RTCRayIntersection rtc_isect_;
    RTCRay rtc_ray_;
    for (int id = 0; id < nd; ++id) {
#pragma omp single
      {
        if (current)
          scene.load(id);
        else
          scene.load(id, &sinfo);
      }
#pragma omp for schedule(dynamic, 8)
      for (long q = 0; q < long(queue[id].size()); ++q) {
        const long i = queue[id][q];
        const float* o = &org[3 * i];
        const float* d = &dir[3 * i];
        bool hit;
        if (current) {
          hit = scene.intersect(o, d, &rtc_isect_);
          if (hit) {  // Scene::updateIntersection recomputes color / Ns in place
            rtc_isect_.color = 0xDEADBEEFu;
            rtc_isect_.Ns[0] = rtc_isect_.Ns[1] = rtc_isect_.Ns[2] = -7.f;
            scene.updateIntersection(&rtc_isect_);
          }
        } else {
          hit = scene.intersect(sinfo.rtc_scene, sinfo.cache_block, o, d, &rtc_isect_);
        }
        ++ncalls;
        float t, u, v;
        uint32_t p;
        or_brute_intersect(m.tri[id].data(), m.faces[id].size() / 3, o, d, nullptr, nullptr, 1,
                           &t, &u, &v, &p);
        bool ok = check_hit(m, id, rtc_isect_, hit, t, u, v, p);
        if (ok && hit) {
          // a shadow ray toward the light from the hit, in the same domain
          float ps[3], wi[3];
          shadow_ray(o, d, t, ps, wi);
          const bool occ = current ? scene.occluded(ps, wi, &rtc_ray_)
                                   : scene.occluded(sinfo.rtc_scene, ps, wi, &rtc_ray_);
          uint8_t oo;
          or_brute_occluded(m.tri[id].data(), m.faces[id].size() / 3, ps, wi, nullptr, nullptr,
                            1, &oo);
          ok = ok && occ == (oo != 0) && (!occ || rtc_ray_.geomID == 0);
          ++nhit;
          if (occ) ++nocc;
        }
        if (!ok) ++bad;
      }
    }
  }
  std::printf("mode %s threads %d cache %d rays %zu domain-list mismatches %ld calls %ld "
              "hits %ld occluded %ld mismatches %ld\n",
              current ? "current" : "single", T, cache, n, bad_lists, ncalls.load(), nhit.load(),
              nocc.load(), bad.load());
  if (bad.load() || nhit.load() < 1000 || nocc.load() == 0 || nocc.load() == nhit.load()) {
    std::printf("FAIL\n");
    return 1;
  }
  std::printf("ok\n");
  return 0;
}

// mode "batched": per thread and domain one gather -> stream call -> scatter
int run_batched(const char* desc, const char* ply, int T, int cache, int img) {
  spray_amd::Scene<> scene;
  scene.init(desc, ply, "", cache, 0, false, 1);
  const int nd = int(scene.getNumDomains());
  const float pos[3] = {90.172180f, 84.141418f, 82.480225f}, at[3] = {30.f, 28.649426f, 30.f},
              up[3] = {0.f, 1.f, 0.f};
  float cam[14];
  or_camera_init(pos, at, up, 90.f, img, img, cam);
  const size_t n = size_t(img) * size_t(img);
  std::vector<float> org(3 * n), dir(3 * n);
  std::vector<int32_t> pix(n), sam(n);
  or_eye_rays_ooc(cam, img, 1, 0, 0, img, img, org.data(), dir.data(), pix.data(), sam.data());
  Meshes m;
  load_meshes(desc, ply, scene, &m, true);

  // domain lists of the whole queue in one call (Isector::isectDomains)
  std::vector<int32_t> ids(n * size_t(nd)), cnt(n), oids(n * size_t(nd)), ocnt(n);
  std::vector<float> ts(n * size_t(nd)), ots(n * size_t(nd));
  scene.intersectDomains1M(org.data(), dir.data(), n, ids.data(), ts.data(), cnt.data(), nd);
  or_domain_query(org.data(), dir.data(), n, m.boxes.data(), nd, nd, oids.data(), ots.data(),
                  ocnt.data());
  long bad_lists = 0;
  for (size_t i = 0; i < n; ++i) {
    bool ok = cnt[i] == ocnt[i];
    for (int k = 0; ok && k < cnt[i]; ++k)
      ok = ids[i * nd + k] == oids[i * nd + k] && same(ts[i * nd + k], ots[i * nd + k]);
    if (!ok) ++bad_lists;
  }
  std::vector<std::vector<long>> queue(nd);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < cnt[i]; ++k) queue[ids[i * nd + k]].push_back(long(i));

  // per (domain, thread) results of the timed drain, checked afterwards
  struct Part {
    std::vector<long> rays;
    std::vector<RTCRayIntersection> isect;
    std::vector<long> src;  // shadow ray -> position in rays
    std::vector<RTCRay> shadow;
  };
  std::vector<std::vector<Part>> parts(nd, std::vector<Part>(T));
  std::atomic<long> npair{0}, nshadow{0}, ncalls{0};
  spray::SceneInfo sinfo;  // the reference's own record (ooc_pcontext.h:83)
  // warm the lanes (first call per thread creates its stream)
  scene.load(0, &sinfo);
#pragma omp parallel num_threads(T)
  {
    RTCRayIntersection w;
    spray_amd::Scene<>::makeRay(&org[0], &dir[0], &w);
    scene.intersect1M(sinfo, &w, 1);
  }
  const double t0 = now();
#pragma omp parallel num_threads(T)
  {
    const int me = omp_get_thread_num();
    for (int id = 0; id < nd; ++id) {
#pragma omp single
      scene.load(id, &sinfo);
      // this thread's share of the queue (omp for static: contiguous)
      const long qn = long(queue[id].size());
      const long b = qn * me / T, e = qn * (me + 1) / T;
      Part& P = parts[id][me];
      if (e > b) {
        P.rays.assign(queue[id].begin() + b, queue[id].begin() + e);
        P.isect.resize(P.rays.size());
        for (size_t k = 0; k < P.rays.size(); ++k)  // gather
          spray_amd::Scene<>::makeRay(&org[3 * P.rays[k]], &dir[3 * P.rays[k]], &P.isect[k]);
        scene.intersect1M(sinfo, P.isect.data(), P.isect.size());
        ++ncalls;
        for (size_t k = 0; k < P.rays.size(); ++k) {  // scatter, queue order: spawn
          const RTCRayIntersection& r = P.isect[k];
          if (r.geomID == SPRAY_RT_INVALID_ID) continue;
          float ps[3], wi[3];
          shadow_ray(&org[3 * P.rays[k]], &dir[3 * P.rays[k]], r.tfar, ps, wi);
          RTCRay s;
          spray_amd::Scene<>::makeRay(ps, wi, &s);
          P.shadow.push_back(s);
          P.src.push_back(long(k));
        }
        if (!P.shadow.empty()) {
          scene.occluded1M(sinfo, P.shadow.data(), P.shadow.size());
          ++ncalls;
        }
        npair += long(P.rays.size());
        nshadow += long(P.shadow.size());
      }
#pragma omp barrier
    }
  }
  const double dt = now() - t0;

  // checks against the oracle's BVH of each domain
  long bad = 0, nhit = 0, nocc = 0;
  for (int id = 0; id < nd; ++id)
    for (int th = 0; th < T; ++th) {
      const Part& P = parts[id][size_t(th)];
      const size_t k = P.rays.size();
      if (!k) continue;
      std::vector<float> o(3 * k), d(3 * k), t(k), u(k), v(k);
      std::vector<uint32_t> p(k);
      for (size_t j = 0; j < k; ++j) {
        std::memcpy(&o[3 * j], &org[3 * P.rays[j]], 12);
        std::memcpy(&d[3 * j], &dir[3 * P.rays[j]], 12);
      }
      or_bvh_intersect(m.bvh[id], o.data(), d.data(), nullptr, nullptr, k, t.data(), u.data(),
                       v.data(), p.data(), nullptr);
      size_t sh = 0;
      for (size_t j = 0; j < k; ++j) {
        const bool hit = P.isect[j].geomID != SPRAY_RT_INVALID_ID;
        if (!check_hit(m, id, P.isect[j], hit, t[j], u[j], v[j], p[j])) ++bad;
        if (hit) {
          ++nhit;
          // the shadow ray this hit spawned, in queue order
          if (sh >= P.src.size() || P.src[sh] != long(j)) {
            ++bad;
            continue;
          }
          float ps[3], wi[3];
          shadow_ray(&o[3 * j], &d[3 * j], t[j], ps, wi);
          uint8_t oo;
          or_bvh_occluded(m.bvh[id], ps, wi, nullptr, nullptr, 1, &oo, nullptr);
          const bool occ = P.shadow[sh].geomID != SPRAY_RT_INVALID_ID;
          if (occ != (oo != 0) || (occ && P.shadow[sh].geomID != 0)) ++bad;
          if (occ) ++nocc;
          ++sh;
        }
      }
      if (sh != P.src.size()) ++bad;
    }
  const double rate = double(npair.load() + nshadow.load()) / dt / 1e6;

  // the CPU baseline of the same drain: the oracle's canonical BVH (C,
  // OpenMP over T threads) on every queue's rays and the shadow rays of its
  // hits, gathers included -- the reference's Embree drain, restated
  long cpu_rays = 0;
  double cpu_s = 0.0;
  {
    omp_set_num_threads(T);
    const double c0 = now();
    for (int id = 0; id < nd; ++id) {
      const size_t k = queue[id].size();
      if (!k) continue;
      std::vector<float> o(3 * k), d(3 * k), t(k), u(k), v(k);
      std::vector<uint32_t> p(k);
      for (size_t j = 0; j < k; ++j) {
        std::memcpy(&o[3 * j], &org[3 * queue[id][j]], 12);
        std::memcpy(&d[3 * j], &dir[3 * queue[id][j]], 12);
      }
      or_bvh_intersect(m.bvh[id], o.data(), d.data(), nullptr, nullptr, k, t.data(), u.data(),
                       v.data(), p.data(), nullptr);
      std::vector<float> so, sd;
      for (size_t j = 0; j < k; ++j) {
        if (p[j] == 0xFFFFFFFFu) continue;
        float ps[3], wi[3];
        shadow_ray(&o[3 * j], &d[3 * j], t[j], ps, wi);
        so.insert(so.end(), ps, ps + 3);
        sd.insert(sd.end(), wi, wi + 3);
      }
      std::vector<uint8_t> oo(so.size() / 3 + 1);
      if (!so.empty())
        or_bvh_occluded(m.bvh[id], so.data(), sd.data(), nullptr, nullptr, so.size() / 3,
                        oo.data(), nullptr);
      cpu_rays += long(k + so.size() / 3);
    }
    cpu_s = now() - c0;
  }

  // the per-ray form on the first queues (same calls as mode "single"), timed
  long single_rays = 0;
  double single_s = 0.0;
  {
    const double s0 = now();
    for (int id = 0; id < nd && single_rays < 40000; ++id) {
      scene.load(id, &sinfo);
#pragma omp parallel for num_threads(T) schedule(dynamic, 64)
      for (long q = 0; q < long(queue[id].size()); ++q) {
        RTCRayIntersection r;
        const long i = queue[id][q];
        scene.intersect(sinfo.rtc_scene, sinfo.cache_block, &org[3 * i], &dir[3 * i], &r);
      }
      single_rays += long(queue[id].size());
    }
    single_s = now() - s0;
  }
  std::printf("mode batched threads %d cache %d rays %zu pairs %ld shadow %ld calls %ld "
              "drain_s %.4f batched_Mrays_s %.2f per_ray_Mrays_s %.3f (%ld rays) "
              "oracle_Mrays_s %.2f (%d threads) "
              "domain-list mismatches %ld hits %ld occluded %ld mismatches %ld\n",
              T, cache, n, npair.load(), nshadow.load(), ncalls.load(), dt, rate,
              single_rays / single_s / 1e6, single_rays, cpu_rays / cpu_s / 1e6, T, bad_lists,
              nhit, nocc, bad);
  if (bad || bad_lists || nhit < 1000 || nocc == 0 || nocc == nhit) {
    std::printf("FAIL\n");
    return 1;
  }
  std::printf("ok\n");
  return 0;
}

// the scene file's lights, read independently of the engine (the checker's
// view; SceneLoader::parseLight, scene_loader.cc:205-231)
std::vector<or_light> read_lights(const char* desc) {
  std::vector<or_light> out;
  std::ifstream in(desc);
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string tag, kind;
    if (!(ss >> tag) || tag != "light" || !(ss >> kind)) continue;
    or_light L{};
    if (kind == "point") {
      L.type = OR_LIGHT_POINT;
      ss >> L.pos[0] >> L.pos[1] >> L.pos[2];
    } else {
      L.type = OR_LIGHT_HEMISPHERE;
    }
    ss >> L.radiance[0] >> L.radiance[1] >> L.radiance[2];
    out.push_back(L);
  }
  return out;
}

bool same_vec(const float* a, const float* b) { return std::memcmp(a, b, 12) == 0; }

// mode "shade": the reference's application types through the adapter
// (spray_amd::Scene<spray::RefTypes>, tests/cpp/ref_mock.h): getBound() as
// the app's Aabb, buildWbvh(), the in-situ partition's getDomains(rank),
// getLights() as std::vector<Light*> and getBsdf(id) as const Bsdf*, used by
// a ShaderPt written with the reference's expressions inside the batched
// drain -- every shadow and continuation ray it spawns checked bit for bit
// against the oracle's ShaderPt (or_shade), every shadow's occlusion against
// the oracle's BVH.
int run_shade(const char* desc, const char* ply, int T, int cache, int img) {
  typedef spray_amd::Scene<spray::RefTypes> SceneT;
  SceneT scene;
  const int kRanks = 4;
  scene.init(desc, ply, "", cache, 0, true, kRanks);
  scene.buildWbvh();  // SprayRenderer::init (spray_renderer.inl:47)
  const int nd = int(scene.getNumDomains());
  long bad = 0;

  // getBound (spray_renderer.inl:96): the app's Aabb, the union of the boxes
  spray::Aabb aabb = scene.getBound();
  for (int k = 0; k < 3; ++k) {
    float lo = INFINITY, hi = -INFINITY;
    for (const auto& d : scene.getDomains()) {
      lo = std::min(lo, d.world_aabb.bounds[0][k]);
      hi = std::max(hi, d.world_aabb.bounds[1][k]);
    }
    if (!same(aabb.bounds[0][k], lo) || !same(aabb.bounds[1][k], hi)) ++bad;
  }
  // the in-situ contexts' view of the partition (insitu_tcontext.inl:98)
  const spray_amd::InsituPartition* partition_ = &scene.getInsituPartition();
  std::vector<float> boxes(6 * size_t(nd));
  for (int d = 0; d < nd; ++d)
    for (int k = 0; k < 3; ++k) {
      boxes[6 * size_t(d) + size_t(k)] = scene.getDomains()[size_t(d)].world_aabb.bounds[0][k];
      boxes[6 * size_t(d) + 3 + size_t(k)] = scene.getDomains()[size_t(d)].world_aabb.bounds[1][k];
    }
  std::vector<int> owner(static_cast<size_t>(nd));
  const float bnd[6] = {aabb.bounds[0].x, aabb.bounds[0].y, aabb.bounds[0].z,
                        aabb.bounds[1].x, aabb.bounds[1].y, aabb.bounds[1].z};
  spray_rt_insitu_partition(boxes.data(), nd, bnd, kRanks, owner.data());
  int listed = 0;
  for (int rank = 0; rank < kRanks; ++rank) {
    const auto& ids = partition_->getDomains(rank);
    for (int id : ids) {
      ++listed;
      if (partition_->rank(id) != rank || owner[size_t(id)] != rank) ++bad;
    }
  }
  if (listed != nd || partition_->getNumDomains() != nd) ++bad;

  // lights and materials as the app's own classes
  const std::vector<or_light> ref_lights = read_lights(desc);
  std::vector<spray::Light*> lights_ = scene.getLights();
  if (lights_.size() != ref_lights.size()) ++bad;
  for (size_t l = 0; l < lights_.size() && l < ref_lights.size(); ++l)
    if (lights_[l]->isAreaLight() != (ref_lights[l].type == OR_LIGHT_HEMISPHERE)) ++bad;
  for (int d = 0; d < nd; ++d) {
    const spray::Bsdf* b = scene.getBsdf(d);
    if (!b || b->isDelta() || !dynamic_cast<const spray::DiffuseBsdf*>(b)) ++bad;
  }
  const long bad_scene = bad;

  spray::ooc::ShaderPt<SceneT>::Config cfg{2, 2, glm::vec3(0.4f, 0.4f, 0.4f), 10.0f};
  spray::ooc::ShaderPt<SceneT> shader;
  shader.init(cfg, &scene);
  or_shader P{};
  P.shader = OR_SHADER_PT;
  P.bounces = cfg.bounces;
  P.samples = cfg.ao_samples;
  P.nlights = int(ref_lights.size());
  for (int k = 0; k < 3; ++k) P.ks[k] = cfg.ks[k];
  P.shininess = cfg.shininess;
  for (size_t l = 0; l < ref_lights.size() && l < OR_MAX_LIGHTS; ++l) P.lights[l] = ref_lights[l];
  const int ns = or_shadow_slots(&P);

  // camera at the scene, image x image rays at 1 spp
  float c[3], e[3];
  for (int k = 0; k < 3; ++k) {
    c[k] = (aabb.bounds[0][k] + aabb.bounds[1][k]) * 0.5f;
    e[k] = aabb.bounds[1][k] - aabb.bounds[0][k];
  }
  const float pos[3] = {c[0] + 1.1f * e[0], c[1] + 0.9f * e[1], c[2] + 1.2f * e[2]};
  const float up[3] = {0.f, 1.f, 0.f};
  float cam[14];
  or_camera_init(pos, c, up, 60.f, img, img, cam);
  const size_t n = size_t(img) * size_t(img);
  std::vector<float> org(3 * n), dir(3 * n);
  std::vector<int32_t> pix(n), sam(n);
  or_eye_rays_ooc(cam, img, 1, 0, 0, img, img, org.data(), dir.data(), pix.data(), sam.data());
  Meshes m;
  load_meshes(desc, ply, scene, &m, true);
  std::vector<int32_t> ids(n * size_t(nd)), cnt(n);
  std::vector<float> ts(n * size_t(nd));
  scene.intersectDomains1M(org.data(), dir.data(), n, ids.data(), ts.data(), cnt.data(), nd);
  std::vector<std::vector<long>> queue(nd);
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < cnt[i]; ++k) queue[ids[i * nd + k]].push_back(long(i));

  struct Part {
    std::vector<long> rays;
    std::vector<RTCRayIntersection> isect;
    std::vector<spray::ooc::Ray> shadows, next;
    std::vector<int> nshadow, nnext;  // per hit, in queue order
    std::vector<RTCRay> srays;
  };
  std::vector<std::vector<Part>> parts(nd, std::vector<Part>(T));
  spray::SceneInfo sinfo;  // the reference's own record (ooc_pcontext.h:83)
#pragma omp parallel num_threads(T)
  {
    const int me = omp_get_thread_num();
    for (int id = 0; id < nd; ++id) {
#pragma omp single
      scene.load(id, &sinfo);
      const long qn = long(queue[id].size());
      const long b = qn * me / T, e2 = qn * (me + 1) / T;
      Part& Q = parts[id][me];
      if (e2 > b) {
        Q.rays.assign(queue[id].begin() + b, queue[id].begin() + e2);
        Q.isect.resize(Q.rays.size());
        for (size_t k = 0; k < Q.rays.size(); ++k)
          SceneT::makeRay(&org[3 * Q.rays[k]], &dir[3 * Q.rays[k]], &Q.isect[k]);
        scene.intersect1M(sinfo, Q.isect.data(), Q.isect.size());
        for (size_t k = 0; k < Q.rays.size(); ++k) {  // procRads: shade every hit
          const RTCRayIntersection& r = Q.isect[k];
          if (r.geomID == SPRAY_RT_INVALID_ID) continue;
          spray::ooc::Ray rin{};
          std::memcpy(rin.org, &org[3 * Q.rays[k]], 12);
          std::memcpy(rin.dir, &dir[3 * Q.rays[k]], 12);
          rin.w[0] = rin.w[1] = rin.w[2] = 1.0f;
          rin.pixid = pix[size_t(Q.rays[k])];
          rin.samid = sam[size_t(Q.rays[k])];
          const size_t s0 = Q.shadows.size(), n0 = Q.next.size();
          shader(id, rin, r, &Q.shadows, &Q.next, 0);
          Q.nshadow.push_back(int(Q.shadows.size() - s0));
          Q.nnext.push_back(int(Q.next.size() - n0));
        }
        Q.srays.resize(Q.shadows.size());
        for (size_t k = 0; k < Q.shadows.size(); ++k)
          SceneT::makeRay(Q.shadows[k].org, Q.shadows[k].dir, &Q.srays[k]);
        if (!Q.srays.empty()) scene.occluded1M(sinfo, Q.srays.data(), Q.srays.size());
      }
#pragma omp barrier
    }
  }

  // checks: the oracle's ShaderPt over the same hit records, per part
  long nhit = 0, nshadow = 0, nnext = 0, nocc = 0;
  for (int id = 0; id < nd; ++id)
    for (int th = 0; th < T; ++th) {
      const Part& Q = parts[id][size_t(th)];
      std::vector<float> o, d, w;
      std::vector<or_hit> h;
      std::vector<int32_t> hp, hs;
      for (size_t k = 0; k < Q.rays.size(); ++k) {
        const RTCRayIntersection& r = Q.isect[k];
        if (r.geomID == SPRAY_RT_INVALID_ID) continue;
        or_hit x{};
        x.t = r.tfar;
        x.u = r.u;
        x.v = r.v;
        x.prim = r.primID;
        std::memcpy(x.ng, r.Ng, 12);
        x.color = r.color;
        std::memcpy(x.ns, r.Ns, 12);
        x.domain = id;
        h.push_back(x);
        o.insert(o.end(), &org[3 * Q.rays[k]], &org[3 * Q.rays[k]] + 3);
        d.insert(d.end(), &dir[3 * Q.rays[k]], &dir[3 * Q.rays[k]] + 3);
        hp.push_back(pix[size_t(Q.rays[k])]);
        hs.push_back(sam[size_t(Q.rays[k])]);
      }
      const size_t nh = h.size();
      if (nh != Q.nshadow.size()) {
        ++bad;
        continue;
      }
      if (!nh) continue;
      w.assign(3 * nh, 1.0f);
      std::vector<uint8_t> valid(nh, 1), svalid(nh * size_t(ns));
      std::vector<float> so(3 * nh * size_t(ns)), sd(so.size()), sw(so.size());
      if (or_shade(&P, nullptr, 0, 0, o.data(), d.data(), h.data(), w.data(), valid.data(),
                   hp.data(), hs.data(), nh, so.data(), sd.data(), sw.data(), svalid.data()))
        ++bad;
      size_t sj = 0, nj = 0;
      for (size_t j = 0; j < nh; ++j) {
        ++nhit;
        int got = 0;
        for (int k = 0; k < ns; ++k) {
          const size_t slot = j * size_t(ns) + size_t(k);
          if (!svalid[slot]) continue;
          ++got;
          if (sj >= Q.shadows.size()) {
            ++bad;
            continue;
          }
          const spray::ooc::Ray& sh = Q.shadows[sj];
          if (!same_vec(sh.org, &so[3 * slot]) || !same_vec(sh.dir, &sd[3 * slot]) ||
              !same_vec(sh.w, &sw[3 * slot]))
            ++bad;
          uint8_t oo;
          or_bvh_occluded(m.bvh[id], sh.org, sh.dir, nullptr, nullptr, 1, &oo, nullptr);
          const bool occ = Q.srays[sj].geomID != SPRAY_RT_INVALID_ID;
          if (occ != (oo != 0) || (occ && Q.srays[sj].geomID != 0)) ++bad;
          if (occ) ++nocc;
          ++sj;
          ++nshadow;
        }
        if (got != Q.nshadow[j]) ++bad;
        if (int(valid[j]) != Q.nnext[j]) ++bad;
        if (valid[j]) {
          const spray::ooc::Ray& nx = Q.next[nj++];
          if (!same_vec(nx.org, &o[3 * j]) || !same_vec(nx.dir, &d[3 * j]) ||
              !same_vec(nx.w, &w[3 * j]) || nx.depth != 1)
            ++bad;
          ++nnext;
        }
      }
    }
  std::printf("mode shade threads %d cache %d rays %zu lights %zu scene-interface mismatches %ld "
              "hits %ld shadows %ld next %ld occluded %ld mismatches %ld\n",
              T, cache, n, lights_.size(), bad_scene, nhit, nshadow, nnext, nocc, bad);
  if (bad || nhit < 500 || nshadow < 500 || nnext < 500 || nocc == 0) {
    std::printf("FAIL\n");
    return 1;
  }
  std::printf("ok\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr,
                 "usage: %s scene.spray ply_path threads cache_size [single|current|batched|shade] "
                 "[image]\n",
                 argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[3]), cache = std::atoi(argv[4]);
  const std::string mode = argc > 5 ? argv[5] : "single";
  try {
    if (mode == "batched") return run_batched(argv[1], argv[2], T, cache,
                                              argc > 6 ? std::atoi(argv[6]) : 512);
    if (mode == "shade") return run_shade(argv[1], argv[2], T, cache,
                                          argc > 6 ? std::atoi(argv[6]) : 256);
    return run_single(argv[1], argv[2], T, cache, mode == "current");
  } catch (const std::exception& e) {
    std::printf("FAIL exception: %s\n", e.what());
    return 1;
  }
}
