// Mock ooc drain over the SceneT drop-in (include/spray_scene.hpp) from N
// OpenMP threads, with the reference's call shapes (ooc_tcontext.inl:28-100,
// ooc_pcontext.h:144-157, ooc_isector.h:116-124):
//
//   #pragma omp single   scene.load(id, &sinfo);
//   every thread:        scene.intersect(sinfo.rtc_scene, sinfo.cache_block,
//                                        r->org, r->dir, &rtc_isect_);
//                        scene.occluded(sinfo.rtc_scene, pos, wi, &rtc_ray_);
//                        scene.intersectDomains(ray_ext);
//
// Every result is checked against the CPU oracle (oracle/oracle.h): domain
// lists bit-exact against or_domain_query, each per-domain closest hit
// (t, u, v, primID, Ng, color, Ns) and occlusion bit-exact against brute
// force over that domain's triangles.  Test infrastructure: built by
// __graft_entry__.build(), run by tests/test_gpu_adapter.py.
//
//   scene_adapter_test <scene.spray> <ply_path> <threads> <cache_size>
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s scene.spray ply_path threads cache_size\n", argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[3]), cache = std::atoi(argv[4]);
  spray_amd::Scene<> scene;
  scene.init(argv[1], argv[2], "", cache, 0, false, 1);
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
  const float light[3] = {0.f, 500.f, 1000.f};

  // per-domain oracle meshes (TriMeshBuffer::load through the host layer)
  std::vector<std::vector<float>> tri(nd);
  std::vector<std::vector<uint32_t>> faces(nd), colors(nd);
  std::vector<std::vector<float>> normals(nd);
  std::vector<float> boxes(6 * size_t(nd));
  for (int d = 0; d < nd; ++d) {
    size_t nv = 0, nf = 0;
    spray_host_domain_mesh(argv[1], argv[2], d, &nv, &nf, nullptr, nullptr, nullptr, nullptr);
    std::vector<float> v(3 * nv);
    faces[d].resize(3 * nf);
    colors[d].resize(nv);
    normals[d].resize(3 * nv);
    spray_host_domain_mesh(argv[1], argv[2], d, &nv, &nf, v.data(), faces[d].data(),
                           colors[d].data(), normals[d].data());
    tri[d].resize(12 * nf);
    or_prep_tris(v.data(), faces[d].data(), nf, tri[d].data());
    std::memcpy(&boxes[6 * size_t(d)], scene.getDomains()[size_t(d)].world_aabb, 24);
  }

  std::atomic<long> bad{0}, nhit{0}, nocc{0}, ncalls{0};
  // domain lists from every thread at once (Isector::isectDomains)
  std::vector<std::vector<int>> lists(n);
  std::vector<int32_t> oids(n * size_t(nd)), ocnt(n);
  std::vector<float> ots(n * size_t(nd));
  or_domain_query(org.data(), dir.data(), n, boxes.data(), nd, nd, oids.data(), ots.data(),
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
  spray_amd::SceneInfo sinfo;
#pragma omp parallel num_threads(T)
  {
    RTCRayIntersection rtc_isect_;
    RTCRay rtc_ray_;
    for (int id = 0; id < nd; ++id) {
#pragma omp single
      scene.load(id, &sinfo);
#pragma omp for schedule(dynamic, 8)
      for (long q = 0; q < long(queue[id].size()); ++q) {
        const long i = queue[id][q];
        const float* o = &org[3 * i];
        const float* d = &dir[3 * i];
        const bool hit = scene.intersect(sinfo.rtc_scene, sinfo.cache_block, o, d, &rtc_isect_);
        ++ncalls;
        float t, u, v;
        uint32_t p;
        or_brute_intersect(tri[id].data(), faces[id].size() / 3, o, d, nullptr, nullptr, 1, &t,
                           &u, &v, &p);
        bool ok = hit == (p != 0xFFFFFFFFu);
        if (ok && hit) {
          uint32_t col;
          float ns[3];
          or_epilogue(faces[id].data(), colors[id].data(), normals[id].data(), &p, &u, &v, 1,
                      &col, ns);
          const float* ng = &tri[id][12 * p + 9];
          ok = rtc_isect_.primID == p && same(rtc_isect_.tfar, t) && same(rtc_isect_.u, u) &&
               same(rtc_isect_.v, v) && rtc_isect_.geomID == 0 && rtc_isect_.color == col;
          for (int k = 0; k < 3; ++k)
            ok = ok && same(rtc_isect_.Ns[k], ns[k]) && same(rtc_isect_.Ng[k], ng[k]);
          // a shadow ray toward the light from the hit, in the same domain
          float ps[3], wi[3];
          for (int k = 0; k < 3; ++k) ps[k] = o[k] + t * d[k];
          float len = 0.f;
          for (int k = 0; k < 3; ++k) {
            wi[k] = light[k] - ps[k];
            len += wi[k] * wi[k];
          }
          len = std::sqrt(len);
          for (int k = 0; k < 3; ++k) wi[k] /= len;
          const bool occ = scene.occluded(sinfo.rtc_scene, ps, wi, &rtc_ray_);
          uint8_t oo;
          or_brute_occluded(tri[id].data(), faces[id].size() / 3, ps, wi, nullptr, nullptr, 1,
                            &oo);
          ok = ok && occ == (oo != 0) && (!occ || rtc_ray_.geomID == 0);
          ++nhit;
          if (occ) ++nocc;
        }
        if (!ok) ++bad;
      }
    }
  }
  std::printf("threads %d cache %d rays %zu domain-list mismatches %ld calls %ld hits %ld "
              "occluded %ld mismatches %ld\n",
              T, cache, n, bad_lists, ncalls.load(), nhit.load(), nocc.load(), bad.load());
  if (bad.load() || nhit.load() < 1000 || nocc.load() == 0 || nocc.load() == nhit.load()) {
    std::printf("FAIL\n");
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
