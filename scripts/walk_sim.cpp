// walk_sim.cpp -- CPU model of the wave-level execution of the GPU walks
// (research tool for scripts/walk_sim.py, not part of the product).
//
// The device kernels' traversal loops re-run in lockstep per 64-lane wave
// on the engine's own host-built trees (bvh_build.cpp: the canonical BVH2
// and its 4-wide quantized collapse), counting what bounds a latency- or
// divergence-bound walk: the wave-level loop iterations (each one dependent
// node or triangle fetch round trip) and the lanes active in each (SIMD lane
// utilisation).  Arithmetic is plain float (the conservative culling
// margins of rt_device.h are left out), so the counts model the walks, not
// their bits.
//
//   per-lane any hit (AO rays): occluded_tree_q4 (rt_device.h), the while-
//   while walk over QNode4s, inside scene_ray's loop over the ray's domains;
//   packet walk (camera / shadow rays): trace_tree_packet over BvhNodes,
//   inside scene_ray_packet's loop over the union of the lanes' domains.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "bvh_build.h"
#include "rt_common.h"

using namespace spray_rt;

namespace {

constexpr float kInf = INFINITY;
constexpr int32_t kNone = INT32_MAX;

struct Dom {
  BvhImage img;
  std::vector<QNode4> q4;
  QGrid grid{};
  float box[6];
  bool ok = false;
};

struct Scene {
  std::vector<Dom> d;
};

struct Ray {
  float o[3], d[3], inv[3];
};

Ray make_ray(const float* o, const float* d) {
  Ray r;
  for (int k = 0; k < 3; ++k) {
    r.o[k] = o[k];
    r.d[k] = d[k];
    const float dd = std::fabs(d[k]) < 1e-20f ? std::copysign(1e-20f, d[k]) : d[k];
    r.inv[k] = 1.0f / dd;
  }
  return r;
}

bool slab(const Ray& r, const float* lo, const float* hi, float tnear, float tfar, float* te) {
  float t0 = tnear, t1 = tfar;
  for (int k = 0; k < 3; ++k) {
    float a = (lo[k] - r.o[k]) * r.inv[k], b = (hi[k] - r.o[k]) * r.inv[k];
    if (a > b) std::swap(a, b);
    t0 = std::max(t0, a);
    t1 = std::min(t1, b);
  }
  *te = t0;
  return t0 <= t1;
}

bool tri_test(const Ray& r, const float* x, float tnear, float* t) {
  // x: v0 xyz, e1 xyz, e2 xyz, Ng xyz (e1 = v0 - v1, e2 = v2 - v0)
  const float cx = x[0] - r.o[0], cy = x[1] - r.o[1], cz = x[2] - r.o[2];
  const float rx = r.d[1] * cz - r.d[2] * cy, ry = r.d[2] * cx - r.d[0] * cz,
              rz = r.d[0] * cy - r.d[1] * cx;
  const float den = x[9] * r.d[0] + x[10] * r.d[1] + x[11] * r.d[2];
  const float ad = std::fabs(den);
  float U = rx * x[6] + ry * x[7] + rz * x[8];
  float V = rx * x[3] + ry * x[4] + rz * x[5];
  float T = x[9] * cx + x[10] * cy + x[11] * cz;
  if (den < 0) {
    U = -U;
    V = -V;
    T = -T;
  }
  if (!(den != 0 && U >= 0 && V >= 0 && U + V <= ad)) return false;
  *t = T / ad;
  return *t > tnear;
}

void q4_box(const Dom& D, const QNode4& n, int c, float lo[3], float hi[3]) {
  for (int j = 0; j < 3; ++j) {
    lo[j] = D.grid.base[j] + float(n.q[6 * c + j]) * D.grid.scale[j];
    hi[j] = D.grid.base[j] + float(n.q[6 * c + 3 + j]) * D.grid.scale[j];
  }
}

// ---- per-lane any hit: one lane's occluded_tree_q4 state ----
struct Lane {
  Ray r;
  const Dom* D = nullptr;
  std::vector<int32_t> stk;
  int32_t cur = kNone, leaf = kNone;
  bool active = false;  // inside the current occluded_tree_q4 call
  bool hit = false;
};

int32_t pop(Lane& L) {
  if (L.stk.empty()) return kNone;
  const int32_t v = L.stk.back();
  L.stk.pop_back();
  return v;
}

// one node step of the while loop for lane L (its cur >= 0)
void node_step(Lane& L) {
  const QNode4& n = L.D->q4[size_t(L.cur)];
  int32_t next = kNone;
  float tn = kInf;
  for (int c = 0; c < 4; ++c) {
    if (n.child[c] == kNoChild) continue;
    float lo[3], hi[3], te;
    q4_box(*L.D, n, c, lo, hi);
    if (!slab(L.r, lo, hi, kRayEpsilon, kInf, &te)) continue;
    if (next == kNone || te < tn) {
      if (next != kNone) L.stk.push_back(next);
      next = n.child[c];
      tn = te;
    } else {
      L.stk.push_back(n.child[c]);
    }
  }
  L.cur = next != kNone ? next : pop(L);
  if (L.cur < 0 && L.cur != kNone && L.leaf == kNone) {
    L.leaf = L.cur;
    L.cur = pop(L);
  }
}

int g_redistribute = 0;

}  // namespace

extern "C" {

void ws_set_mode(int redistribute) { g_redistribute = redistribute; }

void* ws_scene_create(int n) {
  Scene* s = new Scene;
  s->d.resize(size_t(n));
  return s;
}
void ws_scene_free(void* s) { delete static_cast<Scene*>(s); }

int ws_set_domain(void* sp, int id, const float* v, size_t nv, const uint32_t* f, size_t nf,
                  const float* box) {
  Dom& D = static_cast<Scene*>(sp)->d[size_t(id)];
  if (!build_bvh(v, nv, f, nf, &D.img)) return -1;
  int bound = 0;
  if (!quantize_nodes4(D.img.nodes, &D.grid, &D.q4, &bound)) return -2;
  std::memcpy(D.box, box, 24);
  D.ok = true;
  return bound;
}

// Per-lane any hit, waves of 64 consecutive rays.  lists: ids[i * maxhits
// + k], k < cnt[i] (the sorted domain list).  out (per wave, 6 counters):
// node-loop iterations, lane node steps, leaf-loop iterations (triangle
// tests, max over lanes per leaf phase), lane triangle tests, outer domain
// iterations, rays occluded.  occ[i] written.
void ws_lane_ah(void* sp, const float* org, const float* dir, size_t n, const int32_t* ids,
                const int32_t* cnt, int maxhits, long long* out, uint8_t* occ) {
  const Scene& S = *static_cast<Scene*>(sp);
  const size_t nw = (n + 63) / 64;
#pragma omp parallel for schedule(dynamic, 16)
  for (long w = 0; w < long(nw); ++w) {
    long long c[6] = {0, 0, 0, 0, 0, 0};
    Lane L[64];
    const size_t i0 = size_t(w) * 64;
    const int nl = int(std::min<size_t>(64, n - i0));
    int maxd = 0;
    for (int l = 0; l < nl; ++l) {
      L[l].r = make_ray(org + 3 * (i0 + l), dir + 3 * (i0 + l));
      maxd = std::max(maxd, int(cnt[i0 + l]));
    }
    for (int k = 0; k < maxd; ++k) {  // scene_ray's domain loop, lockstep
      bool any = false;
      for (int l = 0; l < nl; ++l) {
        Lane& A = L[l];
        A.active = !A.hit && k < cnt[i0 + l];
        if (!A.active) continue;
        any = true;
        A.D = &S.d[size_t(ids[(i0 + l) * size_t(maxhits) + k])];
        A.stk.clear();
        A.cur = A.D->q4.empty() ? kNone : 0;
        A.leaf = kNone;
      }
      if (!any) break;
      ++c[4];
      for (;;) {  // occluded_tree_q4's outer loop
        // node while loop: lanes with cur an inner node; break when every
        // looping lane holds a leaf
        for (;;) {
          bool ran[64] = {false};
          int looping = 0;
          for (int l = 0; l < nl; ++l) {
            Lane& A = L[l];
            ran[l] = A.active && A.cur >= 0 && A.cur != kNone;
            looping += ran[l];
          }
          if (!looping) break;
          ++c[0];
          for (int l = 0; l < nl; ++l)
            if (ran[l]) {
              node_step(L[l]);
              ++c[1];
            }
          // __ballot(leaf == kNone) over the lanes that executed this step
          int noleaf = 0;
          for (int l = 0; l < nl; ++l)
            if (ran[l] && L[l].leaf == kNone) ++noleaf;
          if (noleaf == 0) break;
        }
        // leaf loop
        if (g_redistribute) {
          // every parked leaf (and a second leaf the walk stopped on) as
          // (lane, triangle) tasks spread over the wave's 64 lanes
          long long T = 0;
          for (int l = 0; l < nl; ++l) {
            Lane& A = L[l];
            if (!A.active || A.leaf == kNone) continue;
            int32_t lv[2] = {A.leaf, kNone};
            A.leaf = kNone;
            if (A.cur < 0 && A.cur != kNone) {
              lv[1] = A.cur;
              A.cur = pop(A);
            }
            for (int k = 0; k < 2; ++k) {
              if (lv[k] == kNone) continue;
              const uint32_t enc = ~uint32_t(lv[k]);
              const uint32_t first = enc >> 2, cnt4 = (enc & 3u) + 1u;
              for (uint32_t q = 0; q < cnt4; ++q) {
                float t;
                ++T;
                if (tri_test(A.r, &A.D->img.tris[12 * size_t(first + q)], kRayEpsilon, &t))
                  A.hit = true;
              }
            }
            if (A.hit) {
              A.active = false;
            } else if (A.cur < 0 && A.cur != kNone) {  // popped a leaf: parked for the next phase
              A.leaf = A.cur;
              A.cur = pop(A);
            }
          }
          c[2] += (T + 63) / 64;
          c[3] += T;
        }
        for (;;) {
          if (g_redistribute) break;
          int maxt = 0, any_leaf = 0;
          for (int l = 0; l < nl; ++l) {
            Lane& A = L[l];
            if (!A.active || A.leaf == kNone) continue;
            ++any_leaf;
            const uint32_t enc = ~uint32_t(A.leaf);
            const uint32_t first = enc >> 2, cnt4 = (enc & 3u) + 1u;
            int tested = 0;
            for (uint32_t q = 0; q < cnt4; ++q) {
              float t;
              ++tested;
              if (tri_test(A.r, &A.D->img.tris[12 * size_t(first + q)], kRayEpsilon, &t)) {
                A.hit = true;
                break;
              }
            }
            c[3] += tested;
            maxt = std::max(maxt, tested);
            if (A.hit) {
              A.active = false;  // returns true
              continue;
            }
            A.leaf = kNone;
            if (A.cur < 0 && A.cur != kNone) {
              A.leaf = A.cur;
              A.cur = pop(A);
            }
          }
          if (!any_leaf) break;
          c[2] += maxt;
        }
        bool more = false;
        for (int l = 0; l < nl; ++l) {
          Lane& A = L[l];
          if (!A.active) continue;
          if (A.cur == kNone) {
            A.active = false;  // returns false
          } else {
            more = true;
          }
        }
        if (!more) break;
      }
    }
    for (int l = 0; l < nl; ++l) {
      occ[i0 + l] = L[l].hit ? 1 : 0;
      c[5] += L[l].hit ? 1 : 0;
    }
    for (int k = 0; k < 6; ++k) out[6 * size_t(w) + k] = c[k];
  }
}

// The same any hit as one state machine per lane: a lane that finishes a
// domain moves on to the next one of its list inside the walk's loops (no
// per-domain wave barrier), leaf triangles are spread over the wave, and --
// refill != 0 -- a lane whose ray is done takes the next ray of the wave's
// chunk of `chunk` rays (a refill needs the new ray's domain list: counted
// as refill rounds, the wave iterations in which some lane refilled).
// refill 1: at once, inside the node loop; refill R >= 2: only between
// phases (after a triangle phase), once at least R lanes are idle.
// out (per wave, 8 counters): node iterations, lane node steps, triangle
// iterations (spread), lane triangle tests, refill rounds, refills, triangle
// iterations with per-lane leaf tests (max per lane per phase), 0.
void ws_lane_ah2(void* sp, const float* org, const float* dir, size_t n, const int32_t* ids,
                 const int32_t* cnt, int maxhits, int chunk, int refill, long long* out,
                 uint8_t* occ) {
  const Scene& S = *static_cast<Scene*>(sp);
  const size_t nw = (n + size_t(chunk) - 1) / size_t(chunk);
#pragma omp parallel for schedule(dynamic, 4)
  for (long w = 0; w < long(nw); ++w) {
    long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    Lane L[64];
    int ray[64], kk[64];
    const bool at_once = refill == 1;
    const size_t i0 = size_t(w) * size_t(chunk);
    const size_t i1 = std::min(n, i0 + size_t(chunk));
    size_t next = i0;
    // a lane starts domain k of its ray (or finishes the ray)
    auto start_domain = [&](int l) {
      Lane& A = L[l];
      const size_t i = size_t(ray[l]);
      while (kk[l] < cnt[i]) {
        A.D = &S.d[size_t(ids[i * size_t(maxhits) + kk[l]])];
        A.stk.clear();
        A.leaf = kNone;
        A.cur = A.D->q4.empty() ? kNone : 0;
        if (A.cur != kNone) return true;
        ++kk[l];
      }
      return false;
    };
    auto take_ray = [&](int l) {
      Lane& A = L[l];
      while (next < i1) {
        ray[l] = int(next++);
        kk[l] = 0;
        A.r = make_ray(org + 3 * size_t(ray[l]), dir + 3 * size_t(ray[l]));
        A.hit = false;
        A.active = true;
        if (start_domain(l)) return true;
        occ[size_t(ray[l])] = 0;
      }
      A.active = false;
      return false;
    };
    // a lane whose walk of the current domain ended without a hit
    auto domain_done = [&](int l) {
      ++kk[l];
      if (start_domain(l)) return 0;
      occ[size_t(ray[l])] = 0;
      L[l].active = false;
      return 1;  // ray done
    };
    for (int l = 0; l < 64; ++l) {
      L[l].active = false;
      if (next < i1) take_ray(l);
    }
    for (;;) {
      // node loop
      for (;;) {
        bool ran[64] = {false};
        int looping = 0;
        for (int l = 0; l < 64; ++l) {
          ran[l] = L[l].active && L[l].cur >= 0 && L[l].cur != kNone;
          looping += ran[l];
        }
        if (!looping) break;
        ++c[0];
        int refilled = 0;
        for (int l = 0; l < 64; ++l) {
          if (!ran[l]) continue;
          node_step(L[l]);
          ++c[1];
          if (L[l].cur == kNone && L[l].leaf == kNone && domain_done(l) && at_once) {
            refilled += take_ray(l);
          }
        }
        if (refilled) {
          ++c[4];
          c[5] += refilled;
        }
        int noleaf = 0;
        for (int l = 0; l < 64; ++l)
          if (ran[l] && L[l].active && L[l].leaf == kNone) ++noleaf;
        if (noleaf == 0) break;
      }
      // triangle phase, spread over the wave
      long long T = 0;
      int refilled = 0, tmax = 0;
      for (int l = 0; l < 64; ++l) {
        Lane& A = L[l];
        if (!A.active || A.leaf == kNone) continue;
        const long long T0 = T;
        int32_t lv[2] = {A.leaf, kNone};
        A.leaf = kNone;
        if (A.cur < 0 && A.cur != kNone) {
          lv[1] = A.cur;
          A.cur = pop(A);
        }
        for (int k = 0; k < 2; ++k) {
          if (lv[k] == kNone) continue;
          const uint32_t enc = ~uint32_t(lv[k]);
          const uint32_t first = enc >> 2, cnt4 = (enc & 3u) + 1u;
          for (uint32_t q = 0; q < cnt4; ++q) {
            float t;
            ++T;
            if (tri_test(A.r, &A.D->img.tris[12 * size_t(first + q)], kRayEpsilon, &t))
              A.hit = true;
          }
        }
        tmax = std::max(tmax, int(T - T0));
        if (A.hit) {
          occ[size_t(ray[l])] = 1;
          A.active = false;
          if (at_once) refilled += take_ray(l);
        } else if (A.cur < 0 && A.cur != kNone) {
          A.leaf = A.cur;
          A.cur = pop(A);
        } else if (A.cur == kNone && domain_done(l) && at_once) {
          refilled += take_ray(l);
        }
      }
      if (refill >= 2) {  // between phases, once enough lanes are idle
        int idle = 0;
        for (int l = 0; l < 64; ++l) idle += !L[l].active;
        if (idle >= refill || idle == 64)
          for (int l = 0; l < 64 && next < i1; ++l)
            if (!L[l].active) refilled += take_ray(l);
      }
      if (refilled) {
        ++c[4];
        c[5] += refilled;
      }
      c[2] += (T + 63) / 64;
      c[3] += T;
      c[6] += tmax;
      bool any = false;
      for (int l = 0; l < 64; ++l) any |= L[l].active;
      if (!any) break;
    }
    for (int k = 0; k < 8; ++k) out[8 * size_t(w) + k] = c[k];
  }
}

// Packet walk (trace_tree_packet) of waves of `packet` consecutive rays
// over the union of their domain lists (visit order: the first lane with
// work, its next listed domain).  any: occlusion (lanes leave when
// occluded), else closest hit with the running t as the cut.  out (per
// wave, 5 counters): node fetches, leaf fetches, domain visits, lane slab
// tests, lane triangle tests.
void ws_packet(void* sp, int any, const float* org, const float* dir, size_t n,
               const int32_t* ids, const int32_t* cnt, int maxhits, int packet, long long* out) {
  const Scene& S = *static_cast<Scene*>(sp);
  const size_t nw = (n + size_t(packet) - 1) / size_t(packet);
#pragma omp parallel for schedule(dynamic, 16)
  for (long w = 0; w < long(nw); ++w) {
    long long c[5] = {0, 0, 0, 0, 0};
    const size_t i0 = size_t(w) * size_t(packet);
    const int nl = int(std::min<size_t>(size_t(packet), n - i0));
    std::vector<Ray> R(static_cast<size_t>(nl));
    std::vector<float> best(static_cast<size_t>(nl), kInf);
    std::vector<uint8_t> done(static_cast<size_t>(nl), 0);
    std::vector<uint64_t> mask(static_cast<size_t>(nl), 0), mask2(static_cast<size_t>(nl), 0);  // up to 128 domains
    for (int l = 0; l < nl; ++l) {
      R[size_t(l)] = make_ray(org + 3 * (i0 + l), dir + 3 * (i0 + l));
      for (int k = 0; k < cnt[i0 + l]; ++k) {
        const int d = ids[(i0 + l) * size_t(maxhits) + k];
        if (d < 64) mask[size_t(l)] |= 1ull << d; else mask2[size_t(l)] |= 1ull << (d - 64);
      }
    }
    std::vector<int32_t> stk;
    std::vector<uint8_t> act(static_cast<size_t>(nl));
    for (;;) {
      int lead = -1;
      for (int l = 0; l < nl && lead < 0; ++l)
        if ((mask[size_t(l)] | mask2[size_t(l)]) && !(any && done[size_t(l)])) lead = l;
      if (lead < 0) break;
      // the lead lane's next domain in its list
      int d = -1;
      for (int k = 0; k < cnt[i0 + lead] && d < 0; ++k) {
        const int x = ids[(i0 + lead) * size_t(maxhits) + k];
        if (x < 64 ? (mask[size_t(lead)] >> x) & 1 : (mask2[size_t(lead)] >> (x - 64)) & 1)
          d = x;
      }
      int nact = 0;
      for (int l = 0; l < nl; ++l) {
        uint64_t& m = d < 64 ? mask[size_t(l)] : mask2[size_t(l)];
        const uint64_t b = 1ull << (d & 63);
        act[size_t(l)] = (m & b) && !(any && done[size_t(l)]);
        m &= ~b;
        nact += act[size_t(l)];
      }
      if (!nact) continue;
      ++c[2];
      const Dom& D = S.d[size_t(d)];
      if (D.img.nodes.empty()) continue;
      stk.clear();
      int32_t cur = 0;
      for (;;) {
        const BvhNode& nd = D.img.nodes[size_t(cur)];
        ++c[0];
        bool al = false, ar = false;
        int first_both = -1;
        std::vector<uint8_t> hl(static_cast<size_t>(nl)), hr(static_cast<size_t>(nl));
        std::vector<float> tl(static_cast<size_t>(nl)), tr(static_cast<size_t>(nl));
        for (int l = 0; l < nl; ++l) {
          if (!act[size_t(l)]) continue;
          const float cut = any ? kInf : best[size_t(l)];
          hl[size_t(l)] = slab(R[size_t(l)], nd.l_lo, nd.l_hi, kRayEpsilon, cut, &tl[size_t(l)]);
          hr[size_t(l)] = slab(R[size_t(l)], nd.r_lo, nd.r_hi, kRayEpsilon, cut, &tr[size_t(l)]);
          c[3] += 2;
          al |= hl[size_t(l)];
          ar |= hr[size_t(l)];
          if (hl[size_t(l)] && hr[size_t(l)] && first_both < 0) first_both = l;
        }
        const bool lf = first_both < 0 || tl[size_t(first_both)] <= tr[size_t(first_both)];
        int32_t next = kNone;
        for (int k = 0; k < 2; ++k) {
          const bool left = (k == 0) == lf;
          const int32_t ch = left ? nd.left : nd.right;
          if (!(left ? al : ar)) continue;
          if (ch < 0) {
            ++c[1];
            const uint32_t enc = ~uint32_t(ch);
            const uint32_t first = enc >> 2, cn = (enc & 3u) + 1u;
            for (int l = 0; l < nl; ++l) {
              if (!act[size_t(l)] || !(left ? hl[size_t(l)] : hr[size_t(l)])) continue;
              for (uint32_t q = 0; q < cn; ++q) {
                float t;
                ++c[4];
                if (!tri_test(R[size_t(l)], &D.img.tris[12 * size_t(first + q)], kRayEpsilon, &t))
                  continue;
                if (any) {
                  done[size_t(l)] = 1;
                  act[size_t(l)] = 0;
                  break;
                }
                if (t < best[size_t(l)]) best[size_t(l)] = t;
              }
            }
            if (any) {
              bool still = false;
              for (int l = 0; l < nl; ++l) still |= act[size_t(l)] != 0;
              if (!still) break;
            }
          } else if (next == kNone) {
            next = ch;
          } else {
            stk.push_back(ch);
          }
        }
        if (any) {
          bool still = false;
          for (int l = 0; l < nl; ++l) still |= act[size_t(l)] != 0;
          if (!still) break;
        }
        if (next == kNone) {
          if (stk.empty()) break;
          next = stk.back();
          stk.pop_back();
        }
        cur = next;
      }
    }
    for (int k = 0; k < 5; ++k) out[5 * size_t(w) + k] = c[k];
  }
}

}  // extern "C"
