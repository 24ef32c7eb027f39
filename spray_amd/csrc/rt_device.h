// rt_device.h -- device-side building blocks shared by the gfx950 kernels
// (rt_kernels.hip, ooc_kernels.hip): ray / box / triangle tests, BVH2
// traversal of one domain tree, the updateIntersection epilogue, the
// top-level domain mask and the point-light shadow spawn.
//
// Every translation unit is compiled with -ffp-contract=off: each fused
// multiply-add here is an explicit fmaf(), so t/u/v/Ng are bit-identical to
// the CPU oracle (oracle/oracle.c) and across kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "rt_common.h"
#include "rt_kernels.h"
#include "spray_rt.h"

namespace spray_rt {
namespace {

constexpr float kInf = __builtin_inff();
constexpr int32_t kNone = INT_MAX;
constexpr int32_t kNoChildRef = INT32_MIN;  // empty child (bvh_build.h kNoChild)

inline unsigned grid_for(size_t M) { return unsigned((M + kBlock - 1) / kBlock); }

// Pointers read out of the slot table are generic; re-qualify them as global
// so the loads are global_load_* (not flat_*, which also ticks lgkmcnt).
#define GAS __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const GAS T* gptr(const T* p) {
  return (const GAS T*)(p);
}
typedef float v4f __attribute__((ext_vector_type(4)));
// 16-B global load of element i of a float4 array
__device__ __forceinline__ float4 ld4(const void* base, size_t i) {
  const v4f v = reinterpret_cast<const GAS v4f*>(gptr(base))[i];
  return make_float4(v.x, v.y, v.z, v.w);
}

// Node / triangle fetch of the per-lane walks: each lane loads its own 16-B
// pieces through the vector memory path (the packet walks fetch through the
// scalar data cache instead, trace_tree_packet).
#define CAS __attribute__((address_space(4)))
__device__ __forceinline__ void ld_node(const void* nodes, size_t nb, float4& n0, float4& n1,
                                        float4& n2, float4& n3) {
  n0 = ld4(nodes, nb);
  n1 = ld4(nodes, nb + 1);
  n2 = ld4(nodes, nb + 2);
  n3 = ld4(nodes, nb + 3);
}
__device__ __forceinline__ void ld_tri(const void* tris, uint32_t p, float4& a, float4& b,
                                       float4& c) {
  a = ld4(tris, 3 * size_t(p));
  b = ld4(tris, 3 * size_t(p) + 1);
  c = ld4(tris, 3 * size_t(p) + 2);
}

// ---------------------------------------------------------------------------
// ray / box / triangle primitives
// ---------------------------------------------------------------------------
// Culling arithmetic (slab tests only; results never depend on it while it
// is conservative).  t of a plane is fmaf(bound, inv, -o * inv); its error is
// below 2^-24 (3 |o inv| + |bound inv|).  The node boxes' padding (1e-6 of
// the bound's magnitude, bvh_build.cpp) covers the |bound inv| part; the
// |o inv| part -- origins far from a box, or far from the world origin --
// is covered per ray: the near planes use o inv + ex, the far planes
// o inv - ex (signs by the direction), ex = 2^-21 |o inv| per axis, so the
// per-node cost is unchanged.  oracle.c evaluates the same operations.
struct Ray {
  float ox, oy, oz;
  float dx, dy, dz;
  float ix, iy, iz;     // 1/d with |d| clamped at kDirClamp (culling only)
  float olx, oly, olz;  // lo-plane offsets: o * inv + sign(inv) ex
  float ohx, ohy, ohz;  // hi-plane offsets: o * inv - sign(inv) ex
};

__device__ __forceinline__ void ray_axis(float o, float i, float& ol, float& oh) {
  const float oi = o * i;
  const float s = copysignf(0x1p-21f * fabsf(oi), i);
  ol = oi + s;
  oh = oi - s;
}

__device__ __forceinline__ float clamp_dir(float d) {
  return fabsf(d) < kDirClamp ? copysignf(kDirClamp, d) : d;
}

__device__ __forceinline__ Ray make_ray(float ox, float oy, float oz, float dx,
                                        float dy, float dz) {
  Ray r;
  r.ox = ox; r.oy = oy; r.oz = oz;
  r.dx = dx; r.dy = dy; r.dz = dz;
  r.ix = 1.0f / clamp_dir(dx);
  r.iy = 1.0f / clamp_dir(dy);
  r.iz = 1.0f / clamp_dir(dz);
  ray_axis(ox, r.ix, r.olx, r.ohx);
  ray_axis(oy, r.iy, r.oly, r.ohy);
  ray_axis(oz, r.iz, r.olz, r.ohz);
  return r;
}

// Conservative slab test of a (padded) node box against [tnear, tfar].
__device__ __forceinline__ bool slab(const Ray& r, float lx, float ly, float lz,
                                     float hx, float hy, float hz, float tnear,
                                     float tfar, float& tenter) {
  float t0x = fmaf(lx, r.ix, -r.olx), t1x = fmaf(hx, r.ix, -r.ohx);
  float t0y = fmaf(ly, r.iy, -r.oly), t1y = fmaf(hy, r.iy, -r.ohy);
  float t0z = fmaf(lz, r.iz, -r.olz), t1z = fmaf(hz, r.iz, -r.ohz);
  float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)),
                     fmaxf(fminf(t0z, t1z), tnear));
  float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)),
                     fminf(fmaxf(t0z, t1z), tfar * kTfarSlack));
  tenter = tmin;
  return tmin <= tmax;
}

// Embree 2.17 MoellerTrumboreIntersector1 restated (e1 = v0-v1, e2 = v2-v0,
// Ng = e1 x e2; edge tests scaled by |den|); t, u, v by IEEE division.
// Record: a = v0.xyz e1.x | b = e1.yz e2.xy | c = e2.z Ng.xyz
__device__ __forceinline__ bool tri_test(const Ray& r, float tnear, float4 a,
                                         float4 b, float4 c, float& t,
                                         float& u, float& v) {
  const float cx = a.x - r.ox, cy = a.y - r.oy, cz = a.z - r.oz;
  const float rx = fmaf(r.dy, cz, -(r.dz * cy));
  const float ry = fmaf(r.dz, cx, -(r.dx * cz));
  const float rz = fmaf(r.dx, cy, -(r.dy * cx));
  const float den = fmaf(c.w, r.dz, fmaf(c.z, r.dy, c.y * r.dx));
  const float absden = fabsf(den);
  float U = fmaf(rz, c.x, fmaf(ry, b.w, rx * b.z));  // R . e2
  float V = fmaf(rz, b.y, fmaf(ry, b.x, rx * a.w));  // R . e1
  float T = fmaf(c.w, cz, fmaf(c.z, cy, c.y * cx));  // Ng . C
  if (den < 0.0f) {
    U = -U;
    V = -V;
    T = -T;
  }
  if (!(den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= absden)) return false;
  const float tt = T / absden;
  if (!(tt > tnear)) return false;
  t = tt;
  u = U / absden;
  v = V / absden;
  return true;
}

// Reference domain-box test: intersectAabb (src/render/aabb.h:139-169) with
// t0 = SPRAY_RAY_EPSILON, t1 = +inf (RTCRayExt::reset, rays.h:149-169).  The
// exact float ops of the reference (division-based inverse, sub then mul).
struct DRay {
  float ox, oy, oz, ix, iy, iz;
};
__device__ __forceinline__ DRay make_dray(float ox, float oy, float oz,
                                          float dx, float dy, float dz) {
  DRay r;
  r.ox = ox; r.oy = oy; r.oz = oz;
  r.ix = 1.0f / dx;
  r.iy = 1.0f / dy;
  r.iz = 1.0f / dz;
  return r;
}
__device__ __forceinline__ bool aabb_ref6(float lx, float ly, float lz, float hx,
                                          float hy, float hz, const DRay& r,
                                          float& tmin_out) {
  const bool sx = r.ix < 0.0f, sy = r.iy < 0.0f, sz = r.iz < 0.0f;
  float tmin = ((sx ? hx : lx) - r.ox) * r.ix;
  float tmax = ((sx ? lx : hx) - r.ox) * r.ix;
  const float tymin = ((sy ? hy : ly) - r.oy) * r.iy;
  const float tymax = ((sy ? ly : hy) - r.oy) * r.iy;
  if ((tmin > tymax) || (tymin > tmax)) return false;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  const float tzmin = ((sz ? hz : lz) - r.oz) * r.iz;
  const float tzmax = ((sz ? lz : hz) - r.oz) * r.iz;
  if ((tmin > tzmax) || (tzmin > tmax)) return false;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  tmin_out = tmin;
  return (tmin < kInf) && (tmax > kRayEpsilon);
}
__device__ __forceinline__ bool aabb_ref(const float* box, const DRay& r,
                                         float& tmin_out) {
  return aabb_ref6(box[0], box[1], box[2], box[3], box[4], box[5], r, tmin_out);
}

// ---------------------------------------------------------------------------
// BVH2 traversal of one slot (canonical order, see oracle.c traverse())
// ---------------------------------------------------------------------------
struct Best {
  float t;
  uint32_t prim;  // PLY face index (tie-break key)
  uint32_t leaf;  // leaf-order triangle index (u, v, Ng are re-derived from it)
};

// ANY = occlusion (returns true at the first hit with t <= tfar_any).
// Closest hit: keeps the lexicographic minimum of (t, prim) starting from
// best; a candidate with t == best.t wins only with a smaller face index.
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool trace_tree(const void* nodes, const void* tris,
                                           const uint32_t* prims_, const Ray& r,
                                           float tnear, float tfar_any,
                                           Best& best, int32_t* stk,
                                           unsigned& nnode, unsigned& ntri) {
  // u, v of the winner are not carried through the traversal (2 VGPRs less at
  // the occupancy-limiting point): hit_uv() recomputes them bit-identically.
  const GAS uint32_t* __restrict__ prims = gptr(prims_);
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    const size_t nb = 4 * size_t(cur);
    float4 n0, n1, n2, n3;
    ld_node(nodes, nb, n0, n1, n2, n3);
    if (COUNT) ++nnode;
    const float tcut = ANY ? tfar_any : best.t;
    float tl, tr;
    const bool hl = slab(r, n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, tnear, tcut, tl);
    const bool hr = slab(r, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, tnear, tcut, tr);
    int32_t c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y);
    bool h0 = hl, h1 = hr;
    if (hl && hr && tr < tl) {
      const int32_t x = c0;
      c0 = c1;
      c1 = x;
    } else if (!hl && hr) {
      c0 = c1;
      h0 = true;
      h1 = false;
    }
    int32_t next = kNone;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int32_t c = k == 0 ? c0 : c1;
      const bool h = k == 0 ? h0 : h1;
      if (!h) continue;
      if (c < 0) {
        const uint32_t enc = ~uint32_t(c);
        const uint32_t first = enc >> 2, cnt = (enc & 3u) + 1u;
        for (uint32_t q = 0; q < cnt; ++q) {
          const uint32_t p = first + q;
          float4 a, b, cc;
          ld_tri(tris, p, a, b, cc);
          if (COUNT) ++ntri;
          float t, u, v;
          if (!tri_test(r, tnear, a, b, cc, t, u, v)) continue;
          if (ANY) {
            if (t <= tfar_any) return true;
          } else {
            const uint32_t pid = prims[p];
            if (t < best.t || (t == best.t && pid < best.prim)) {
              best.t = t;
              best.prim = pid;
              best.leaf = p;
            }
          }
        }
      } else if (next == kNone) {
        next = c;
      } else {
        stk[sp * kBlock] = c;
        ++sp;
      }
    }
    if (next == kNone) {
      if (sp == 0) break;
      --sp;
      next = stk[sp * kBlock];
    }
    cur = next;
  }
  return false;
}

// Any hit, one ray per lane, as a "while-while" walk with postponed leaves
// (Aila & Laine 2009): a lane that reaches a leaf parks it and keeps
// descending inner nodes until every active lane of the wave holds a leaf,
// then the lanes test their leaves' triangles together.  Leaf tests (the
// expensive, divergent part of the per-lane walk) then run with most lanes
// active instead of one lane's leaf stalling the rest at every step.  The
// result -- is there a hit with tnear < t <= tfar -- does not depend on the
// visit order, and culling stays conservative, so it equals trace_tree's.
// Leaves go through the per-lane stack like inner nodes; a visit still
// pushes at most one entry, so the stack bound (tree depth) is unchanged.
//
// The fp32 walk of the 64-B nodes (OOC drains); scene slots use the 4-wide
// quantized form below.
//
// Quantized nodes (occluded_tree_q4): the grid decode is folded into the
// ray's slab constants (t = q * (scale / d) + (base - o) / d); the extra grid
// step every quantized box carries covers the rounding, so culling stays
// conservative and the result is the fp32 walk's.
//
__device__ __forceinline__ float q_lo(float w) { return float(__float_as_uint(w) & 0xFFFFu); }
__device__ __forceinline__ float q_hi(float w) { return float(__float_as_uint(w) >> 16); }

struct QRay {
  float ix, iy, iz;     // scale * inv
  float olx, oly, olz;  // lo-plane offsets
  float ohx, ohy, ohz;  // hi-plane offsets
};

__device__ __forceinline__ void q_axis(float base, float scale, float ix, float oix, float& qix,
                                       float& ol, float& oh) {
  const float o = -fmaf(base, ix, -oix);
  qix = scale * ix;
  const float ex = 0x1p-20f * ((fabsf(oix) + fabsf(o)) + 65536.0f * fabsf(qix));
  const float sx = copysignf(ex, ix);
  ol = o + sx;  // lo plane: t - ex when ix > 0 (near), t + ex when ix < 0 (far)
  oh = o - sx;
}

__device__ __forceinline__ bool slab_q(const QRay& r, float lx, float ly, float lz, float hx,
                                       float hy, float hz, float tnear, float tfar,
                                       float& tenter) {
  float t0x = fmaf(lx, r.ix, -r.olx), t1x = fmaf(hx, r.ix, -r.ohx);
  float t0y = fmaf(ly, r.iy, -r.oly), t1y = fmaf(hy, r.iy, -r.ohy);
  float t0z = fmaf(lz, r.iz, -r.olz), t1z = fmaf(hz, r.iz, -r.ohz);
  float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)),
                     fmaxf(fminf(t0z, t1z), tnear));
  float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)),
                     fminf(fmaxf(t0z, t1z), tfar * kTfarSlack));
  tenter = tmin;
  return tmin <= tmax;
}

__device__ __forceinline__ bool occluded_tree_ww(const void* nodes, const void* tris,
                                                 const Ray& r, float tnear, float tfar,
                                                 int32_t* stk) {
  int sp = 0;
  int32_t cur = 0;       // next entry: inner node >= 0, leaf < 0, kNone = done
  int32_t leaf = kNone;  // the parked leaf
  for (;;) {
    while (cur >= 0 && cur != kNone) {
      float tl, tr;
      float4 n0, n1, n2, n3;
      ld_node(nodes, 4 * size_t(cur), n0, n1, n2, n3);
      const bool hl = slab(r, n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, tnear, tfar, tl);
      const bool hr = slab(r, n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, tnear, tfar, tr);
      int32_t c0 = __float_as_int(n3.x);
      int32_t c1 = __float_as_int(n3.y);
      if (hl && hr && tr < tl) {
        const int32_t x = c0;
        c0 = c1;
        c1 = x;
      }
      if (hl && hr) {
        stk[sp * kBlock] = c1;
        ++sp;
        cur = c0;
      } else if (hl || hr) {
        cur = hl ? c0 : c1;
      } else {
        cur = sp ? stk[--sp * kBlock] : kNone;
      }
      if (cur < 0 && leaf == kNone) {  // park the leaf, keep descending
        leaf = cur;
        cur = sp ? stk[--sp * kBlock] : kNone;
      }
      if (__ballot(leaf == kNone) == 0) break;  // every active lane holds a leaf
    }
    while (leaf != kNone) {
      const uint32_t enc = ~uint32_t(leaf);
      const uint32_t first = enc >> 2, cnt = (enc & 3u) + 1u;
      for (uint32_t q = 0; q < cnt; ++q) {
        float4 a, b, c;
        ld_tri(tris, first + q, a, b, c);
        float t, u, v;
        if (tri_test(r, tnear, a, b, c, t, u, v) && t <= tfar) return true;
      }
      leaf = kNone;
      if (cur < 0) {  // the walk stopped on a second leaf
        leaf = cur;
        cur = sp ? stk[--sp * kBlock] : kNone;
      }
    }
    if (cur == kNone) return false;
  }
}

// The same while-while any hit over the slot's 4-wide quantized nodes
// (QNode4, rt_common.h): a visit tests four child boxes, goes on with the
// nearest entered child and pushes the others (at most three), so a ray
// walks about half the levels of the BVH2 with twice the boxes per fetch --
// half the dependent node-fetch round trips and loop iterations, which bound
// this divergent walk.  The stack holds STK entries in LDS (stride kBlock)
// and kQ4Stack - STK in private memory; the host collapse bounds the pending
// entries by kQ4Stack.  Empty children (kNoChild) are never entered.
template <int STK>
__device__ __forceinline__ bool occluded_tree_q4(const void* nodes, const void* tris,
                                                 const Ray& r, float tnear, float tfar,
                                                 int32_t* stk) {
  const char* nbytes = static_cast<const char*>(nodes);
  QRay qr;
  {
    const float4 base = ld4(nbytes - sizeof(QGrid), 0);
    const float4 scale = ld4(nbytes - sizeof(QGrid), 1);
    q_axis(base.x, scale.x, r.ix, r.ox * r.ix, qr.ix, qr.olx, qr.ohx);
    q_axis(base.y, scale.y, r.iy, r.oy * r.iy, qr.iy, qr.oly, qr.ohy);
    q_axis(base.z, scale.z, r.iz, r.oz * r.iz, qr.iz, qr.olz, qr.ohz);
  }
  constexpr int kOvf = kQ4Stack > STK ? kQ4Stack - STK : 1;
  int32_t ovf[kOvf];
  int sp = 0;
  auto push = [&](int32_t v) {
    if (STK >= kQ4Stack || sp < STK)
      stk[sp * kBlock] = v;
    else
      ovf[sp - STK] = v;
    ++sp;
  };
  auto pop = [&]() -> int32_t {
    if (sp == 0) return kNone;
    --sp;
    return (STK >= kQ4Stack || sp < STK) ? stk[sp * kBlock] : ovf[sp - STK];
  };
  int32_t cur = 0;       // next entry: inner node >= 0, leaf < 0, kNone = done
  int32_t leaf = kNone;  // the parked leaf
  for (;;) {
    while (cur >= 0 && cur != kNone) {
      const char* qp = nbytes - 128 - 64 * size_t(cur);
      const float4 a = ld4(qp, 0), b = ld4(qp, 1), c = ld4(qp, 2), d = ld4(qp, 3);
      const int32_t ref[4] = {__float_as_int(d.x), __float_as_int(d.y), __float_as_int(d.z),
                              __float_as_int(d.w)};
      float t[4];
      bool h[4];
      h[0] = slab_q(qr, q_lo(a.x), q_hi(a.x), q_lo(a.y), q_hi(a.y), q_lo(a.z), q_hi(a.z),
                    tnear, tfar, t[0]);
      h[1] = slab_q(qr, q_lo(a.w), q_hi(a.w), q_lo(b.x), q_hi(b.x), q_lo(b.y), q_hi(b.y),
                    tnear, tfar, t[1]);
      h[2] = slab_q(qr, q_lo(b.z), q_hi(b.z), q_lo(b.w), q_hi(b.w), q_lo(c.x), q_hi(c.x),
                    tnear, tfar, t[2]);
      h[3] = slab_q(qr, q_lo(c.y), q_hi(c.y), q_lo(c.z), q_hi(c.z), q_lo(c.w), q_hi(c.w),
                    tnear, tfar, t[3]);
      // the nearest entered child next, the others pushed (sorting them far
      // to near, or no order at all, measured slower: DESIGN.md section 4)
      int32_t next = kNone;
      float tn = kInf;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!h[k] || ref[k] == kNoChildRef) continue;
        if (next == kNone || t[k] < tn) {
          if (next != kNone) push(next);
          next = ref[k];
          tn = t[k];
        } else {
          push(ref[k]);
        }
      }
      cur = next != kNone ? next : pop();
      if (cur < 0 && leaf == kNone) {  // park the leaf, keep descending
        leaf = cur;
        cur = pop();
      }
      if (__ballot(leaf == kNone) == 0) break;  // every active lane holds a leaf
    }
    while (leaf != kNone) {
      const uint32_t enc = ~uint32_t(leaf);
      const uint32_t first = enc >> 2, cnt = (enc & 3u) + 1u;
      for (uint32_t q = 0; q < cnt; ++q) {
        float4 a, b, c;
        ld_tri(tris, first + q, a, b, c);
        float t, u, v;
        if (tri_test(r, tnear, a, b, c, t, u, v) && t <= tfar) return true;
      }
      leaf = kNone;
      if (cur < 0) {  // the walk stopped on a second leaf
        leaf = cur;
        cur = pop();
      }
    }
    if (cur == kNone) return false;
  }
}

// Packet traversal of one domain tree by the whole wave.  The tree pointers
// and the walk (current node, stack) are wave-uniform: nodes and triangles
// come through scalar loads (one fetch per wave, broadcast), and a child is
// visited when the exact-per-lane slab test of any participating lane (act)
// accepts it, nearer side first by majority.  Each lane keeps its own
// result with the same winner rule as trace_tree, and since a lane only
// ever skips boxes its own conservative test rejected, the per-lane results
// are those of the per-lane walk.  ANY: a lane that finds an occluder sets
// hit and leaves the packet; the walk ends when no lane participates.
// wstk: kStack entries of LDS per wave.
typedef float v16f __attribute__((ext_vector_type(16)));

template <bool ANY>
__device__ __forceinline__ void trace_tree_packet(uint64_t nodes_u, uint64_t tris_u,
                                                  uint64_t prims_u, const Ray& r,
                                                  float tnear, float tfar_any, Best& best,
                                                  bool& act, bool& hit, int32_t* wstk) {
  const CAS v16f* nodes = reinterpret_cast<const CAS v16f*>(nodes_u);
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    // the whole 64-B node in one scalar fetch (one round trip per step)
    const v16f n = nodes[cur];
    const float tcut = ANY ? tfar_any : best.t;
    float tl = 0.f, tr = 0.f;
    const bool hl = slab(r, n[0], n[1], n[2], n[3], n[4], n[5], tnear, tcut, tl) && act;
    const bool hr = slab(r, n[6], n[7], n[8], n[9], n[10], n[11], tnear, tcut, tr) && act;
    const int32_t cl = __builtin_amdgcn_readfirstlane(__float_as_int(n[12]));
    const int32_t cr = __builtin_amdgcn_readfirstlane(__float_as_int(n[13]));
    const uint64_t bl = __ballot(hl), br = __ballot(hr);
    // near side of the first lane that enters both children (a majority
    // vote measured slower)
    const uint64_t both = bl & br;
    const bool lf = both ? __builtin_amdgcn_readlane(int(tl <= tr), __ffsll((long long)both) - 1) != 0
                         : true;
    int32_t next = kNone;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool left = (k == 0) == lf;
      const int32_t c = left ? cl : cr;
      if (!(left ? bl : br)) continue;
      if (c < 0) {
        const bool h = left ? hl : hr;
        const uint32_t enc = ~uint32_t(c);
        const uint32_t first = enc >> 2, cnt = (enc & 3u) + 1u;
        // the leaf's (up to four) 48-B triangles in three scalar fetches
        const CAS v16f* tq = reinterpret_cast<const CAS v16f*>(tris_u + 48ull * first);
        const v16f t0 = tq[0], t1 = tq[1], t2 = tq[2];
        const float tv[48] = {t0[0], t0[1], t0[2],  t0[3],  t0[4],  t0[5],  t0[6],  t0[7],
                              t0[8], t0[9], t0[10], t0[11], t0[12], t0[13], t0[14], t0[15],
                              t1[0], t1[1], t1[2],  t1[3],  t1[4],  t1[5],  t1[6],  t1[7],
                              t1[8], t1[9], t1[10], t1[11], t1[12], t1[13], t1[14], t1[15],
                              t2[0], t2[1], t2[2],  t2[3],  t2[4],  t2[5],  t2[6],  t2[7],
                              t2[8], t2[9], t2[10], t2[11], t2[12], t2[13], t2[14], t2[15]};
#pragma unroll
        for (uint32_t qq = 0; qq < 4; ++qq) {
          if (qq >= cnt) break;
          if (!h) continue;
          const float* x = tv + 12 * qq;
          float t, u, v;
          if (!tri_test(r, tnear, make_float4(x[0], x[1], x[2], x[3]),
                        make_float4(x[4], x[5], x[6], x[7]),
                        make_float4(x[8], x[9], x[10], x[11]), t, u, v))
            continue;
          const uint32_t p = first + qq;
          if (ANY) {
            if (t <= tfar_any) {
              hit = true;
              act = false;
            }
          } else {
            const uint32_t pid = reinterpret_cast<const CAS uint32_t*>(prims_u)[p];
            if (t < best.t || (t == best.t && pid < best.prim)) {
              best.t = t;
              best.prim = pid;
              best.leaf = p;
            }
          }
        }
        if (ANY && __ballot(act) == 0) return;
      } else if (next == kNone) {
        next = c;
      } else {
        wstk[sp] = c;
        ++sp;
      }
    }
    if (next == kNone) {
      if (sp == 0) break;
      --sp;
      next = __builtin_amdgcn_readfirstlane(wstk[sp]);
    }
    cur = next;
  }
}

template <bool ANY, bool COUNT>
__device__ __forceinline__ bool trace_slot(const SlotDesc& s, const Ray& r,
                                           float tnear, float tfar_any,
                                           Best& best, int32_t* stk,
                                           unsigned& nnode, unsigned& ntri) {
  return trace_tree<ANY, COUNT>(s.nodes, s.tris, s.prims, r, tnear, tfar_any, best,
                                stk, nnode, ntri);
}

// u, v (and Ng) of the accepted triangle: the same tri_test on the same
// operands, hence the same bits as during the traversal.
__device__ __forceinline__ float4 hit_uv(const SlotDesc& s, const Ray& r,
                                         float tnear, uint32_t leaf, float& u,
                                         float& v) {
  const float4 a = ld4(s.tris, 3 * size_t(leaf)), b = ld4(s.tris, 3 * size_t(leaf) + 1),
               c = ld4(s.tris, 3 * size_t(leaf) + 2);
  float t;
  tri_test(r, tnear, a, b, c, t, u, v);
  return c;
}

// TriMeshBuffer::updateIntersection (src/render/trimesh_buffer.cc:328-360).
__device__ __forceinline__ void epilogue(const SlotDesc& s, uint32_t prim,
                                         float u, float v, uint32_t& color,
                                         float& nsx, float& nsy, float& nsz) {
  const GAS uint32_t* faces = gptr(s.faces);
  const uint32_t f0 = faces[3 * prim], f1 = faces[3 * prim + 1],
                 f2 = faces[3 * prim + 2];
  const float w = 1.f - u - v;
  if (s.colors) {
    const GAS uint32_t* colors = gptr(s.colors);
    const uint32_t c0 = colors[f0], c1 = colors[f1], c2 = colors[f2];
    uint32_t ch[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int sh = 16 - 8 * k;
      const float a = float((c0 >> sh) & 0xffu), b = float((c1 >> sh) & 0xffu),
                  c = float((c2 >> sh) & 0xffu);
      ch[k] = uint32_t((a * w + b * u) + c * v);
    }
    color = (ch[0] << 16) | (ch[1] << 8) | ch[2];
  } else {
    color = 0;
  }
  if (s.normals) {
    const GAS float* n0 = gptr(s.normals) + 3 * f0;
    const GAS float* n1 = gptr(s.normals) + 3 * f1;
    const GAS float* n2 = gptr(s.normals) + 3 * f2;
    nsx = (n0[0] * w + n1[0] * u) + n2[0] * v;
    nsy = (n0[1] * w + n1[1] * u) + n2[1] * v;
    nsz = (n0[2] * w + n1[2] * u) + n2[2] * v;
  } else {
    nsx = nsy = nsz = 0.0f;
  }
}

// Domain list of one ray as a bitmask: WbvhEmbree::intersect
// (src/render/wbvh_embree.cc:126-148) over the top-level tree staged in LDS.
// Every node test is the reference's intersectAabb (exact ops) on exact union
// boxes, so the mask equals the brute-force list over all domain boxes.
template <int W>
__device__ __forceinline__ void tlas_mask(const float4* stl, int ntlas, int32_t* stk,
                                          float4 o4, float4 d4, uint64_t* m) {
#pragma unroll
  for (int w = 0; w < W; ++w) m[w] = 0;
  if (ntlas <= 0) return;
  const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    const float4 a = stl[4 * cur], b = stl[4 * cur + 1], c = stl[4 * cur + 2],
                 e = stl[4 * cur + 3];
    const int32_t cl = __float_as_int(e.x), cr = __float_as_int(e.y);
    float tm;
    const bool hl = aabb_ref6(a.x, a.y, a.z, a.w, b.x, b.y, dr, tm);
    const bool hr = cr != INT_MIN && aabb_ref6(b.z, b.w, c.x, c.y, c.z, c.w, dr, tm);
    int32_t next = kNone;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int32_t ch = k == 0 ? cl : cr;
      if (!(k == 0 ? hl : hr)) continue;
      if (ch < 0) {
        const int d = int(~uint32_t(ch) >> 2);
#pragma unroll
        for (int w = 0; w < W; ++w)
          if (w == (d >> 6)) m[w] |= 1ull << (d & 63);
      } else if (next == kNone) {
        next = ch;
      } else {
        stk[sp * kBlock] = ch;
        ++sp;
      }
    }
    if (next == kNone) {
      if (sp == 0) break;
      --sp;
      next = stk[sp * kBlock];
    }
    cur = next;
  }
}

// The same mask, traversed once per wave: every active lane evaluates the
// exact test at each node the wave visits, and a child is visited when any
// lane's test accepts it (ballot).  A lane that rejects a box rejects every
// box inside it (monotone ops on exact unions), so each lane's bits are
// exactly its own domain list.  Control flow and the stack (wstk, kStack
// entries of LDS per wave) are wave-uniform: no per-lane stack traffic and
// no divergence -- neighbouring rays share nearly all of their top-level
// path.
// Internal children carry padded boxes (build_domain_tree) and are tested
// with the fast slab -- a superset of the exact test -- leaf children with
// the reference's exact intersectAabb, which alone sets a lane's bit.
template <int W>
__device__ __forceinline__ void tlas_mask_wave(const float4* stl, int ntlas, int32_t* wstk,
                                               const Ray& r, float4 o4, float4 d4,
                                               uint64_t* m) {
#pragma unroll
  for (int w = 0; w < W; ++w) m[w] = 0;
  if (ntlas <= 0) return;
  const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    const float4 a = stl[4 * cur], b = stl[4 * cur + 1], c = stl[4 * cur + 2],
                 e = stl[4 * cur + 3];
    const int32_t cl = __builtin_amdgcn_readfirstlane(__float_as_int(e.x));
    const int32_t cr = __builtin_amdgcn_readfirstlane(__float_as_int(e.y));
    float tm;
    const bool hl = cl < 0 ? aabb_ref6(a.x, a.y, a.z, a.w, b.x, b.y, dr, tm)
                           : slab(r, a.x, a.y, a.z, a.w, b.x, b.y, 0.f, kInf, tm);
    const bool hr = cr == INT_MIN ? false
                    : cr < 0      ? aabb_ref6(b.z, b.w, c.x, c.y, c.z, c.w, dr, tm)
                                  : slab(r, b.z, b.w, c.x, c.y, c.z, c.w, 0.f, kInf, tm);
    const bool al = __ballot(hl) != 0, ar = __ballot(hr) != 0;
    int32_t next = kNone;
    if (cl < 0) {
      const int d = int(~uint32_t(cl) >> 2);
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (hl && w == (d >> 6)) m[w] |= 1ull << (d & 63);
    } else if (al) {
      next = cl;
    }
    if (cr < 0) {
      if (cr != INT_MIN) {
        const int d = int(~uint32_t(cr) >> 2);
#pragma unroll
        for (int w = 0; w < W; ++w)
          if (hr && w == (d >> 6)) m[w] |= 1ull << (d & 63);
      }
    } else if (ar) {
      if (next == kNone) {
        next = cr;
      } else {
        wstk[sp] = cr;
        ++sp;
      }
    }
    if (next == kNone) {
      if (sp == 0) break;
      --sp;
      next = __builtin_amdgcn_readfirstlane(wstk[sp]);
    }
    cur = next;
  }
}

// ooc::ShaderPt point-light branch for camera rays (ooc_shader_pt.h:93-171,
// blinnPhong reflection.h:202-214, hasPositive utils/math.h:76-78).
struct ShadePt {
  float lp[3], lr[3], ks[3], shininess;
};

__device__ __forceinline__ bool shadow_pt(const spray_rt_ray& ray,
                                          const spray_rt_hit& h,
                                          const ShadePt& sh, float pos[3],
                                          float wi[3]) {
  if (h.domain < 0) return false;
  const float* o = ray.org;
  const float* d = ray.dir;
  pos[0] = d[0] * h.t + o[0];
  pos[1] = d[1] * h.t + o[1];
  pos[2] = d[2] * h.t + o[2];
  const float kd[3] = {
      float(double((h.color >> 16) & 0xffu) * 0.00392156862745098),
      float(double((h.color >> 8) & 0xffu) * 0.00392156862745098),
      float(double(h.color & 0xffu) * 0.00392156862745098)};
  const float wo[3] = {-d[0], -d[1], -d[2]};
  const float cos_i = (wo[0] * h.ns[0] + wo[1] * h.ns[1]) + wo[2] * h.ns[2];
  float n[3] = {h.ns[0], h.ns[1], h.ns[2]};
  if (!(cos_i > 0.0f)) {
    n[0] = -n[0];
    n[1] = -n[1];
    n[2] = -n[2];
  }
  float inv = 1.0f / sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
  n[0] *= inv;
  n[1] *= inv;
  n[2] *= inv;
  float l[3] = {sh.lp[0] - pos[0], sh.lp[1] - pos[1], sh.lp[2] - pos[2]};
  inv = 1.0f / sqrtf((l[0] * l[0] + l[1] * l[1]) + l[2] * l[2]);
  wi[0] = l[0] * inv;
  wi[1] = l[1] * inv;
  wi[2] = l[2] * inv;
  float ct = (n[0] * wi[0] + n[1] * wi[1]) + n[2] * wi[2];
  ct = ct < 0.0f ? 0.0f : (ct > 1.0f ? 1.0f : ct);
  float hh[3] = {wi[0] + wo[0], wi[1] + wo[1], wi[2] + wo[2]};
  inv = 1.0f / sqrtf((hh[0] * hh[0] + hh[1] * hh[1]) + hh[2] * hh[2]);
  hh[0] *= inv;
  hh[1] *= inv;
  hh[2] *= inv;
  float ndh = (n[0] * hh[0] + n[1] * hh[1]) + n[2] * hh[2];
  ndh = ndh < 0.0f ? 0.0f : (ndh > 1.0f ? 1.0f : ndh);
  const float pw = powf(ndh, sh.shininess);
  bool pos_any = false;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float cs = sh.ks[k] * pw, cd = kd[k] * ct;
    if ((sh.lr[k] * (cd + cs)) * 1.0f > 0.0f) pos_any = true;
  }
  return pos_any;
}

}  // namespace
}  // namespace spray_rt
