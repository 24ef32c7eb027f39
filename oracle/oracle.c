/*
 * oracle.c -- CPU restatement of SpRay's intersect / occluded hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity against Embree 2.17.1 is
 * UNPINNED (Embree absent, reference has no tests); see DESIGN.md "Oracle".
 *
 * Conventions shared bit-for-bit with spray_amd/csrc/rt_kernels.hip:
 *  - compiled with -ffp-contract=off; fmaf() is written out where the GPU
 *    kernel uses a fused multiply-add, everything else is plain IEEE ops in
 *    source order.
 *  - triangle test = Embree 2 Moeller-Trumbore (e1 = v0-v1, e2 = v2-v0,
 *    Ng = e1 x e2, edge tests scaled by |den|), t/u/v by IEEE division.
 *  - closest hit = lexicographic minimum of (t, primID): independent of
 *    traversal order, so BVH and brute force agree exactly.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_INF (__builtin_inff())
#define OR_RAY_EPSILON 0.001f /* SPRAY_RAY_EPSILON, src/render/spray.h:46 */
#define OR_STACK 64

/* ------------------------------------------------------------------ */
/* small vector helpers (glm semantics, no contraction)                */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } f3;

static inline f3 mk3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 mul3s(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
/* glm::dot: tmp = a*b; tmp.x + tmp.y + tmp.z */
static inline float gdot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* glm::cross */
static inline f3 gcross(f3 a, f3 b) {
  return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* glm::normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt */
static inline f3 gnorm(f3 a) { return mul3s(a, 1.0f / sqrtf(gdot(a, a))); }
static inline float clampf(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

/* kernel-side helpers: explicit FMA forms shared with rt_kernels.hip */
static inline float kdot(const float a[3], const float b[3]) {
  return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0]));
}
static inline void kcross(const float a[3], const float b[3], float r[3]) {
  r[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
  r[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
  r[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}

/* ------------------------------------------------------------------ */
/* host data preparation                                               */
/* ------------------------------------------------------------------ */

/* TriMeshBuffer::load vertex transform, src/render/trimesh_buffer.cc:141-157:
 * v = x * vec4(v, 1).  glm's mat4*vec4 sums (m0*v.x + m1*v.y) + (m2*v.z +
 * m3*v.w).  m is column-major (glm layout): m[c*4 + r]. */
void or_transform_vertices(const float m[16], float* v, size_t nverts) {
  for (size_t i = 0; i < nverts; ++i) {
    float x = v[3 * i], y = v[3 * i + 1], z = v[3 * i + 2], w = 1.0f;
    float o[3];
    for (int r = 0; r < 3; ++r) {
      float a0 = m[0 * 4 + r] * x, a1 = m[1 * 4 + r] * y;
      float a2 = m[2 * 4 + r] * z, a3 = m[3 * 4 + r] * w;
      o[r] = (a0 + a1) + (a2 + a3);
    }
    v[3 * i] = o[0];
    v[3 * i + 1] = o[1];
    v[3 * i + 2] = o[2];
  }
}

/* SceneLoader::load world bound, src/io/scene_loader.cc:351-357: only the two
 * corners are transformed. */
void or_world_aabb(const float m[16], const float lo[3], const float hi[3],
                   float out[6]) {
  float a[3] = {lo[0], lo[1], lo[2]}, b[3] = {hi[0], hi[1], hi[2]};
  or_transform_vertices(m, a, 1);
  or_transform_vertices(m, b, 1);
  memcpy(out, a, sizeof(a));
  memcpy(out + 3, b, sizeof(b));
}

/* TriMeshBuffer::computeNormals, src/render/trimesh_buffer.cc:267-326:
 * unnormalised area-weighted sums of (v1-v0)x(v2-v0), face order. */
void or_compute_normals(const float* v, size_t nverts, const uint32_t* f,
                        size_t nfaces, float* n) {
  memset(n, 0, sizeof(float) * 3 * nverts);
  for (size_t i = 0; i < nfaces; ++i) {
    size_t a = (size_t)f[3 * i] * 3, b = (size_t)f[3 * i + 1] * 3,
           c = (size_t)f[3 * i + 2] * 3;
    f3 v0 = mk3(v[a], v[a + 1], v[a + 2]);
    f3 v1 = mk3(v[b], v[b + 1], v[b + 2]);
    f3 v2 = mk3(v[c], v[c + 1], v[c + 2]);
    f3 uu = sub3(v1, v0), vv = sub3(v2, v0);
    float nx = uu.y * vv.z - uu.z * vv.y;
    float ny = uu.z * vv.x - uu.x * vv.z;
    float nz = uu.x * vv.y - uu.y * vv.x;
    n[a] += nx; n[a + 1] += ny; n[a + 2] += nz;
    n[b] += nx; n[b + 1] += ny; n[b + 2] += nz;
    n[c] += nx; n[c + 1] += ny; n[c + 2] += nz;
  }
}

/* ------------------------------------------------------------------ */
/* camera, sampler, eye rays                                           */
/* ------------------------------------------------------------------ */

/* Camera::init, src/render/camera.h:128-166 (float/double mix kept). */
void or_camera_init(const float pos[3], const float lookat[3],
                    const float up[3], float vfov, int image_w, int image_h,
                    float cam[14]) {
  float aspect = (float)image_w / (float)image_h;
  float theta = (float)((double)vfov * 3.14159265358979323846 / 180.0);
  float half_h = (float)tan((double)(theta / 2.0f));
  float half_w = aspect * half_h;
  f3 P = mk3(pos[0], pos[1], pos[2]);
  f3 L = mk3(lookat[0], lookat[1], lookat[2]);
  f3 U = mk3(up[0], up[1], up[2]);
  f3 w = sub3(P, L);
  f3 u = gcross(U, w);
  f3 v = gcross(w, u);
  w = gnorm(w);
  u = gnorm(u);
  v = gnorm(v);
  f3 center = sub3(P, w);
  f3 ll = sub3(sub3(center, mul3s(u, half_w)), mul3s(v, half_h));
  f3 wv = mul3s(u, 2.0f * half_w);
  f3 hv = mul3s(v, 2.0f * half_h);
  cam[0] = P.x; cam[1] = P.y; cam[2] = P.z;
  cam[3] = ll.x; cam[4] = ll.y; cam[5] = ll.z;
  cam[6] = wv.x; cam[7] = wv.y; cam[8] = wv.z;
  cam[9] = hv.x; cam[10] = hv.y; cam[11] = hv.z;
  cam[12] = (float)image_w;
  cam[13] = (float)image_h;
}

/* Camera::generateRay + getDirection, src/render/camera.h:168-209. */
void or_camera_ray(const float cam[14], float x, float y, float dir[3]) {
  float u = x / cam[12], v = y / cam[13];
  f3 ll = mk3(cam[3], cam[4], cam[5]);
  f3 wv = mk3(cam[6], cam[7], cam[8]);
  f3 hv = mk3(cam[9], cam[10], cam[11]);
  f3 P = mk3(cam[0], cam[1], cam[2]);
  f3 d = sub3(add3(add3(ll, mul3s(wv, u)), mul3s(hv, v)), P);
  d = gnorm(d);
  dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

/* deps/embree/random_sampler.h:34-108 */
static inline uint32_t mm_mix(uint32_t hash, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = (k << 15) | (k >> 17);
  k *= 0x1b873593u;
  hash ^= k;
  hash = ((hash << 13) | (hash >> 19)) * 5u + 0xe6546b64u;
  return hash;
}
static inline uint32_t mm_fin(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
uint32_t or_sampler_init1(int id) { return mm_fin(mm_mix(0u, (uint32_t)id)); }
uint32_t or_sampler_init2(int p, int s) {
  return mm_fin(mm_mix(mm_mix(0u, (uint32_t)p), (uint32_t)s));
}
float or_sampler_get1d(uint32_t* s) {
  *s = *s * 1664525u + 1013904223u;
  return (float)(int32_t)(*s >> 1) * 4.656612873077392578125e-10f;
}

/* ooc::Tracer::genMultiEyes / genSingleEyes, src/ooc/ooc_tracer.inl:84-172:
 * bufid = spp*(y0*tw + x0) + s, jitter seeded by the TILE-LOCAL bufid. */
void or_eye_rays_ooc(const float cam[14], int image_w, int spp, int tx, int ty,
                     int tw, int th, float* org, float* dir, int32_t* pixid,
                     int32_t* samid) {
  long total = (long)tw * th;
#pragma omp parallel for schedule(static)
  for (long p = 0; p < total; ++p) {
    int y0 = (int)(p / tw), x0 = (int)(p % tw);
    int x = tx + x0, y = ty + y0;
    for (int s = 0; s < spp; ++s) {
      int bufid = spp * (y0 * tw + x0) + s;
      float fx, fy;
      if (spp > 1) {
        uint32_t st = or_sampler_init1(bufid);
        fx = (float)x + or_sampler_get1d(&st);
        fy = (float)y + or_sampler_get1d(&st);
      } else {
        fx = (float)x;
        fy = (float)y;
      }
      float* o = org + 3 * (size_t)bufid;
      o[0] = cam[0]; o[1] = cam[1]; o[2] = cam[2];
      or_camera_ray(cam, fx, fy, dir + 3 * (size_t)bufid);
      if (pixid) pixid[bufid] = y * image_w + x;
      if (samid) samid[bufid] = bufid;
    }
  }
}

/* insitu::genMultiSampleEyeRays, src/insitu/insitu_ray.h:138-182: jitter
 * seeded by (pixid, s); samid relative to the blocking tile. */
void or_eye_rays_insitu(const float cam[14], int image_w, int spp, int bx,
                        int by, int bw, int bh, int tx, int ty, int tw, int th,
                        float* org, float* dir, int32_t* pixid,
                        int32_t* samid) {
  (void)bh;
  long total = (long)tw * th;
#pragma omp parallel for schedule(static)
  for (long p = 0; p < total; ++p) {
    int y = ty + (int)(p / tw), x = tx + (int)(p % tw);
    for (int s = 0; s < spp; ++s) {
      int bufid = (tw * (y - ty) + (x - tx)) * spp + s;
      int pid = image_w * y + x;
      float fx, fy;
      if (spp > 1) {
        uint32_t st = or_sampler_init2(pid, s);
        fx = (float)x + or_sampler_get1d(&st);
        fy = (float)y + or_sampler_get1d(&st);
      } else {
        fx = (float)x;
        fy = (float)y;
      }
      float* o = org + 3 * (size_t)bufid;
      o[0] = cam[0]; o[1] = cam[1]; o[2] = cam[2];
      or_camera_ray(cam, fx, fy, dir + 3 * (size_t)bufid);
      if (pixid) pixid[bufid] = pid;
      if (samid)
        samid[bufid] = spp > 1 ? (bw * (y - by) + (x - bx)) * spp + s
                               : bw * (y - by) + (x - bx);
    }
  }
}

/* ------------------------------------------------------------------ */
/* domain query (a5)                                                   */
/* ------------------------------------------------------------------ */

/* intersectAabb, src/render/aabb.h:139-169 (float org/dir overload), with the
 * ray extents of RTCRayExt::reset (rays.h:149-169): t0 = 0.001, t1 = +inf.
 * WbvhEmbree::cbIntersect1 (wbvh_embree.cc:126-148) pushes (id, tmin). */
static inline int aabb_hit(const float* box, const float o[3], const float d[3],
                           float t0, float t1, float* tmin_o) {
  float inv0 = 1.0f / d[0], inv1 = 1.0f / d[1], inv2 = 1.0f / d[2];
  int s0 = inv0 < 0.0f, s1 = inv1 < 0.0f, s2 = inv2 < 0.0f;
  /* bounds[0] = lo (box[0..2]), bounds[1] = hi (box[3..5]) */
  float tmin = (box[3 * s0 + 0] - o[0]) * inv0;
  float tmax = (box[3 * (1 - s0) + 0] - o[0]) * inv0;
  float tymin = (box[3 * s1 + 1] - o[1]) * inv1;
  float tymax = (box[3 * (1 - s1) + 1] - o[1]) * inv1;
  if ((tmin > tymax) || (tymin > tmax)) return 0;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin = (box[3 * s2 + 2] - o[2]) * inv2;
  float tzmax = (box[3 * (1 - s2) + 2] - o[2]) * inv2;
  if ((tmin > tzmax) || (tzmin > tmax)) return 0;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  *tmin_o = tmin;
  return (tmin < t1) && (tmax > t0);
}

/* Sorted domain list: DomainList::push/sort, src/render/rays.h:71-86, key
 * (t asc, id asc).  Insertion sort -- lists are short (<= ndomains). */
static int domain_list(const float* boxes, int ndom, const float o[3],
                       const float d[3], int maxhits, int32_t* ids, float* ts,
                       int* overflow) {
  int cnt = 0;
  for (int b = 0; b < ndom; ++b) {
    float tmin;
    if (!aabb_hit(boxes + 6 * b, o, d, OR_RAY_EPSILON, OR_INF, &tmin)) continue;
    /* insert (tmin, b) keeping order; ids arrive ascending so equal t keeps
     * the earlier (smaller) id first */
    int k = cnt < maxhits ? cnt : maxhits;
    if (cnt >= maxhits) {
      *overflow = 1;
      if (!(tmin < ts[maxhits - 1])) { ++cnt; continue; }
      k = maxhits - 1;
    }
    while (k > 0 && tmin < ts[k - 1]) {
      ts[k] = ts[k - 1];
      ids[k] = ids[k - 1];
      --k;
    }
    ts[k] = tmin;
    ids[k] = b;
    ++cnt;
  }
  return cnt < maxhits ? cnt : maxhits;
}

int or_domain_query(const float* org, const float* dir, size_t n,
                    const float* boxes, int ndom, int maxhits, int32_t* ids,
                    float* ts, int32_t* counts) {
  int nover = 0;
#pragma omp parallel for schedule(static) reduction(+ : nover)
  for (long i = 0; i < (long)n; ++i) {
    int over = 0;
    counts[i] = domain_list(boxes, ndom, org + 3 * i, dir + 3 * i, maxhits,
                            ids + (size_t)i * maxhits, ts + (size_t)i * maxhits,
                            &over);
    nover += over;
  }
  return nover;
}

/* ------------------------------------------------------------------ */
/* triangle test (Embree 2.17 MoellerTrumboreIntersector1 restated)    */
/* ------------------------------------------------------------------ */

void or_prep_tris(const float* v, const uint32_t* f, size_t nf, float* tri) {
  for (size_t i = 0; i < nf; ++i) {
    const float* a = v + 3 * (size_t)f[3 * i];
    const float* b = v + 3 * (size_t)f[3 * i + 1];
    const float* c = v + 3 * (size_t)f[3 * i + 2];
    float* r = tri + 12 * i;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
    r[3] = a[0] - b[0]; r[4] = a[1] - b[1]; r[5] = a[2] - b[2]; /* e1=v0-v1 */
    r[6] = c[0] - a[0]; r[7] = c[1] - a[1]; r[8] = c[2] - a[2]; /* e2=v2-v0 */
    kcross(r + 3, r + 6, r + 9);                                 /* Ng=e1xe2 */
  }
}

/* Returns 1 and t/u/v when the ray's line crosses the triangle at t > tnear.
 * Depth-vs-tfar is decided by the caller (closest-hit or any-hit rule). */
static inline int tri_test(const float o[3], const float d[3], float tnear,
                           const float* tr, float* t, float* u, float* v) {
  float c[3] = {tr[0] - o[0], tr[1] - o[1], tr[2] - o[2]};
  float r[3];
  kcross(d, c, r);
  float den = kdot(tr + 9, d);
  float absden = fabsf(den);
  float U = kdot(r, tr + 6);
  float V = kdot(r, tr + 3);
  if (den < 0.0f) { U = -U; V = -V; }
  if (!(den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= absden)) return 0;
  float T = kdot(tr + 9, c);
  if (den < 0.0f) T = -T;
  float tt = T / absden;
  if (!(tt > tnear)) return 0;
  *t = tt;
  *u = U / absden;
  *v = V / absden;
  return 1;
}

/* closest-hit acceptance: (t, prim) lexicographic, initial (tfar, ~0u) so a
 * hit at exactly tfar is accepted as Embree's T <= |den|*tfar does. */
static inline int ch_better(float t, uint32_t p, float bt, uint32_t bp) {
  return (t < bt) || (t == bt && p < bp);
}

void or_brute_intersect(const float* tri, size_t nf, const float* org,
                        const float* dir, const float* tnear,
                        const float* tfar, size_t n, float* t_out,
                        float* u_out, float* v_out, uint32_t* prim_out) {
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < (long)n; ++i) {
    const float* o = org + 3 * i;
    const float* d = dir + 3 * i;
    float bt = tfar ? tfar[i] : OR_INF, bu = 0, bv = 0;
    uint32_t bp = 0xFFFFFFFFu;
    float tn = tnear ? tnear[i] : OR_RAY_EPSILON;
    for (size_t k = 0; k < nf; ++k) {
      float t, u, v;
      if (tri_test(o, d, tn, tri + 12 * k, &t, &u, &v) &&
          ch_better(t, (uint32_t)k, bt, bp)) {
        bt = t; bu = u; bv = v; bp = (uint32_t)k;
      }
    }
    t_out[i] = bp == 0xFFFFFFFFu ? (tfar ? tfar[i] : OR_INF) : bt;
    u_out[i] = bu;
    v_out[i] = bv;
    prim_out[i] = bp;
  }
}

void or_brute_occluded(const float* tri, size_t nf, const float* org,
                       const float* dir, const float* tnear,
                       const float* tfar, size_t n, uint8_t* occ) {
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < (long)n; ++i) {
    float tf = tfar ? tfar[i] : OR_INF;
    float tn = tnear ? tnear[i] : OR_RAY_EPSILON;
    uint8_t hit = 0;
    for (size_t k = 0; k < nf && !hit; ++k) {
      float t, u, v;
      if (tri_test(org + 3 * i, dir + 3 * i, tn, tri + 12 * k, &t, &u, &v) &&
          t <= tf)
        hit = 1;
    }
    occ[i] = hit;
  }
}

/* float64 checker: same geometry, computed in double from the float
 * vertices; flags hits within relative 1e-5 of an edge (margin). */
void or_f64_intersect(const float* vv, const uint32_t* f, size_t nf,
                      const float* org, const float* dir, float tnear,
                      size_t n, double* t_out, int32_t* prim_out,
                      uint8_t* margin_out) {
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < (long)n; ++i) {
    double o[3] = {org[3 * i], org[3 * i + 1], org[3 * i + 2]};
    double d[3] = {dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]};
    double bt = INFINITY, bmargin = 0;
    int32_t bp = -1;
    for (size_t k = 0; k < nf; ++k) {
      const float* A = vv + 3 * (size_t)f[3 * k];
      const float* B = vv + 3 * (size_t)f[3 * k + 1];
      const float* C = vv + 3 * (size_t)f[3 * k + 2];
      double e1[3], e2[3], p[3], q[3], s[3];
      for (int j = 0; j < 3; ++j) {
        e1[j] = (double)B[j] - (double)A[j];
        e2[j] = (double)C[j] - (double)A[j];
        s[j] = o[j] - (double)A[j];
      }
      p[0] = d[1] * e2[2] - d[2] * e2[1];
      p[1] = d[2] * e2[0] - d[0] * e2[2];
      p[2] = d[0] * e2[1] - d[1] * e2[0];
      double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
      if (det == 0.0) continue;
      double inv = 1.0 / det;
      double u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * inv;
      q[0] = s[1] * e1[2] - s[2] * e1[1];
      q[1] = s[2] * e1[0] - s[0] * e1[2];
      q[2] = s[0] * e1[1] - s[1] * e1[0];
      double v = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
      double t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
      double m = fmin(fmin(u, v), 1.0 - u - v);
      if (m < -1e-5 || t <= (double)tnear) continue;
      if (t < bt) {
        bt = t;
        bp = (int32_t)k;
        bmargin = m;
      }
    }
    t_out[i] = bt;
    prim_out[i] = bp;
    margin_out[i] = (uint8_t)(bp >= 0 && bmargin < 1e-5);
  }
}

/* ------------------------------------------------------------------ */
/* canonical BVH2 builder                                              */
/* ------------------------------------------------------------------ */
/* Binned SAH (32 bins on each of the 3 axes over the centroid bounds),
 * leaves of <= 4 triangles, depth-first layout (node 0 = root, left subtree
 * before right), leaf triangles appended in creation order.  Child refs:
 * >= 0 internal node index, < 0 leaf: ~((first << 2) | (count - 1)).
 * When a subtree could exceed OR_MAX_DEPTH the split falls back to the
 * object median on the widest centroid axis. */
#define OR_BINS 32
#define OR_LEAF 4
#define OR_MAX_DEPTH 24

typedef struct { float lo[3], hi[3]; } box3;

struct or_bvh {
  float* nodes; /* [cap][16] */
  size_t nnodes, cap;
  uint32_t* order; /* [nf] */
  size_t norder;
  float* tri;      /* [nf][12] in leaf order */
  size_t nf;
  int depth;
  /* build scratch */
  box3* pbox;
  float* cent; /* [nf][3] */
  uint32_t* idx;
  uint32_t* tmp;
};

static inline void box_empty(box3* b) {
  b->lo[0] = b->lo[1] = b->lo[2] = OR_INF;
  b->hi[0] = b->hi[1] = b->hi[2] = -OR_INF;
}
static inline void box_grow(box3* b, const box3* o) {
  for (int j = 0; j < 3; ++j) {
    if (o->lo[j] < b->lo[j]) b->lo[j] = o->lo[j];
    if (o->hi[j] > b->hi[j]) b->hi[j] = o->hi[j];
  }
}
static inline float box_area(const box3* b) {
  float dx = b->hi[0] - b->lo[0], dy = b->hi[1] - b->lo[1],
        dz = b->hi[2] - b->lo[2];
  return (dx * dy + dy * dz) + dz * dx;
}

static int ceil_log2(size_t x) {
  int l = 0;
  while (((size_t)1 << l) < x) ++l;
  return l;
}

static size_t alloc_node(or_bvh* b) {
  if (b->nnodes == b->cap) {
    b->cap = b->cap ? 2 * b->cap : 64;
    b->nodes = (float*)realloc(b->nodes, b->cap * 16 * sizeof(float));
  }
  memset(b->nodes + 16 * b->nnodes, 0, 16 * sizeof(float));
  return b->nnodes++;
}

/* returns child ref; *bb_out = bounds of the subtree */
static int32_t build_rec(or_bvh* b, size_t begin, size_t end, int depth,
                         box3* bb_out) {
  size_t n = end - begin;
  box3 bb, cb;
  box_empty(&bb);
  box_empty(&cb);
  for (size_t i = begin; i < end; ++i) {
    uint32_t p = b->idx[i];
    box_grow(&bb, &b->pbox[p]);
    box3 c;
    for (int j = 0; j < 3; ++j) c.lo[j] = c.hi[j] = b->cent[3 * p + j];
    box_grow(&cb, &c);
  }
  *bb_out = bb;
  if (depth > b->depth) b->depth = depth;
  if (n <= OR_LEAF) {
    uint32_t first = (uint32_t)b->norder;
    for (size_t i = begin; i < end; ++i) b->order[b->norder++] = b->idx[i];
    return ~(int32_t)((first << 2) | (uint32_t)(n - 1));
  }

  int axis = -1, split = -1;
  size_t mid = begin;
  float ext[3] = {cb.hi[0] - cb.lo[0], cb.hi[1] - cb.lo[1], cb.hi[2] - cb.lo[2]};
  int need_median = depth + ceil_log2((n + OR_LEAF - 1) / OR_LEAF) >= OR_MAX_DEPTH;

  if (!need_median) {
    float best = OR_INF;
    for (int a = 0; a < 3; ++a) {
      if (!(ext[a] > 0.0f)) continue;
      float scale = (float)OR_BINS / ext[a];
      box3 bins[OR_BINS];
      uint32_t cnt[OR_BINS];
      for (int k = 0; k < OR_BINS; ++k) { box_empty(&bins[k]); cnt[k] = 0; }
      for (size_t i = begin; i < end; ++i) {
        uint32_t p = b->idx[i];
        int k = (int)((b->cent[3 * p + a] - cb.lo[a]) * scale);
        if (k > OR_BINS - 1) k = OR_BINS - 1;
        if (k < 0) k = 0;
        box_grow(&bins[k], &b->pbox[p]);
        cnt[k]++;
      }
      /* right sweep */
      float rarea[OR_BINS];
      uint32_t rcnt[OR_BINS];
      box3 acc;
      box_empty(&acc);
      uint32_t c = 0;
      for (int k = OR_BINS - 1; k > 0; --k) {
        box_grow(&acc, &bins[k]);
        c += cnt[k];
        rarea[k] = c ? box_area(&acc) : 0.0f;
        rcnt[k] = c;
      }
      box_empty(&acc);
      c = 0;
      for (int k = 0; k < OR_BINS - 1; ++k) {
        box_grow(&acc, &bins[k]);
        c += cnt[k];
        if (c == 0 || rcnt[k + 1] == 0) continue;
        float cost = (float)c * box_area(&acc) + (float)rcnt[k + 1] * rarea[k + 1];
        if (cost < best) {
          best = cost;
          axis = a;
          split = k + 1; /* bins [0, split) go left */
        }
      }
    }
  }

  if (axis >= 0) {
    /* stable partition by bin < split */
    float scale = (float)OR_BINS / ext[axis];
    size_t l = begin, r = 0;
    for (size_t i = begin; i < end; ++i) {
      uint32_t p = b->idx[i];
      int k = (int)((b->cent[3 * p + axis] - cb.lo[axis]) * scale);
      if (k > OR_BINS - 1) k = OR_BINS - 1;
      if (k < 0) k = 0;
      if (k < split) b->idx[l++] = p;
      else b->tmp[r++] = p;
    }
    memcpy(b->idx + l, b->tmp, r * sizeof(uint32_t));
    mid = l;
  } else {
    /* object median on the widest centroid axis (stable: by centroid, then
     * index); degenerate centroid bounds keep the current order */
    int a = 0;
    if (ext[1] > ext[a]) a = 1;
    if (ext[2] > ext[a]) a = 2;
    if (ext[a] > 0.0f) {
      /* insertion sort is fine for the rare fallback, use merge for size */
      size_t m = n;
      uint32_t* src = b->idx + begin;
      uint32_t* dst = b->tmp;
      for (size_t w = 1; w < m; w *= 2) {
        for (size_t lo = 0; lo < m; lo += 2 * w) {
          size_t mi = lo + w < m ? lo + w : m, hi = lo + 2 * w < m ? lo + 2 * w : m;
          size_t x = lo, y = mi, o = lo;
          while (x < mi && y < hi) {
            float cx = b->cent[3 * src[x] + a], cy = b->cent[3 * src[y] + a];
            if (cy < cx || (cy == cx && src[y] < src[x])) dst[o++] = src[y++];
            else dst[o++] = src[x++];
          }
          while (x < mi) dst[o++] = src[x++];
          while (y < hi) dst[o++] = src[y++];
        }
        uint32_t* t = src; src = dst; dst = t;
      }
      if (src != b->idx + begin) memcpy(b->idx + begin, src, m * sizeof(uint32_t));
    }
    mid = begin + n / 2;
  }

  size_t self = alloc_node(b);
  box3 lb, rb;
  int32_t lref = build_rec(b, begin, mid, depth + 1, &lb);
  int32_t rref = build_rec(b, mid, end, depth + 1, &rb);
  float* nd = b->nodes + 16 * self;
  nd[0] = lb.lo[0]; nd[1] = lb.lo[1]; nd[2] = lb.lo[2];
  nd[3] = lb.hi[0]; nd[4] = lb.hi[1]; nd[5] = lb.hi[2];
  nd[6] = rb.lo[0]; nd[7] = rb.lo[1]; nd[8] = rb.lo[2];
  nd[9] = rb.hi[0]; nd[10] = rb.hi[1]; nd[11] = rb.hi[2];
  memcpy(nd + 12, &lref, 4);
  memcpy(nd + 13, &rref, 4);
  return (int32_t)self;
}

or_bvh* or_bvh_build(const float* v, const uint32_t* f, size_t nf) {
  or_bvh* b = (or_bvh*)calloc(1, sizeof(or_bvh));
  b->nf = nf;
  b->order = (uint32_t*)malloc((nf ? nf : 1) * sizeof(uint32_t));
  b->pbox = (box3*)malloc((nf ? nf : 1) * sizeof(box3));
  b->cent = (float*)malloc((nf ? nf : 1) * 3 * sizeof(float));
  b->idx = (uint32_t*)malloc((nf ? nf : 1) * sizeof(uint32_t));
  b->tmp = (uint32_t*)malloc((nf ? nf : 1) * sizeof(uint32_t));
  for (size_t i = 0; i < nf; ++i) {
    box3 pb;
    box_empty(&pb);
    for (int k = 0; k < 3; ++k) {
      box3 pt;
      const float* p = v + 3 * (size_t)f[3 * i + k];
      for (int j = 0; j < 3; ++j) pt.lo[j] = pt.hi[j] = p[j];
      box_grow(&pb, &pt);
    }
    b->pbox[i] = pb;
    for (int j = 0; j < 3; ++j)
      b->cent[3 * i + j] = (pb.lo[j] + pb.hi[j]) * 0.5f;
    b->idx[i] = (uint32_t)i;
  }
  if (nf > 0) {
    if (nf <= OR_LEAF) {
      /* a root that is itself a leaf is stored as a node whose left child is
       * the leaf and right child is an empty box */
      size_t self = alloc_node(b);
      box3 lb;
      int32_t lref = build_rec(b, 0, nf, 1, &lb);
      float* nd = b->nodes + 16 * self;
      nd[0] = lb.lo[0]; nd[1] = lb.lo[1]; nd[2] = lb.lo[2];
      nd[3] = lb.hi[0]; nd[4] = lb.hi[1]; nd[5] = lb.hi[2];
      /* lo = hi = +inf: every slab test misses it (no NaN can arise) */
      nd[6] = nd[7] = nd[8] = OR_INF;
      nd[9] = nd[10] = nd[11] = OR_INF;
      int32_t empty = ~(int32_t)0; /* never reached: box is empty */
      memcpy(nd + 12, &lref, 4);
      memcpy(nd + 13, &empty, 4);
    } else {
      box3 rb;
      build_rec(b, 0, nf, 0, &rb);
    }
  }
  b->tri = (float*)malloc((nf ? nf : 1) * 12 * sizeof(float));
  for (size_t i = 0; i < nf; ++i) {
    uint32_t p = b->order[i];
    uint32_t fv[3] = {f[3 * p], f[3 * p + 1], f[3 * p + 2]};
    or_prep_tris(v, fv, 1, b->tri + 12 * i);
  }
  free(b->pbox); free(b->cent); free(b->idx); free(b->tmp);
  b->pbox = NULL; b->cent = NULL; b->idx = NULL; b->tmp = NULL;
  return b;
}

void or_bvh_free(or_bvh* b) {
  if (!b) return;
  free(b->nodes); free(b->order); free(b->tri); free(b);
}
size_t or_bvh_num_nodes(const or_bvh* b) { return b->nnodes; }
int or_bvh_depth(const or_bvh* b) { return b->depth; }
void or_bvh_export(const or_bvh* b, float* nodes, uint32_t* order) {
  if (nodes) memcpy(nodes, b->nodes, b->nnodes * 16 * sizeof(float));
  if (order) memcpy(order, b->order, b->nf * sizeof(uint32_t));
}

/* ------------------------------------------------------------------ */
/* canonical traversal                                                 */
/* ------------------------------------------------------------------ */
/* Slab test used for culling only (results never depend on it as long as it
 * is conservative): inverse direction with |d| < 1e-20 clamped to
 * +-1e-20, t = fmaf(bound, inv, -(org*inv +- ex)), hit iff
 *   max(tmin.x, tmin.y, tmin.z, tnear) <= min(tmax.x, tmax.y, tmax.z, tfar*(1+2^-16))
 * The rounding error of a plane's t is below 2^-24 (3 |org inv| + |bound
 * inv|): the box padding below covers the bound part, and the per-axis
 * offset ex = 2^-21 |org inv| (near planes use org*inv + ex, far planes
 * org*inv - ex, by the sign of inv) the origin part -- rays from far away or
 * at large coordinates.  The (1+2^-16) widening covers tfar.  (tests/ check
 * BVH == brute force bit-exactly; spray_amd/csrc/rt_device.h, Ray, is the
 * same arithmetic.) */
#define OR_TFAR_SLACK 1.0000153f

typedef struct {
  float o[3], d[3], inv[3], ol[3], oh[3];
} ray_pre;

static inline void ray_prep(ray_pre* r, const float* o, const float* d) {
  for (int j = 0; j < 3; ++j) {
    r->o[j] = o[j];
    r->d[j] = d[j];
    float dj = fabsf(d[j]) < 1e-20f ? copysignf(1e-20f, d[j]) : d[j];
    r->inv[j] = 1.0f / dj;
    float oi = o[j] * r->inv[j];
    float s = copysignf(0x1p-21f * fabsf(oi), r->inv[j]);
    r->ol[j] = oi + s;
    r->oh[j] = oi - s;
  }
}

static inline int slab(const ray_pre* r, const float* lo, const float* hi,
                       float tnear, float tfar, float* tenter) {
  float t0x = fmaf(lo[0], r->inv[0], -r->ol[0]);
  float t1x = fmaf(hi[0], r->inv[0], -r->oh[0]);
  float t0y = fmaf(lo[1], r->inv[1], -r->ol[1]);
  float t1y = fmaf(hi[1], r->inv[1], -r->oh[1]);
  float t0z = fmaf(lo[2], r->inv[2], -r->ol[2]);
  float t1z = fmaf(hi[2], r->inv[2], -r->oh[2]);
  float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)),
                     fmaxf(fminf(t0z, t1z), tnear));
  float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)),
                     fminf(fmaxf(t0z, t1z), tfar * OR_TFAR_SLACK));
  *tenter = tmin;
  return tmin <= tmax;
}

/* Node boxes are padded at build export (or_scene / GPU upload) by
 * OR_BOX_PAD relative to the box extent -- see pad_box(). */
#define OR_BOX_PAD 1e-6f

static inline void pad_box(const float* in, float* out) {
  for (int j = 0; j < 3; ++j) {
    float e = (in[3 + j] - in[j]);
    float m = fmaxf(fmaxf(fabsf(in[j]), fabsf(in[3 + j])), e);
    float p = m * OR_BOX_PAD;
    out[j] = in[j] - p;
    out[3 + j] = in[3 + j] + p;
  }
}

/* One (ray, domain) visit.  mode 0 = closest hit (updates bt, bp, ...),
 * mode 1 = any hit (returns 1 on first hit).  nodes are padded copies. */
static int traverse(const float* nodes, const float* tri, const uint32_t* order,
                    const ray_pre* r, float tnear, float* bt, uint32_t* bp,
                    uint32_t* bl, float* bu, float* bv, int any,
                    float tfar_any, uint64_t* nnode, uint64_t* ntri) {
  int32_t stack[OR_STACK];
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    const float* nd = nodes + 16 * (size_t)cur;
    ++*nnode;
    float tcut = any ? tfar_any : *bt;
    float tl, tr;
    int hl = slab(r, nd + 0, nd + 3, tnear, tcut, &tl);
    int hr = slab(r, nd + 6, nd + 9, tnear, tcut, &tr);
    int32_t cl, cr;
    memcpy(&cl, nd + 12, 4);
    memcpy(&cr, nd + 13, 4);
    int32_t c0 = cl, c1 = cr;
    int h0 = hl, h1 = hr;
    if (hl && hr && tr < tl) { c0 = cr; c1 = cl; }
    else if (!hl && hr) { c0 = cr; h0 = 1; h1 = 0; }
    int32_t next = 0x7FFFFFFF;
    for (int k = 0; k < 2; ++k) {
      int32_t c = k == 0 ? c0 : c1;
      int h = k == 0 ? h0 : h1;
      if (!h) continue;
      if (c < 0) {
        uint32_t enc = ~(uint32_t)c;
        uint32_t first = enc >> 2, cnt = (enc & 3u) + 1u;
        for (uint32_t q = 0; q < cnt; ++q) {
          ++*ntri;
          float t, u, v;
          uint32_t p = first + q;
          if (!tri_test(r->o, r->d, tnear, tri + 12 * (size_t)p, &t, &u, &v))
            continue;
          if (any) {
            if (t <= tfar_any) return 1;
          } else if (ch_better(t, order[p], *bt, *bp)) {
            *bt = t; *bp = order[p]; *bl = p; *bu = u; *bv = v;
          }
        }
      } else if (next == 0x7FFFFFFF) {
        next = c;
      } else {
        stack[sp++] = c;
      }
    }
    if (next == 0x7FFFFFFF) {
      if (sp == 0) break;
      next = stack[--sp];
    }
    cur = next;
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* standalone BVH API (single domain, prim ids = original face ids)    */
/* ------------------------------------------------------------------ */
static float* padded_nodes(const or_bvh* b) {
  float* nd = (float*)malloc((b->nnodes ? b->nnodes : 1) * 16 * sizeof(float));
  memcpy(nd, b->nodes, b->nnodes * 16 * sizeof(float));
  for (size_t i = 0; i < b->nnodes; ++i) {
    float* x = nd + 16 * i;
    if (isfinite(x[0]) && isfinite(x[3])) pad_box(x + 0, x + 0);
    if (isfinite(x[6]) && isfinite(x[9])) pad_box(x + 6, x + 6);
  }
  return nd;
}

void or_bvh_intersect(const or_bvh* b, const float* org, const float* dir,
                      const float* tnear, const float* tfar, size_t n,
                      float* t_out, float* u_out, float* v_out,
                      uint32_t* prim_out, or_counts* cnt) {
  float* nodes = padded_nodes(b);
  uint64_t tn = 0, tt = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tn, tt)
  for (long i = 0; i < (long)n; ++i) {
    ray_pre r;
    ray_prep(&r, org + 3 * i, dir + 3 * i);
    float bt = tfar ? tfar[i] : OR_INF, bu = 0, bv = 0;
    uint32_t bp = 0xFFFFFFFFu, bl = 0;
    uint64_t a = 0, c = 0;
    if (b->nnodes)
      traverse(nodes, b->tri, b->order, &r, tnear ? tnear[i] : OR_RAY_EPSILON,
               &bt, &bp, &bl, &bu, &bv, 0, 0.0f, &a, &c);
    tn += a;
    tt += c;
    t_out[i] = bt;
    u_out[i] = bu;
    v_out[i] = bv;
    prim_out[i] = bp;
  }
  free(nodes);
  if (cnt) {
    cnt->nodes = tn; cnt->tris = tt; cnt->visits = n; cnt->rays = n;
  }
}

void or_bvh_occluded(const or_bvh* b, const float* org, const float* dir,
                     const float* tnear, const float* tfar, size_t n,
                     uint8_t* occ, or_counts* cnt) {
  float* nodes = padded_nodes(b);
  uint64_t tn = 0, tt = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tn, tt)
  for (long i = 0; i < (long)n; ++i) {
    ray_pre r;
    ray_prep(&r, org + 3 * i, dir + 3 * i);
    uint64_t a = 0, c = 0;
    float bt = 0, bu, bv;
    uint32_t bp = 0, bl = 0;
    occ[i] = b->nnodes ? (uint8_t)traverse(nodes, b->tri, b->order, &r,
                                           tnear ? tnear[i] : OR_RAY_EPSILON,
                                           &bt, &bp, &bl, &bu, &bv, 1,
                                           tfar ? tfar[i] : OR_INF, &a, &c)
                       : 0;
    tn += a;
    tt += c;
  }
  free(nodes);
  if (cnt) {
    cnt->nodes = tn; cnt->tris = tt; cnt->visits = n; cnt->rays = n;
  }
}

/* ------------------------------------------------------------------ */
/* whole scene                                                         */
/* ------------------------------------------------------------------ */
typedef struct {
  or_bvh* bvh;
  float* nodes; /* padded */
  uint32_t* faces;
  uint32_t* colors;
  float* normals;
  size_t nv, nf;
  float box[6];
  int valid;
} or_domain;

struct or_scene {
  int ndom;
  or_domain* d;
  float* boxes; /* [ndom][6] */
};

or_scene* or_scene_create(int ndomains) {
  or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
  s->ndom = ndomains;
  s->d = (or_domain*)calloc((size_t)ndomains, sizeof(or_domain));
  s->boxes = (float*)calloc((size_t)ndomains * 6, sizeof(float));
  for (int i = 0; i < ndomains; ++i) {
    /* empty box until set: never hit */
    s->boxes[6 * i + 0] = s->boxes[6 * i + 1] = s->boxes[6 * i + 2] = 1.0f;
    s->boxes[6 * i + 3] = s->boxes[6 * i + 4] = s->boxes[6 * i + 5] = -1.0f;
  }
  return s;
}

void or_scene_free(or_scene* s) {
  if (!s) return;
  for (int i = 0; i < s->ndom; ++i) {
    or_bvh_free(s->d[i].bvh);
    free(s->d[i].nodes); free(s->d[i].faces); free(s->d[i].colors);
    free(s->d[i].normals);
  }
  free(s->d); free(s->boxes); free(s);
}

int or_scene_set_domain(or_scene* s, int id, const float* v, size_t nv,
                        const uint32_t* f, size_t nf, const uint32_t* colors,
                        const float* normals, const float box[6]) {
  if (id < 0 || id >= s->ndom) return -1;
  or_domain* d = &s->d[id];
  or_bvh_free(d->bvh);
  free(d->nodes); free(d->faces); free(d->colors); free(d->normals);
  d->bvh = or_bvh_build(v, f, nf);
  d->nodes = padded_nodes(d->bvh);
  d->nv = nv;
  d->nf = nf;
  d->faces = (uint32_t*)malloc((nf ? nf : 1) * 3 * sizeof(uint32_t));
  memcpy(d->faces, f, nf * 3 * sizeof(uint32_t));
  d->colors = (uint32_t*)malloc((nv ? nv : 1) * sizeof(uint32_t));
  memcpy(d->colors, colors, nv * sizeof(uint32_t));
  d->normals = (float*)malloc((nv ? nv : 1) * 3 * sizeof(float));
  memcpy(d->normals, normals, nv * 3 * sizeof(float));
  memcpy(d->box, box, 6 * sizeof(float));
  memcpy(s->boxes + 6 * id, box, 6 * sizeof(float));
  d->valid = 1;
  return 0;
}

/* A domain of the partition that another rank owns: its box takes part in
 * the domain lists (every rank builds the same lists), its mesh is absent. */
int or_scene_set_box(or_scene* s, int id, const float box[6]) {
  if (id < 0 || id >= s->ndom) return -1;
  memcpy(s->d[id].box, box, 6 * sizeof(float));
  memcpy(s->boxes + 6 * id, box, 6 * sizeof(float));
  return 0;
}

/* TriMeshBuffer::updateIntersection, src/render/trimesh_buffer.cc:328-360:
 * color channels (uint) * float weights, summed w,u,v order, truncated;
 * Ns from unnormalised vertex normals. */
static void epilogue(const or_domain* d, uint32_t prim, float u, float v,
                     or_hit* h) {
  const uint32_t* fc = d->faces + 3 * (size_t)prim;
  uint32_t c0 = d->colors[fc[0]], c1 = d->colors[fc[1]], c2 = d->colors[fc[2]];
  float w = 1.f - u - v;
  uint32_t ch[3];
  for (int k = 0; k < 3; ++k) {
    int sh = 16 - 8 * k;
    float a = (float)((c0 >> sh) & 0xffu), b = (float)((c1 >> sh) & 0xffu),
          c = (float)((c2 >> sh) & 0xffu);
    ch[k] = (uint32_t)((a * w + b * u) + c * v);
  }
  h->color = (ch[0] << 16) | (ch[1] << 8) | ch[2];
  const float* n0 = d->normals + 3 * (size_t)fc[0];
  const float* n1 = d->normals + 3 * (size_t)fc[1];
  const float* n2 = d->normals + 3 * (size_t)fc[2];
  for (int k = 0; k < 3; ++k) h->ns[k] = (n0[k] * w + n1[k] * u) + n2[k] * v;
}

void or_epilogue(const uint32_t* faces, const uint32_t* colors,
                 const float* normals, const uint32_t* prim, const float* u,
                 const float* v, size_t n, uint32_t* color_out, float* ns_out) {
  or_domain d;
  memset(&d, 0, sizeof(d));
  d.faces = (uint32_t*)faces;
  d.colors = (uint32_t*)colors;
  d.normals = (float*)normals;
  for (size_t i = 0; i < n; ++i) {
    if (prim[i] == 0xFFFFFFFFu) continue;
    or_hit h;
    epilogue(&d, prim[i], u[i], v[i], &h);
    color_out[i] = h.color;
    ns_out[3 * i] = h.ns[0];
    ns_out[3 * i + 1] = h.ns[1];
    ns_out[3 * i + 2] = h.ns[2];
  }
}

void or_scene_intersect(const or_scene* s, const float* org, const float* dir,
                        size_t n, or_hit* hits, or_counts* cnt, int nthreads) {
  uint64_t tn = 0, tt = 0, tv = 0;
#ifdef _OPENMP
  int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(nt) reduction(+ : tn, tt, tv)
#endif
  for (long i = 0; i < (long)n; ++i) {
    int32_t ids[64];
    float ts[64];
    int over = 0;
    int maxh = s->ndom < 64 ? s->ndom : 64;
    int c = domain_list(s->boxes, s->ndom, org + 3 * i, dir + 3 * i, maxh, ids,
                        ts, &over);
    ray_pre r;
    ray_prep(&r, org + 3 * i, dir + 3 * i);
    float bt = OR_INF, bu = 0, bv = 0;
    int bd = -1;
    uint32_t bpl = 0, bpo = 0xFFFFFFFFu;
    uint64_t a = 0, b = 0;
    for (int k = 0; k < c; ++k) {
      const or_domain* d = &s->d[ids[k]];
      if (!d->valid || d->bvh->nnodes == 0) continue;
      /* carried tfar: once a hit exists a later list entry must be strictly
       * nearer (earlier entry wins a tie): prim sentinel 0 makes ch_better
       * strict. */
      float lt = bt, lu = 0, lv = 0;
      uint32_t lp = bd >= 0 ? 0u : 0xFFFFFFFFu, ll = 0;
      traverse(d->nodes, d->bvh->tri, d->bvh->order, &r, OR_RAY_EPSILON, &lt,
               &lp, &ll, &lu, &lv, 0, 0.0f, &a, &b);
      ++tv;
      if (lt < bt || (bd < 0 && lp != 0xFFFFFFFFu)) {
        bt = lt; bu = lu; bv = lv; bd = ids[k]; bpl = ll; bpo = lp;
      }
    }
    tn += a;
    tt += b;
    or_hit* h = hits + i;
    if (bd < 0) {
      h->t = OR_INF; h->u = 0; h->v = 0; h->prim = 0xFFFFFFFFu;
      h->ng[0] = h->ng[1] = h->ng[2] = 0;
      h->color = 0;
      h->ns[0] = h->ns[1] = h->ns[2] = 0;
      h->domain = -1;
    } else {
      const or_domain* d = &s->d[bd];
      const float* tr = d->bvh->tri + 12 * (size_t)bpl;
      h->t = bt; h->u = bu; h->v = bv;
      h->prim = bpo;
      h->ng[0] = tr[9]; h->ng[1] = tr[10]; h->ng[2] = tr[11];
      h->domain = bd;
      epilogue(d, h->prim, bu, bv, h);
    }
  }
  if (cnt) {
    cnt->nodes = tn; cnt->tris = tt; cnt->visits = tv; cnt->rays = n;
  }
}

void or_scene_occluded(const or_scene* s, const float* org, const float* dir,
                       size_t n, uint8_t* occ, or_counts* cnt, int nthreads) {
  uint64_t tn = 0, tt = 0, tv = 0;
#ifdef _OPENMP
  int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(nt) reduction(+ : tn, tt, tv)
#endif
  for (long i = 0; i < (long)n; ++i) {
    int32_t ids[64];
    float ts[64];
    int over = 0;
    int maxh = s->ndom < 64 ? s->ndom : 64;
    int c = domain_list(s->boxes, s->ndom, org + 3 * i, dir + 3 * i, maxh, ids,
                        ts, &over);
    ray_pre r;
    ray_prep(&r, org + 3 * i, dir + 3 * i);
    uint64_t a = 0, b = 0;
    uint8_t o = 0;
    for (int k = 0; k < c && !o; ++k) {
      const or_domain* d = &s->d[ids[k]];
      if (!d->valid || d->bvh->nnodes == 0) continue;
      float bt = 0, bu, bv;
      uint32_t bp = 0, bl = 0;
      o = (uint8_t)traverse(d->nodes, d->bvh->tri, d->bvh->order, &r,
                            OR_RAY_EPSILON, &bt, &bp, &bl, &bu, &bv, 1, OR_INF,
                            &a, &b);
      ++tv;
    }
    tn += a;
    tt += b;
    occ[i] = o;
  }
  if (cnt) {
    cnt->nodes = tn; cnt->tris = tt; cnt->visits = tv; cnt->rays = n;
  }
}

/* ------------------------------------------------------------------ */
/* shadow-ray spawn (caller side of the hot path)                      */
/* ------------------------------------------------------------------ */

/* ooc::ShaderPt::operator(), src/ooc/ooc_shader_pt.h:93-171, point light
 * branch for a camera ray (Lin = 1): pos = dir*t + org, normal_ff faces wo,
 * wi = normalize(light - pos), Lr = blinnPhong(...) (reflection.h:202-214),
 * spawn iff hasPositive(Lr) (utils/math.h:76-78). */
size_t or_spawn_shadows_pt(const float* org, const float* dir,
                           const or_hit* hits, size_t n,
                           const float lp[3], const float lr[3],
                           const float ks[3], float shininess, float* sorg,
                           float* sdir, int32_t* src) {
  size_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    const or_hit* h = hits + i;
    if (h->domain < 0) continue;
    const float* o = org + 3 * i;
    const float* d = dir + 3 * i;
    f3 pos = mk3(d[0] * h->t + o[0], d[1] * h->t + o[1], d[2] * h->t + o[2]);
    /* util::unpack(uint32, vec3&): channel * SPRAY_1_OVER_255 (a double) */
    f3 kd = mk3((float)((double)((h->color >> 16) & 0xff) * 0.00392156862745098),
                (float)((double)((h->color >> 8) & 0xff) * 0.00392156862745098),
                (float)((double)(h->color & 0xff) * 0.00392156862745098));
    f3 normal = mk3(h->ns[0], h->ns[1], h->ns[2]);
    f3 wo = mk3(-d[0], -d[1], -d[2]);
    float cos_i = gdot(wo, normal);
    f3 nff = cos_i > 0.0f ? normal : mk3(-normal.x, -normal.y, -normal.z);
    nff = gnorm(nff);
    f3 wi = gnorm(sub3(mk3(lp[0], lp[1], lp[2]), pos));
    float costheta = clampf(gdot(nff, wi), 0.0f, 1.0f);
    f3 hh = gnorm(add3(wi, wo));
    float ndh = clampf(gdot(nff, hh), 0.0f, 1.0f);
    float pw = powf(ndh, shininess);
    float L[3];
    float kdv[3] = {kd.x, kd.y, kd.z};
    for (int k = 0; k < 3; ++k) {
      float cs = ks[k] * pw, cd = kdv[k] * costheta;
      L[k] = (lr[k] * (cd + cs)) * (1.0f / 1.0f);
    }
    if (!(L[0] > 0.0f || L[1] > 0.0f || L[2] > 0.0f)) continue;
    sorg[3 * m] = pos.x; sorg[3 * m + 1] = pos.y; sorg[3 * m + 2] = pos.z;
    sdir[3 * m] = wi.x; sdir[3 * m + 1] = wi.y; sdir[3 * m + 2] = wi.z;
    if (src) src[m] = (int32_t)i;
    ++m;
  }
  return m;
}

/* getCosineHemisphereSample (render/sampler.cc:54-60): ConcentricDiskSampling
 * (sampler.h:49-92; theta *= SPRAY_PI / 4.f is a double product, M_PI being
 * a double), cosineHemisphereSample (sampler.h:112-120), localToWorld
 * (sampler.h:101-110), cosineHemispherePdf (sampler.h:126-128).  glm calls
 * cosf/sinf; here cos/sin are evaluated in double and rounded once, which
 * the GPU path reproduces bit for bit (the two may differ from glibc's cosf
 * by an ulp on rare arguments). */
static void cosine_hemisphere(float u1, float u2, f3 N, f3* wi, float* pdf) {
  float sx = 2 * u1 - 1, sy = 2 * u2 - 1, rr, th, dx, dy;
  if (sx == 0.0f && sy == 0.0f) {
    dx = 0.0f; dy = 0.0f;
  } else {
    if (sx >= -sy) {
      if (sx > sy) { rr = sx; th = sy > 0.0f ? sy / rr : 8.0f + sy / rr; }
      else { rr = sy; th = 2.0f - sx / rr; }
    } else {
      if (sx <= sy) { rr = -sx; th = 4.0f - sy / rr; }
      else { rr = -sy; th = 6.0f + sx / rr; }
    }
    th = (float)((double)th * (3.14159265358979323846 / 4.0));
    dx = rr * (float)cos((double)th);
    dy = rr * (float)sin((double)th);
  }
  f3 lv = mk3(dx, dy, sqrtf(fmaxf(0.f, (1.f - dx * dx) - dy * dy)));
  lv = gnorm(lv);
  f3 dx0 = mk3(0, N.z, -N.y), dx1 = mk3(-N.z, 0, N.x);
  f3 ax = gnorm(gdot(dx0, dx0) > gdot(dx1, dx1) ? dx0 : dx1);
  f3 ay = gnorm(gcross(N, ax));
  f3 w = mk3((ax.x * lv.x + ay.x * lv.y) + N.x * lv.z,
             (ax.y * lv.x + ay.y * lv.y) + N.y * lv.z,
             (ax.z * lv.x + ay.z * lv.y) + N.z * lv.z);
  *wi = gnorm(w);
  *pdf = lv.z * 0.3183098861837907f;
}

static inline f3 unpack_rgb(uint32_t c) {
  /* util::unpack(uint32, vec3&): channel * SPRAY_1_OVER_255 (a double) */
  return mk3((float)((double)((c >> 16) & 0xff) * 0.00392156862745098),
             (float)((double)((c >> 8) & 0xff) * 0.00392156862745098),
             (float)((double)(c & 0xff) * 0.00392156862745098));
}

/* ooc::ShaderAo, src/ooc/ooc_shader_ao.h:120-146 with DiffuseBsdf::
 * sampleRandom (reflection.h:245-249) and cosine_hemisphere above. */
size_t or_spawn_shadows_ao(const float* org, const float* dir,
                           const int32_t* pixid, const or_hit* hits, size_t n,
                           int nsamples, float* sorg, float* sdir,
                           int32_t* src) {
  size_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    const or_hit* h = hits + i;
    if (h->domain < 0) continue;
    const float* o = org + 3 * i;
    const float* d = dir + 3 * i;
    f3 pos = mk3(d[0] * h->t + o[0], d[1] * h->t + o[1], d[2] * h->t + o[2]);
    f3 kd = unpack_rgb(h->color);
    f3 normal = mk3(h->ns[0], h->ns[1], h->ns[2]);
    f3 wo = mk3(-d[0], -d[1], -d[2]);
    float cos_i = gdot(wo, normal);
    f3 N = cos_i > 0.0f ? normal : mk3(-normal.x, -normal.y, -normal.z);
    N = gnorm(N);
    float ao_w = 1.0f / (float)nsamples;
    for (int l = 0; l < nsamples; ++l) {
      uint32_t st = or_sampler_init1(pixid[i] * (l + 1));
      float u1 = or_sampler_get1d(&st), u2 = or_sampler_get1d(&st);
      f3 w;
      float pdf;
      cosine_hemisphere(u1, u2, N, &w, &pdf);
      float costheta = clampf(gdot(N, w), 0.0f, 1.0f);
      float kdv[3] = {kd.x, kd.y, kd.z};
      int pos_any = 0;
      for (int k = 0; k < 3; ++k) {
        float Lr = kdv[k] * (0.3183098861837907f * costheta * ao_w / pdf);
        if (Lr > 0.0f) pos_any = 1;
      }
      if (!pos_any) continue;
      sorg[3 * m] = pos.x; sorg[3 * m + 1] = pos.y; sorg[3 * m + 2] = pos.z;
      sdir[3 * m] = w.x; sdir[3 * m + 1] = w.y; sdir[3 * m + 2] = w.z;
      if (src) src[m] = (int32_t)i;
      ++m;
    }
  }
  return m;
}

/* ------------------------------------------------------------------ */
/* path shading + film (callers of the hot path) */
/* ------------------------------------------------------------------ */

int or_shadow_slots(const or_shader* P) {
  if (P->shader == OR_SHADER_AO) return P->samples;
  int k = 0;
  for (int l = 0; l < P->nlights; ++l)
    k += P->lights[l].type == OR_LIGHT_HEMISPHERE ? P->samples : 1;
  return k;
}

static inline int has_pos(f3 v) { return v.x > 0.0f || v.y > 0.0f || v.z > 0.0f; }

/* blinnPhong, render/reflection.h:202-214 (glm::pow rounded once from
 * double, as cos/sin above) */
static f3 blinn_phong(float costheta, f3 kd, const float ks[3], float shin, f3 li,
                      f3 wi, f3 n, f3 wo) {
  f3 hh = gnorm(add3(wi, wo));
  float ndh = clampf(gdot(n, hh), 0.0f, 1.0f);
  float pw = (float)pow((double)ndh, (double)shin);
  return mk3(li.x * (kd.x * costheta + ks[0] * pw), li.y * (kd.y * costheta + ks[1] * pw),
             li.z * (kd.z * costheta + ks[2] * pw));
}

/* FrDielectric / Refract, reflection.h:134-172 */
static float fr_dielectric(float cosI, float etaI, float etaT, f3 wo, f3 nff, f3* wt) {
  float sin2I = fmaxf(0.0f, 1.0f - (cosI * cosI));
  float eta = etaI / etaT;
  float sin2T = eta * eta * sin2I;
  if (sin2T >= 1.0f) return 1.0f;
  float cosT = sqrtf(1.0f - sin2T);
  float rparl = ((etaT * cosI) - (etaI * cosT)) / ((etaT * cosI) + (etaI * cosT));
  float rperp = ((etaI * cosI) - (etaT * cosT)) / ((etaI * cosI) + (etaT * cosT));
  float fr = (rparl * rparl + rperp * rperp) / 2.0f;
  float a = eta * cosI - cosT;
  *wt = mk3((eta * -wo.x) + (nff.x * a), (eta * -wo.y) + (nff.y * a), (eta * -wo.z) + (nff.z * a));
  return fr;
}
static int refract_(float cosI, float etaI, float etaT, f3 wo, f3 nff, f3* wt) {
  float sin2I = fmaxf(0.0f, 1.0f - (cosI * cosI));
  float eta = etaI / etaT;
  float sin2T = eta * eta * sin2I;
  if (sin2T >= 1.0f) return 0;
  float cosT = sqrtf(1.0f - sin2T);
  float a = eta * cosI - cosT;
  *wt = mk3((eta * -wo.x) + (nff.x * a), (eta * -wo.y) + (nff.y * a), (eta * -wo.z) + (nff.z * a));
  return 1;
}

/* One shading pass of ooc::ShaderPt (ooc_shader_pt.h:93-227) or
 * ooc::ShaderAo (ooc_shader_ao.h:92-197) over n positional path slots at
 * bounce `bounce` (0 = camera rays; next_actual_depth = bounce + 1 since
 * this restatement resolves every hit exactly, with no speculative
 * history).  Slot i's shadow k lands at i*nshadow + k; its next radiance
 * ray replaces (org, dir) i with valid[i] = 1.  Returns the number of
 * cases the reference aborts on (glass with both reflection and
 * transmission, ooc_shader_pt.h:206-207; AO on a delta BSDF,
 * reflection.h:268-271), which are skipped. */
int or_shade(const or_shader* P, const or_bsdf* bsdf, int nbsdf, int bounce,
             float* org, float* dir, const or_hit* hits, float* w, uint8_t* valid,
             const int32_t* pixid, const int32_t* samid, size_t n, float* sorg,
             float* sdir, float* sw, uint8_t* svalid) {
  const int ns = or_shadow_slots(P);
  const int nad = bounce + 1;
  int bad = 0;
  for (size_t i = 0; i < n; ++i) {
    for (int k = 0; k < ns; ++k) svalid[i * ns + k] = 0;
    if (!valid[i]) continue;
    valid[i] = 0;
    const or_hit* h = hits + i;
    if (h->domain < 0) continue;
    const float* o = org + 3 * i;
    const float* d = dir + 3 * i;
    f3 pos = mk3(d[0] * h->t + o[0], d[1] * h->t + o[1], d[2] * h->t + o[2]);
    f3 kd = unpack_rgb(h->color);
    f3 normal = mk3(h->ns[0], h->ns[1], h->ns[2]);
    f3 wo = mk3(-d[0], -d[1], -d[2]);
    f3 Lin = mk3(w[3 * i], w[3 * i + 1], w[3 * i + 2]);
    float cos_i = gdot(wo, normal);
    int entering = cos_i > 0.0f;
    f3 nff = gnorm(entering ? normal : mk3(-normal.x, -normal.y, -normal.z));
    int bt = (h->domain < nbsdf && bsdf) ? bsdf[h->domain].type : OR_BSDF_DIFFUSE;
    int delta = bt != OR_BSDF_DIFFUSE;
    f3 wi;
    float pdf;
#define EMIT(k, L)                                                         \
  do {                                                                     \
    size_t j_ = i * ns + (k);                                              \
    sorg[3 * j_] = pos.x; sorg[3 * j_ + 1] = pos.y; sorg[3 * j_ + 2] = pos.z; \
    sdir[3 * j_] = wi.x; sdir[3 * j_ + 1] = wi.y; sdir[3 * j_ + 2] = wi.z;  \
    sw[3 * j_] = (L).x; sw[3 * j_ + 1] = (L).y; sw[3 * j_ + 2] = (L).z;     \
    svalid[j_] = 1;                                                        \
  } while (0)
    if (P->shader == OR_SHADER_AO) {
      if (delta) {
        ++bad;
      } else {
        const float ao_w = 1.0f / (float)P->samples;
        for (int l = 0; l < P->samples; ++l) {
          uint32_t st = or_sampler_init1(pixid[i] * (l + 1));
          float u1 = or_sampler_get1d(&st), u2 = or_sampler_get1d(&st);
          cosine_hemisphere(u1, u2, nff, &wi, &pdf);
          float ct = clampf(gdot(nff, wi), 0.0f, 1.0f);
          float s = 0.3183098861837907f * ct * ao_w / pdf;
          f3 L = mk3((Lin.x * kd.x) * s, (Lin.y * kd.y) * s, (Lin.z * kd.z) * s);
          if (has_pos(L)) EMIT(l, L);
        }
      }
    } else if (!delta) {
      uint32_t st = or_sampler_init1(samid[i] * nad);
      int k = 0;
      for (int l = 0; l < P->nlights; ++l) {
        const or_light* lt = P->lights + l;
        f3 li = mk3(lt->radiance[0], lt->radiance[1], lt->radiance[2]);
        if (lt->type == OR_LIGHT_HEMISPHERE) {
          for (int s = 0; s < P->samples; ++s, ++k) {
            float u1 = or_sampler_get1d(&st), u2 = or_sampler_get1d(&st);
            cosine_hemisphere(u1, u2, nff, &wi, &pdf);
            if (pdf > 0.0f) {
              float ct = clampf(gdot(nff, wi), 0.0f, 1.0f);
              f3 bp = blinn_phong(ct, kd, P->ks, P->shininess, li, wi, nff, wo);
              float sc = 1.0f / (pdf * (float)P->samples);
              f3 L = mk3((Lin.x * bp.x) * sc, (Lin.y * bp.y) * sc, (Lin.z * bp.z) * sc);
              if (has_pos(L)) EMIT(k, L);
            }
          }
        } else {
          wi = gnorm(sub3(mk3(lt->pos[0], lt->pos[1], lt->pos[2]), pos));
          pdf = 1.0f;
          float ct = clampf(gdot(nff, wi), 0.0f, 1.0f);
          f3 bp = blinn_phong(ct, kd, P->ks, P->shininess, li, wi, nff, wo);
          float sc = 1.0f / pdf;
          f3 L = mk3((Lin.x * bp.x) * sc, (Lin.y * bp.y) * sc, (Lin.z * bp.z) * sc);
          if (has_pos(L)) EMIT(k, L);
          ++k;
        }
      }
    }
#undef EMIT
    if (nad >= P->bounces) continue;
    f3 won = gnorm(wo);
    f3 nw = mk3(0, 0, 0);
    int emit = 0;
    if (delta) {
      if (cos_i != 0.0f) {
        float c = clampf(cos_i, -1.0f, 1.0f);
        float ac = fabsf(c);
        if (!entering) c = ac;
        int refl = 0, trans = 0;
        float fr = 0.0f;
        f3 wt = mk3(0, 0, 0);
        const float* bp = bsdf[h->domain].p;
        if (bt == OR_BSDF_MIRROR) {
          fr = 1.0f; refl = 1;
        } else if (bt == OR_BSDF_GLASS) {
          float eI = entering ? bp[0] : bp[1], eT = entering ? bp[1] : bp[0];
          fr = fr_dielectric(c, eI, eT, won, nff, &wt);
          if (fr == 1.0f) refl = 1;
          else if (fr == 0.0f) trans = 1;
          else { refl = 1; trans = 1; }
        } else { /* transmission */
          float eI = entering ? bp[0] : bp[1], eT = entering ? bp[1] : bp[0];
          if (refract_(c, eI, eT, won, nff, &wt)) { trans = 1; fr = 0.0f; }
          else { refl = 1; fr = 1.0f; }
        }
        if (refl && trans) {
          ++bad;
        } else if (refl) {
          float s2 = 2.0f * gdot(won, nff);
          wi = gnorm(mk3(-won.x + s2 * nff.x, -won.y + s2 * nff.y, -won.z + s2 * nff.z));
          float s = fr / ac;
          nw = mk3(Lin.x * s, Lin.y * s, Lin.z * s);
          emit = has_pos(nw);
        } else if (trans) {
          wi = gnorm(wt);
          float s = (1.0f - fr) / ac;
          nw = mk3(Lin.x * s, Lin.y * s, Lin.z * s);
          emit = has_pos(nw);
        }
      }
    } else {
      uint32_t st = or_sampler_init1(samid[i] * nad);
      float u1 = or_sampler_get1d(&st), u2 = or_sampler_get1d(&st);
      cosine_hemisphere(u1, u2, nff, &wi, &pdf);
      float ct = clampf(gdot(nff, wi), 0.0f, 1.0f);
      nw = mk3((((Lin.x * kd.x) * 0.3183098861837907f) * ct) / pdf,
               (((Lin.y * kd.y) * 0.3183098861837907f) * ct) / pdf,
               (((Lin.z * kd.z) * 0.3183098861837907f) * ct) / pdf);
      emit = has_pos(nw);
    }
    if (emit) {
      org[3 * i] = pos.x; org[3 * i + 1] = pos.y; org[3 * i + 2] = pos.z;
      dir[3 * i] = wi.x; dir[3 * i + 1] = wi.y; dir[3 * i + 2] = wi.z;
      w[3 * i] = nw.x; w[3 * i + 1] = nw.y; w[3 * i + 2] = nw.z;
      valid[i] = 1;
    }
  }
  return bad;
}

/* TContext::retire (ooc_tcontext.inl:123-135) + HdrImage::add(pixid, rgb,
 * double scale) (display/image.h:90-99): every unoccluded shadow adds
 * scale * w to its pixel (float += double product).  Slots come in pixel
 * groups of spp (the eye-ray layout); within a pixel the adds run in slot
 * order then shadow order -- the reference's order is that of its OpenMP
 * retire loop, which this fixes. */
void or_film(float* image, const int32_t* pixid, size_t n, int spp, int nshadow,
             const float* sw, const uint8_t* svalid, const uint8_t* occ,
             double scale) {
  (void)spp;
  for (size_t i = 0; i < n; ++i) {
    float* px = image + 4 * (size_t)pixid[i];
    for (int k = 0; k < nshadow; ++k) {
      size_t j = i * nshadow + k;
      if (!svalid[j] || occ[j]) continue;
      px[0] = (float)((double)px[0] + scale * (double)sw[3 * j]);
      px[1] = (float)((double)px[1] + scale * (double)sw[3 * j + 1]);
      px[2] = (float)((double)px[2] + scale * (double)sw[3 * j + 2]);
    }
  }
}
