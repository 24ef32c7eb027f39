// insitu_kernels.hip -- gfx950 kernels of the in-situ exchange (insitu.cpp):
// packing rays into the wire records that travel between ranks, the
// composite-key reduction (VBuf::compositeTbuf, src/insitu/insitu_vbuf.h:
// 109-129, done per ray copy), the winner flags, the occlusion OR back at the
// spawner (compositeObuf), the film of the shaded copies
// (TContext::retireShadows + HdrImage::add, insitu_tcontext.inl:232-241) and
// the next bounce's compaction.  All are HBM-bound streaming passes: one
// thread per record, 16-B (or 8-B) accesses.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "cam_device.h"
#include "insitu_kernels.h"
#include "rt_device.h"
#include "shade_device.h"

namespace spray_rt {
namespace {

// 48-B radiance record: org, dir, path weight, pixel, sample.  tnear and
// tfar are not sent: every radiance ray of the reference carries
// SPRAY_RAY_EPSILON and +inf (RTCRayUtil::makeRadianceRay, rays.h:345-363).
__global__ __launch_bounds__(kBlock) void k_pack_rad(const float4* __restrict__ rays,
                                                     const float4* __restrict__ w,
                                                     const int32_t* __restrict__ pix,
                                                     const int32_t* __restrict__ sam,
                                                     const int64_t* __restrict__ idx, size_t n,
                                                     float4* __restrict__ out) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t i = size_t(idx[j]);
  const float4 a = rays[2 * i], b = rays[2 * i + 1];
  const float4 c = w ? w[i] : make_float4(1.f, 1.f, 1.f, 0.f);  // bounce 0: weights (1, 1, 1)
  out[3 * j] = make_float4(a.x, a.y, a.z, b.x);
  out[3 * j + 1] = make_float4(b.y, b.z, c.x, c.y);
  out[3 * j + 2] = make_float4(c.z, __int_as_float(pix[i]), __int_as_float(sam[i]), 0.f);
}

__global__ __launch_bounds__(kBlock) void k_unpack_rad(const float4* __restrict__ in, size_t m,
                                                       float4* __restrict__ rays,
                                                       float4* __restrict__ w,
                                                       int32_t* __restrict__ pix,
                                                       int32_t* __restrict__ sam) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= m) return;
  const float4 a = in[3 * j], b = in[3 * j + 1], c = in[3 * j + 2];
  rays[2 * j] = make_float4(a.x, a.y, a.z, kRayEpsilon);
  rays[2 * j + 1] = make_float4(a.w, b.x, b.y, kInf);
  w[j] = make_float4(b.z, b.w, c.x, 0.f);
  pix[j] = __float_as_int(c.y);
  sam[j] = __float_as_int(c.z);
}

// 24-B shadow record (org, dir; makeShadowRay, rays.h:389-423, sets
// SPRAY_RAY_EPSILON / +inf too), taken from the spawner's slot sel[src[j]].
__global__ __launch_bounds__(kBlock) void k_pack_shadow(const float4* __restrict__ sh,
                                                        const uint32_t* __restrict__ sel,
                                                        const int64_t* __restrict__ idx,
                                                        size_t n, float* __restrict__ out) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t slot = sel ? sel[idx[j]] : size_t(idx[j]);  // sel null: idx are slots
  const float4 a = sh[2 * slot], b = sh[2 * slot + 1];
  float2* o = reinterpret_cast<float2*>(out + 6 * j);
  o[0] = make_float2(a.x, a.y);
  o[1] = make_float2(a.z, b.x);
  o[2] = make_float2(b.y, b.z);
}

__global__ __launch_bounds__(kBlock) void k_unpack_shadow(const float* __restrict__ in, size_t m,
                                                          float4* __restrict__ rays) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= m) return;
  const float2* p = reinterpret_cast<const float2*>(in + 6 * j);
  const float2 a = p[0], b = p[1], c = p[2];
  rays[2 * j] = make_float4(a.x, a.y, b.x, kRayEpsilon);
  rays[2 * j + 1] = make_float4(b.y, c.x, c.y, kInf);
}

// the spawner's slot table of the compacted shadow rays: gathers the route
// input (32-B rays) of slots sel[0..n)
__global__ __launch_bounds__(kBlock) void k_gather_shadow(const float4* __restrict__ sh,
                                                          const uint32_t* __restrict__ sel,
                                                          size_t n, float4* __restrict__ out) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t slot = sel[j];
  out[2 * j] = sh[2 * slot];
  out[2 * j + 1] = sh[2 * slot + 1];
}

// A rank's own copies, gathered from the holder arrays instead of packed,
// sent to itself and unpacked: the records k_unpack_rad / k_unpack_shadow
// would produce (tnear / tfar reset as on the wire).
__global__ __launch_bounds__(kBlock) void k_gather_rad(const float4* __restrict__ rays,
                                                       const float4* __restrict__ w,
                                                       const int32_t* __restrict__ pix,
                                                       const int32_t* __restrict__ sam,
                                                       const int64_t* __restrict__ idx, size_t n,
                                                       float4* __restrict__ orays,
                                                       float4* __restrict__ ow,
                                                       int32_t* __restrict__ opix,
                                                       int32_t* __restrict__ osam) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t i = size_t(idx[j]);
  const float4 a = rays[2 * i], b = rays[2 * i + 1];
  const float4 c = w ? w[i] : make_float4(1.f, 1.f, 1.f, 0.f);
  orays[2 * j] = make_float4(a.x, a.y, a.z, kRayEpsilon);
  orays[2 * j + 1] = make_float4(b.x, b.y, b.z, kInf);
  ow[j] = make_float4(c.x, c.y, c.z, 0.f);
  opix[j] = pix[i];
  osam[j] = sam[i];
}

__global__ __launch_bounds__(kBlock) void k_gather_shadow_self(const float4* __restrict__ sh,
                                                               const uint32_t* __restrict__ sel,
                                                               const int64_t* __restrict__ idx,
                                                               size_t n,
                                                               float4* __restrict__ rays) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t slot = sel ? sel[idx[j]] : size_t(idx[j]);  // sel null: idx are slots
  const float4 a = sh[2 * slot], b = sh[2 * slot + 1];
  rays[2 * j] = make_float4(a.x, a.y, a.z, kRayEpsilon);
  rays[2 * j + 1] = make_float4(b.x, b.y, b.z, kInf);
}

__global__ __launch_bounds__(kBlock) void k_key_min(const int64_t* __restrict__ idx,
                                                    const unsigned long long* __restrict__ keys,
                                                    size_t n,
                                                    unsigned long long* __restrict__ best) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const unsigned long long k = keys[j];
  if (k != kInsituMissKey) atomicMin(best + idx[j], k);
}

__global__ __launch_bounds__(kBlock) void k_fill_u64(unsigned long long* __restrict__ p,
                                                     size_t n, unsigned long long v) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j < n) p[j] = v;
}

__global__ __launch_bounds__(kBlock) void k_winners(const unsigned long long* __restrict__ key,
                                                    const unsigned long long* __restrict__ best,
                                                    size_t m, uint8_t* __restrict__ win) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= m) return;
  const unsigned long long k = key[j];
  win[j] = (k != kInsituMissKey && k == best[j]) ? 1 : 0;
}

// obuf OR at the spawner: any owner that found an occluder marks the slot
__global__ __launch_bounds__(kBlock) void k_occ_return(const int64_t* __restrict__ idx,
                                                       const uint8_t* __restrict__ ret, size_t n,
                                                       const uint32_t* __restrict__ sel,
                                                       uint8_t* __restrict__ occ) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  if (ret[j]) occ[sel ? sel[idx[j]] : size_t(idx[j])] = 1;
}

// HdrImage::add of the unoccluded shadows of the copies this rank shaded
// (copies of one pixel may sit on any rank, so the adds are atomic -- the
// reference's per-rank images are summed by MPI_Reduce too, image.h:167-181).
// One thread per copy sums its ns slots in order; the copies of one pixel
// are neighbours (the spp samples of a pixel travel together), so a
// segmented scan over the wave's runs of equal pixels leaves one hardware
// fp32 atomic per run and channel at the run's last lane.
__device__ __forceinline__ void film_runs(float* __restrict__ image, bool in, int32_t p,
                                          bool any, float a0, float a1, float a2,
                                          int stride = 4) {
  const int lane = threadIdx.x & 63;
  if (__ballot(any) == 0ull) return;
  // runs of equal pixels: heads, and each lane's run start
  const int32_t pp = __shfl_up(p, 1);
  const bool head = lane == 0 || pp != p;
  const uint64_t heads = __ballot(head);
  const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const int start = 63 - __clzll((long long)(heads & le));
  int cnt = any ? 1 : 0;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float b0 = __shfl_up(a0, off), b1 = __shfl_up(a1, off), b2 = __shfl_up(a2, off);
    const int bc = __shfl_up(cnt, off);
    if (lane - off >= start) {
      a0 += b0;
      a1 += b1;
      a2 += b2;
      cnt += bc;
    }
  }
  const bool tail = lane == 63 || ((heads >> (lane + 1)) & 1ull);
  if (in && tail && cnt) {
    float* px = image + size_t(stride) * size_t(p);
    unsafeAtomicAdd(px, a0);
    unsafeAtomicAdd(px + 1, a1);
    unsafeAtomicAdd(px + 2, a2);
  }
}

__global__ __launch_bounds__(kBlock) void k_film_atomic(float* __restrict__ image,
                                                        const int32_t* __restrict__ pix,
                                                        size_t m, int ns,
                                                        const float4* __restrict__ sw,
                                                        const uint8_t* __restrict__ sv,
                                                        const uint8_t* __restrict__ occ,
                                                        double scale, int stride,
                                                        unsigned long long* __restrict__ tot,
                                                        const uint32_t* __restrict__ nsh,
                                                        unsigned long long nrad) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (tot && i == 0) {
    tot[0] = nrad;
    tot[1] = *nsh;
    tot[2] = 0;
  }
  const bool in = i < m;
  const int32_t p = in ? pix[i] : -1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  bool any = false;
  if (in)
    for (int k = 0; k < ns; ++k) {
      const size_t j = i * size_t(ns) + k;
      if (!sv[j] || occ[j]) continue;
      const float4 L = sw[j];
      a0 += float(scale * double(L.x));
      a1 += float(scale * double(L.y));
      a2 += float(scale * double(L.z));
      any = true;
    }
  film_runs(image, in, p, any, a0, a1, a2, stride);
}

__global__ __launch_bounds__(kBlock) void k_record(const uint8_t* __restrict__ win, size_t m,
                                                   int bounce, int ns,
                                                   const int32_t* __restrict__ sam,
                                                   const spray_rt_hit* __restrict__ hits,
                                                   const uint8_t* __restrict__ sv,
                                                   const uint8_t* __restrict__ occ,
                                                   spray_rt_insitu_rec rec) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= m || !win[i]) return;
  const uint32_t k = atomicAdd(rec.d_count, 1u);
  if (k >= rec.cap) return;
  unsigned long long v = 0, o = 0;
  for (int s = 0; s < ns && s < 64; ++s) {
    const size_t j = i * size_t(ns) + s;
    if (sv[j]) v |= 1ull << s;
    if (sv[j] && occ[j]) o |= 1ull << s;
  }
  rec.samid[k] = sam[i];
  rec.bounce[k] = bounce;
  rec.hits[k] = hits[i];
  rec.svalid[k] = v;
  rec.occluded[k] = o;
}

// the samples a bounce of the all-local path shades: live slots that hit
__global__ __launch_bounds__(kBlock) void k_hit_flags(const uint8_t* __restrict__ valid,
                                                      const spray_rt_hit* __restrict__ hits,
                                                      size_t n, uint8_t* __restrict__ win) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  win[i] = ((!valid || valid[i]) && hits[i].domain >= 0) ? 1 : 0;
}

// the next bounce's holder arrays: rays / weights / pixel / sample of the
// copies sel[0..n) that spawned a radiance ray
__global__ __launch_bounds__(kBlock) void k_gather_next(const float4* __restrict__ rays,
                                                        const float4* __restrict__ w,
                                                        const int32_t* __restrict__ pix,
                                                        const int32_t* __restrict__ sam,
                                                        const uint32_t* __restrict__ sel,
                                                        size_t n, float4* __restrict__ orays,
                                                        float4* __restrict__ ow,
                                                        int32_t* __restrict__ opix,
                                                        int32_t* __restrict__ osam) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t i = sel[j];
  orays[2 * j] = rays[2 * i];
  orays[2 * j + 1] = rays[2 * i + 1];
  ow[j] = w[i];
  opix[j] = pix[i];
  osam[j] = sam[i];
}

__global__ __launch_bounds__(kBlock) void k_weights_one(float4* __restrict__ w, size_t n) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j < n) w[j] = make_float4(1.f, 1.f, 1.f, 0.f);
}

// ---- replicated-ray frames (insitu.cpp, trace_replicated) ----------------
// Every rank holds the frame's eye rays; C = the rays whose domain list is
// not empty (the same ascending list on every rank), L = the rays with a
// domain of this rank on their list.
// *out = max(v[0..n)), one block
__global__ __launch_bounds__(1024) void k_max_u32(const uint32_t* __restrict__ v, size_t n,
                                                  uint32_t* __restrict__ out) {
  __shared__ uint32_t part[1024 / 64];
  uint32_t m = 0;
  for (size_t k = threadIdx.x; k < n; k += 1024) m = max(m, v[k]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, uint32_t(__shfl_xor(int(m), off)));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (int w = 0; w < 1024 / 64; ++w) b = max(b, part[w]);
    *out = b;
  }
}

// The frame totals as bits (byte 64 c + k = bit k of total c) behind the
// occlusion bytes: one SUM all-reduce of bytes adds them up exactly (a
// byte sums at most `world` ones).
__global__ void k_rep_totals(uint8_t* __restrict__ tail, unsigned long long nrad,
                             const unsigned long long* __restrict__ nshadow) {
  const int k = threadIdx.x;  // 192 threads
  const int c = k >> 6, b = k & 63;
  unsigned long long v = c == 0 ? nrad : 0ull;
  if (c == 1)
    for (int q = 0; q < kWinCounters; ++q) v += nshadow[size_t(q) * kWinStride];
  tail[k] = uint8_t((v >> b) & 1ull);
}


// ---- replicated-ray AO frames (insitu.cpp, trace_replicated_ao) ----------
// After the key MIN all-reduce: the winner of ray j of C publishes its hit's
// shading normal and colour (the rest of the group contributes zeros to the
// SUM all-reduce that follows), and every rank gathers C's rays, pixels and
// samples.
__global__ __launch_bounds__(kBlock) void k_rep_ao_publish(RepAoArgs A) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= A.nc) return;
  const uint32_t i = A.idx_c[j];
  const uint64_t key = A.keys_c[j];
  const bool win = key != kInsituMissKey && A.keys_n[j] == key;
  uint4 pub = make_uint4(0u, 0u, 0u, 0u);
  if (win) {
    const spray_rt_hit h = A.hits_n[j];
    pub = make_uint4(__float_as_uint(h.ns[0]), __float_as_uint(h.ns[1]),
                     __float_as_uint(h.ns[2]), h.color);
    if (A.hit_c) A.hit_c[j] = h;
  }
  A.pub[j] = pub;
  A.win[j] = win;
  A.rays_c[2 * j] = A.rays[2 * size_t(i)];
  A.rays_c[2 * j + 1] = A.rays[2 * size_t(i) + 1];
  A.pix_c[j] = A.pix[i];
  A.sam_c[j] = A.sam[i];
}

// The hit of every ray of C as the whole group sees it after the publish
// all-reduce: t and domain from the winning key, normal and colour from the
// winner -- every field ooc::ShaderAo's spawn reads (ao_ok, ao_sample).
__global__ __launch_bounds__(kBlock) void k_rep_ao_hits(RepAoArgs A) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= A.nc) return;
  const uint64_t key = A.keys_c[j];
  const uint4 pub = A.pub[j];
  const bool hit = key != kInsituMissKey;
  float4* h = reinterpret_cast<float4*>(A.hits_all + j);
  h[0] = make_float4(hit ? __uint_as_float(uint32_t(key >> 32)) : kInf, 0.f, 0.f,
                     __uint_as_float(0xFFFFFFFFu));
  h[1] = make_float4(0.f, 0.f, 0.f, __uint_as_float(pub.w));
  h[2] = make_float4(__uint_as_float(pub.x), __uint_as_float(pub.y), __uint_as_float(pub.z),
                     __int_as_float(hit ? int32_t(key & 0xFFFFull) : -1));
}

// bits[w] bit b = occ[32 w + b] != 0 over [0, n): thread t reads bytes
// [16 t, 16 t + 16) as one 16-B load, and the even thread of each pair writes
// the word of both halves
__global__ __launch_bounds__(kBlock) void k_pack_bits(const uint8_t* __restrict__ occ, size_t n,
                                                      uint32_t* __restrict__ bits) {
  const size_t t = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const size_t b0 = 16 * t;
  uint32_t m = 0;
  if (b0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(occ + b0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) m |= uint32_t(((w[q] >> (8 * j)) & 0xFFu) != 0u) << (4 * q + j);
  } else {
    for (int j = 0; j < 16; ++j)
      if (b0 + j < n && occ[b0 + j]) m |= 1u << j;
  }
  const uint32_t hi = __shfl_down(m, 1);  // every lane of the wave takes part
  if ((t & 1) == 0 && b0 < n) bits[t >> 1] = m | (b0 + 16 < n ? hi << 16 : 0u);
}

__device__ __forceinline__ bool rep_ao_occluded(const uint32_t* __restrict__ fields, size_t pos,
                                                int fb) {
  const uint32_t per = 32u / uint32_t(fb);
  return ((fields[pos / per] >> (uint32_t(pos % per) * uint32_t(fb))) & ((1u << fb) - 1u)) != 0u;
}

// Sample l of ray j of C: ooc::ShaderAo's light weight (frame_kernels.hip,
// k_shade, path weight (1, 1, 1)) from the direction the any-hit lanes
// generated (record + (pixel, l) table: hemisphere_apply, the same bits).
__device__ __forceinline__ void rep_ao_weight(const RepAoArgs& A, size_t j, int32_t px, int l,
                                              const float kd[3], float L[3]) {
  const float4* rc = A.rec_ao + 4 * j;
  const float4 n4 = rc[1], x4 = rc[2], y4 = rc[3];
  const float4 l4 = A.lv[size_t(px) * uint32_t(A.ns) + uint32_t(l)];
  const float N[3] = {n4.x, n4.y, n4.z}, ax[3] = {x4.x, x4.y, x4.z}, ay[3] = {y4.x, y4.y, y4.z};
  const float lv[3] = {l4.x, l4.y, l4.z};
  float wi[3], pdf;
  hemisphere_apply(lv, N, ax, ay, wi, pdf);
  const float ao_w = 1.0f / float(A.ns);
  const float ct = gclamp01(gdot3(N, wi));
  const float s = 0.3183098861837907f * ct * ao_w / pdf;
#pragma unroll
  for (int k = 0; k < 3; ++k) L[k] = (1.0f * kd[k]) * s;
}

// The film of the whole frame on one rank (every AO weight and occlusion is
// known there after the all-reduces): one thread per ray of C, its samples
// in order, the unoccluded ones added (k_film_atomic's sums and atomics).
__global__ __launch_bounds__(kBlock) void k_rep_ao_film(RepAoArgs A, float* __restrict__ image,
                                                        double scale) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const bool in = j < A.nc;
  const int32_t p = in ? A.pix_c[j] : -1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  bool any = false;
  if (in) {
    const spray_rt_hit h = A.hits_all[j];
    if (h.domain >= 0) {
      const spray_rt_ray* ray = reinterpret_cast<const spray_rt_ray*>(A.rays_c) + j;
      float kd[3];
      unpack_rgb(h.color, kd);
      for (int l = 0; l < A.ns; ++l) {
        if (!ao_ok(ray, h, p, l, A.ns)) continue;
        if (rep_ao_occluded(A.fields, j * size_t(A.ns) + l, A.fb)) continue;
        float L[3];
        rep_ao_weight(A, j, p, l, kd, L);
        a0 += float(scale * double(L[0]));
        a1 += float(scale * double(L[1]));
        a2 += float(scale * double(L[2]));
        any = true;
      }
    }
  }
  film_runs(image, in, p, any, a0, a1, a2);
}

// Camera frames: the film of U pixels [q0, q1) (pixel q's slots q spp ..
// q spp + spp - 1, in order, each slot's samples in order) into compact
// (3 floats per U pixel, zero elsewhere); the ranks take disjoint slices and
// the reduce of compact adds zeros, so every pixel's sum is one rank's
// sequential sum whatever the rank count.
__global__ __launch_bounds__(kBlock) void k_rep_ao_film_pix(RepAoArgs A, int spp, size_t q0,
                                                            size_t q1,
                                                            float* __restrict__ compact,
                                                            double scale) {
  const size_t q = q0 + size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (q >= q1) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int sm = 0; sm < spp; ++sm) {
    const size_t j = q * size_t(spp) + size_t(sm);
    if (j >= A.nc) break;
    const spray_rt_hit h = A.hits_all[j];
    if (h.domain < 0) continue;
    const int32_t p = A.pix_c[j];
    const spray_rt_ray* ray = reinterpret_cast<const spray_rt_ray*>(A.rays_c) + j;
    float kd[3];
    unpack_rgb(h.color, kd);
    for (int l = 0; l < A.ns; ++l) {
      if (!ao_ok(ray, h, p, l, A.ns)) continue;
      if (rep_ao_occluded(A.fields, j * size_t(A.ns) + l, A.fb)) continue;
      float L[3];
      rep_ao_weight(A, j, p, l, kd, L);
      a0 += float(scale * double(L[0]));
      a1 += float(scale * double(L[1]));
      a2 += float(scale * double(L[2]));
    }
  }
  compact[3 * q] = a0;
  compact[3 * q + 1] = a1;
  compact[3 * q + 2] = a2;
}

// The same with one lane per slot when spp is a power of two <= 64: a
// pixel's spp neighbouring lanes add their sums by a fixed butterfly, and
// its first lane writes them -- the same bits at every rank count.
__global__ __launch_bounds__(kBlock) void k_rep_ao_film_slots(RepAoArgs A, int spp, size_t q0,
                                                              size_t q1,
                                                              float* __restrict__ compact,
                                                              double scale) {
  const size_t j = q0 * size_t(spp) + size_t(blockIdx.x) * kBlock + threadIdx.x;
  const bool in = j < q1 * size_t(spp) && j < A.nc;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  if (in) {
    const spray_rt_hit h = A.hits_all[j];
    if (h.domain >= 0) {
      const int32_t p = A.pix_c[j];
      const spray_rt_ray* ray = reinterpret_cast<const spray_rt_ray*>(A.rays_c) + j;
      float kd[3];
      unpack_rgb(h.color, kd);
      for (int l = 0; l < A.ns; ++l) {
        if (!ao_ok(ray, h, p, l, A.ns)) continue;
        if (rep_ao_occluded(A.fields, j * size_t(A.ns) + l, A.fb)) continue;
        float L[3];
        rep_ao_weight(A, j, p, l, kd, L);
        a0 += float(scale * double(L[0]));
        a1 += float(scale * double(L[1]));
        a2 += float(scale * double(L[2]));
      }
    }
  }
  for (int o = 1; o < spp; o <<= 1) {
    a0 += __shfl_xor(a0, o);
    a1 += __shfl_xor(a1, o);
    a2 += __shfl_xor(a2, o);
  }
  if (in && j % size_t(spp) == 0) {
    const size_t q = j / size_t(spp);
    compact[3 * q] = a0;
    compact[3 * q + 1] = a1;
    compact[3 * q + 2] = a2;
  }
}

// records of the rays this rank won: the winner's hit record, the spawned
// samples (ao_ok) and the occluded ones
__global__ __launch_bounds__(kBlock) void k_rep_ao_record(RepAoArgs A, spray_rt_insitu_rec rec) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= A.nc || !A.win[j]) return;
  const spray_rt_hit h = A.hits_all[j];
  const spray_rt_ray* ray = reinterpret_cast<const spray_rt_ray*>(A.rays_c) + j;
  const int32_t p = A.pix_c[j];
  unsigned long long v = 0, o = 0;
  for (int l = 0; l < A.ns && l < 64; ++l) {
    if (!ao_ok(ray, h, p, l, A.ns)) continue;
    v |= 1ull << l;
    if (rep_ao_occluded(A.fields, j * size_t(A.ns) + l, A.fb)) o |= 1ull << l;
  }
  const uint32_t k = atomicAdd(rec.d_count, 1u);
  if (k >= rec.cap) return;
  rec.samid[k] = A.sam_c[j];
  rec.bounce[k] = 0;
  rec.hits[k] = A.hit_c[j];
  rec.svalid[k] = v;
  rec.occluded[k] = o;
}

// ---- the compact film of a replicated PT frame -------------------------
// Slots = the runs of equal pixels along C (the spp samples of a pixel are
// neighbours), numbered by an inclusive scan of the run heads.
struct RunHead {  // 1 where ray j of C' starts a run of equal pixels
  const uint32_t* idx_c;
  const int32_t* pix;
  __host__ __device__ uint32_t operator()(uint32_t j) const {
    return (j == 0 || pix[idx_c[j]] != pix[idx_c[j - 1]]) ? 1u : 0u;
  }
};

// slot_c[j] = run of ray j (inclusive count - 1), slot_pix[run] = its pixel,
// *d_np = the number of runs
__global__ __launch_bounds__(kBlock) void k_rep_slot_pix(const uint32_t* __restrict__ idx_c,
                                                         const int32_t* __restrict__ pix,
                                                         const uint32_t* __restrict__ incl,
                                                         size_t nc, int32_t* __restrict__ slot_c,
                                                         int32_t* __restrict__ slot_pix,
                                                         uint32_t* __restrict__ d_np) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= nc) return;
  const uint32_t q = incl[j] - 1u;
  slot_c[j] = int32_t(q);
  const int32_t p = pix[idx_c[j]];
  if (j == 0 || p != pix[idx_c[j - 1]]) slot_pix[q] = p;
  if (j == nc - 1) *d_np = q + 1u;
}

// rank 0: the group's sums of the runs into the image (a pixel on several
// runs gets each run's sum)
__global__ __launch_bounds__(kBlock) void k_rep_expand(float* __restrict__ image,
                                                       const int32_t* __restrict__ slot_pix,
                                                       const float* __restrict__ compact,
                                                       size_t np) {
  const size_t q = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (q >= np) return;
  float* px = image + 4 * size_t(slot_pix[q]);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float v = compact[3 * q + k];
    if (v != 0.0f) unsafeAtomicAdd(px + k, v);
  }
}

// ---- replicated PT frames (insitu.cpp, trace_replicated) ----------------
// C' = the eye rays that enter the scene's bounding box: a superset of the
// rays with a domain on their list (every domain box lies inside it and the
// slab test is monotone in the box when no direction component is zero; a
// ray with one is kept), the same on every rank without a top-level walk.
__global__ __launch_bounds__(kBlock) void k_rep_cull(const float4* __restrict__ rays, size_t n,
                                                     SceneBox b, uint8_t* __restrict__ fc) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const float4 o = rays[2 * i], d = rays[2 * i + 1];
  bool in = d.x == 0.0f || d.y == 0.0f || d.z == 0.0f;
  if (!in) {
    const DRay r = make_dray(o.x, o.y, o.z, d.x, d.y, d.z);
    float tm;
    in = aabb_ref6(b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2], r, tm);
  }
  fc[i] = in;
}

// after the MIN of the t bits: lp[j] = this rank's list position of ray j
// where its t is the minimum, 0xFF elsewhere (list positions < 255)
__global__ __launch_bounds__(kBlock) void k_rep_lp(const uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ tmin, size_t nc,
                                                   uint8_t* __restrict__ lp) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= nc) return;
  const uint64_t key = keys[j];
  const bool cand = key != kInsituMissKey && uint32_t(key >> 32) == tmin[j];
  lp[j] = cand ? uint8_t((key >> 16) & 0xFFu) : uint8_t(0xFF);
}

// a block's winners' shadows (cnt per wave) into its spread counter
__device__ __forceinline__ void win_count(int cnt, unsigned long long* nshadow) {
  __shared__ int part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += part[w];
    if (t) atomicAdd(nshadow + size_t(blockIdx.x % kWinCounters) * kWinStride,
                     (unsigned long long)t);
  }
}

// the winner of ray j: its key's t and list position are the group's minima
// (lpmin null: kmin holds the whole 64-bit minimum key); svw = the winner's
// spawned shadow; *nshadow += this rank's winners' shadows
__global__ __launch_bounds__(kBlock) void k_rep_win(const uint64_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ tmin,
                                                    const uint8_t* __restrict__ lpmin,
                                                    const uint64_t* __restrict__ kmin,
                                                    const uint8_t* __restrict__ sv, size_t nc,
                                                    uint8_t* __restrict__ win,
                                                    uint8_t* __restrict__ svw,
                                                    unsigned long long* __restrict__ nshadow) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  bool w = false, s = false;
  if (j < nc) {
    const uint64_t key = keys[j];
    w = key != kInsituMissKey &&
        (lpmin ? (uint32_t(key >> 32) == tmin[j] && uint8_t((key >> 16) & 0xFFu) == lpmin[j])
               : key == kmin[j]);
    s = w && sv[j];
    win[j] = w;
    svw[j] = s;
  }
  const uint64_t b = __ballot(s);
  win_count(__popcll(b), nshadow);
}

// ---- replicated PT frames from the camera (insitu.cpp, trace_camera) ----
// Every pass runs over the rank's own eye-ray table T (its domains' screen
// footprints; a winner is always among them) and addresses the frame's
// shared arrays by U slot (cam_item).  The arrays over U start prefilled
// (memsets: t bits 0xFFFFFFFF = no hit, list positions 0xFF, occlusion 0).
// lp[u] = this rank's list position of its hit where its t is the group's
// minimum
// Deferred list positions (the keyed launch tested only the rank's boxes):
// the position of the own hit's domain d in the ray's sorted list -- the
// number of domains whose box the ray enters before d's (entry t, then id:
// the keyed epilogue's count, the same exact box tests) -- for the slots
// where the own t is the group's minimum, written to lp and into the key.
// The winners of a wave walk the top-level tree together (nodes by scalar
// fetch, a wave-uniform stack), an inner node only when some lane may enter
// it before its own domain.
typedef float v16f_t __attribute__((ext_vector_type(16)));
__device__ __forceinline__ uint32_t list_pos_wave(uint64_t tlas_u, int32_t* wstk, const Ray& r,
                                                  const DRay& dr, float tb, int bd) {
  const __attribute__((address_space(4))) v16f_t* nodes =
      reinterpret_cast<const __attribute__((address_space(4))) v16f_t*>(tlas_u);
  const float tcut = tb > 0.f ? tb : kInf;  // tb * kTfarSlack < tb below 0
  uint32_t p = 0;
  int sp = 0;
  int32_t cur = 0;
  for (;;) {
    const v16f_t n = nodes[cur];
    const int32_t cl = __builtin_amdgcn_readfirstlane(__float_as_int(n[12]));
    const int32_t cr = __builtin_amdgcn_readfirstlane(__float_as_int(n[13]));
    int32_t next = kNone;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int32_t c = k ? cr : cl;
      if (c == INT_MIN) continue;
      float b6[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) b6[q] = n[6 * k + q];
      float tm;
      if (c < 0) {
        const int b = int(~uint32_t(c) >> 2);
        if (aabb_ref6(b6[0], b6[1], b6[2], b6[3], b6[4], b6[5], dr, tm) &&
            (tm < tb || (tm == tb && b < bd)))
          ++p;
      } else if (__ballot(slab(r, b6[0], b6[1], b6[2], b6[3], b6[4], b6[5], -kInf, tcut, tm))) {
        if (next == kNone) {
          next = c;
        } else {
          wstk[sp] = c;
          ++sp;
        }
      }
    }
    if (next == kNone) {
      if (sp == 0) break;
      --sp;
      next = __builtin_amdgcn_readfirstlane(wstk[sp]);
    }
    cur = next;
  }
  return p;
}

__global__ __launch_bounds__(kBlock) void k_cam_lp(CamTable T, int spp,
                                                   uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ tk,
                                                   const uint32_t* __restrict__ tmin,
                                                   uint8_t* __restrict__ lp, int defer, Cam cam,
                                                   int cam_w, const float* __restrict__ boxes,
                                                   const BvhNode* __restrict__ tlas, int ntlas) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  bool win = false;
  size_t u = 0;
  int x = 0, y = 0, s = 0;
  if (j < size_t(T.npix) * uint32_t(spp)) {
    cam_item(T, spp, j, x, y, s, u);
    const uint32_t t = tk[u];
    win = t != 0xFFFFFFFFu && t == tmin[u];
  }
  if (!win) return;
  uint64_t key = keys[u];
  if (defer && ntlas > 0) {
    float fx, fy, d[3];
    insitu_jitter(cam_w, spp, x, y, s, fx, fy);
    cam_dir(cam, fx, fy, d);
    const Ray r = make_ray(cam.p[0], cam.p[1], cam.p[2], d[0], d[1], d[2]);
    const DRay dr = make_dray(cam.p[0], cam.p[1], cam.p[2], d[0], d[1], d[2]);
    const int bd = int(key & 0xFFFFu);
    float tb;
    aabb_ref(boxes + 6 * bd, dr, tb);
    const uint32_t p = list_pos_wave(reinterpret_cast<uint64_t>(tlas),
                                     wstack + (threadIdx.x >> 6) * kStack, r, dr, tb, bd);
    key = (key & ~(0xFFFFull << 16)) | (uint64_t(p) << 16);
    keys[u] = key;
  }
  lp[u] = uint8_t((key >> 16) & 0xFFu);
}

// the winners among the rank's slots (as k_rep_win): win / svw at u
__global__ __launch_bounds__(kBlock) void k_cam_win(CamTable T, int spp,
                                                    const uint64_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ tk,
                                                    const uint32_t* __restrict__ tmin,
                                                    const uint8_t* __restrict__ lpmin,
                                                    const uint64_t* __restrict__ kmin,
                                                    const uint8_t* __restrict__ sv,
                                                    uint8_t* __restrict__ win,
                                                    uint8_t* __restrict__ svw,
                                                    unsigned long long* __restrict__ nshadow) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  bool w = false, sw = false;
  if (j < size_t(T.npix) * uint32_t(spp)) {
    int x, y, s;
    size_t u;
    cam_item(T, spp, j, x, y, s, u);
    const uint32_t t = tk[u];
    if (t != 0xFFFFFFFFu) {
      const uint64_t key = keys[u];
      w = lpmin ? (t == tmin[u] && uint8_t((key >> 16) & 0xFFu) == lpmin[u]) : key == kmin[u];
    }
    sw = w && sv[u];
    win[u] = w;
    svw[u] = sw;
  }
  win_count(__popcll(__ballot(sw)), nshadow);
}

// the rank's winners' unoccluded shadows into per-U-pixel sums (compact,
// 3 floats per pixel of U; a pixel's spp slots are neighbours, film_runs)
__global__ __launch_bounds__(kBlock) void k_cam_film(CamTable T, int spp,
                                                     float* __restrict__ compact,
                                                     const float4* __restrict__ sw,
                                                     const uint8_t* __restrict__ svw,
                                                     const uint8_t* __restrict__ occ,
                                                     double scale) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const bool in = j < size_t(T.npix) * uint32_t(spp);
  int32_t q = -1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  bool any = false;
  if (in) {
    int x, y, s;
    size_t u;
    cam_item(T, spp, j, x, y, s, u);
    q = int32_t(u / uint32_t(spp));
    if (svw[u] && !occ[u]) {
      const float4 L = sw[u];
      a0 = float(scale * double(L.x));
      a1 = float(scale * double(L.y));
      a2 = float(scale * double(L.z));
      any = true;
    }
  }
  film_runs(compact, in, q, any, a0, a1, a2, 3);
}

// rank 0: the group's per-U-pixel sums into the image (U's own table: U
// pixel q = work item q at one sample per pixel)
__global__ __launch_bounds__(kBlock) void k_cam_expand(CamTable U, int image_w,
                                                       const float* __restrict__ compact,
                                                       float* __restrict__ image) {
  const size_t q = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (q >= U.npix) return;
  int x, y, s;
  size_t u;
  cam_item(U, 1, q, x, y, s, u);
  float* px = image + 4 * (size_t(y) * size_t(image_w) + size_t(x));
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float v = compact[3 * q + k];
    if (v != 0.0f) px[k] += v;
  }
}

// per-sample records of the rank's winners (tests): samid of the blocking
// tile = the frame, (W y + x) spp + s (k_eye_rays_insitu)
__global__ __launch_bounds__(kBlock) void k_cam_record(CamTable T, int spp, int image_w,
                                                       const uint8_t* __restrict__ win,
                                                       const spray_rt_hit* __restrict__ hits,
                                                       const uint8_t* __restrict__ svw,
                                                       const uint8_t* __restrict__ occ,
                                                       spray_rt_insitu_rec rec) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= size_t(T.npix) * uint32_t(spp)) return;
  int x, y, s;
  size_t u;
  cam_item(T, spp, j, x, y, s, u);
  if (!win[u]) return;
  const uint32_t k = atomicAdd(rec.d_count, 1u);
  if (k >= rec.cap) return;
  const int32_t pix = image_w * y + x;
  rec.samid[k] = spp > 1 ? pix * spp + s : pix;
  rec.bounce[k] = 0;
  rec.hits[k] = hits[u];
  rec.svalid[k] = svw[u] ? 1ull : 0ull;
  rec.occluded[k] = (svw[u] && occ[u]) ? 1ull : 0ull;
}

// the eye rays of table T at their U slots (the replicated AO frame's
// inputs): k_eye_rays_insitu's operations, pixid, samid
__global__ __launch_bounds__(kBlock) void k_cam_eye_rays(CamTable T, Cam cam, int image_w, int spp,
                                                         float4* __restrict__ rays,
                                                         int32_t* __restrict__ pixid,
                                                         int32_t* __restrict__ samid) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= size_t(T.npix) * uint32_t(spp)) return;
  int x, y, s;
  size_t u;
  cam_item(T, spp, j, x, y, s, u);
  float fx, fy, d[3];
  insitu_jitter(image_w, spp, x, y, s, fx, fy);
  cam_dir(cam, fx, fy, d);
  rays[2 * u] = make_float4(cam.p[0], cam.p[1], cam.p[2], kRayEpsilon);
  rays[2 * u + 1] = make_float4(d[0], d[1], d[2], kInf);
  const int32_t pix = image_w * y + x;
  pixid[u] = pix;
  samid[u] = spp > 1 ? pix * spp + s : pix;
}

// 64-bit keys: the minimum t bits for the shadow rays
__global__ __launch_bounds__(kBlock) void k_tmin_from_keys(const uint64_t* __restrict__ kmin,
                                                           size_t nc, uint32_t* __restrict__ tmin) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= nc) return;
  const uint64_t k = kmin[j];
  tmin[j] = k != kInsituMissKey ? uint32_t(k >> 32) : 0xFFFFFFFFu;
}

__global__ __launch_bounds__(kBlock) void k_gather_i32(const uint32_t* __restrict__ idx, size_t n,
                                                       const int32_t* __restrict__ src,
                                                       int32_t* __restrict__ dst) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j < n) dst[j] = src[idx[j]];
}

// pixel-id maxima per block of pix[0..n) (then k_max_u32)
__global__ __launch_bounds__(kBlock) void k_pix_bmax(const int32_t* __restrict__ pix, size_t n,
                                                     uint32_t* __restrict__ bmax) {
  __shared__ uint32_t wmax[kBlock / 64];
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  uint32_t px = i < n ? uint32_t(max(pix[i], 0)) : 0u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) px = max(px, uint32_t(__shfl_xor(int(px), off)));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = px;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (int w = 0; w < kBlock / 64; ++w) b = max(b, wmax[w]);
    bmax[blockIdx.x] = b;
  }
}
}  // namespace

#define LAUNCH(n, kern, ...)                                  \
  do {                                                        \
    if ((n) == 0) return hipSuccess;                          \
    kern<<<grid_for(n), kBlock, 0, s>>>(__VA_ARGS__);         \
    return hipGetLastError();                                 \
  } while (0)

hipError_t launch_pack_rad(hipStream_t s, const spray_rt_ray* rays, const float* w,
                           const int32_t* pix, const int32_t* sam, const int64_t* idx, size_t n,
                           void* out) {
  LAUNCH(n, k_pack_rad, reinterpret_cast<const float4*>(rays),
         reinterpret_cast<const float4*>(w), pix, sam, idx, n, static_cast<float4*>(out));
}
hipError_t launch_unpack_rad(hipStream_t s, const void* in, size_t m, spray_rt_ray* rays,
                             float* w, int32_t* pix, int32_t* sam) {
  LAUNCH(m, k_unpack_rad, static_cast<const float4*>(in), m, reinterpret_cast<float4*>(rays),
         reinterpret_cast<float4*>(w), pix, sam);
}
hipError_t launch_pack_shadow(hipStream_t s, const spray_rt_ray* slots, const uint32_t* sel,
                              const int64_t* idx, size_t n, void* out) {
  LAUNCH(n, k_pack_shadow, reinterpret_cast<const float4*>(slots), sel, idx, n,
         static_cast<float*>(out));
}
hipError_t launch_unpack_shadow(hipStream_t s, const void* in, size_t m, spray_rt_ray* rays) {
  LAUNCH(m, k_unpack_shadow, static_cast<const float*>(in), m, reinterpret_cast<float4*>(rays));
}
hipError_t launch_gather_shadow(hipStream_t s, const spray_rt_ray* slots, const uint32_t* sel,
                                size_t n, spray_rt_ray* out) {
  LAUNCH(n, k_gather_shadow, reinterpret_cast<const float4*>(slots), sel, n,
         reinterpret_cast<float4*>(out));
}
hipError_t launch_gather_rad(hipStream_t s, const spray_rt_ray* rays, const float* w,
                             const int32_t* pix, const int32_t* sam, const int64_t* idx, size_t n,
                             spray_rt_ray* orays, float* ow, int32_t* opix, int32_t* osam) {
  LAUNCH(n, k_gather_rad, reinterpret_cast<const float4*>(rays),
         reinterpret_cast<const float4*>(w), pix, sam, idx, n, reinterpret_cast<float4*>(orays),
         reinterpret_cast<float4*>(ow), opix, osam);
}
hipError_t launch_gather_shadow_self(hipStream_t s, const spray_rt_ray* slots,
                                     const uint32_t* sel, const int64_t* idx, size_t n,
                                     spray_rt_ray* out) {
  LAUNCH(n, k_gather_shadow_self, reinterpret_cast<const float4*>(slots), sel, idx, n,
         reinterpret_cast<float4*>(out));
}
hipError_t launch_key_min(hipStream_t s, const int64_t* idx, const uint64_t* keys, size_t n,
                          uint64_t* best) {
  LAUNCH(n, k_key_min, idx, reinterpret_cast<const unsigned long long*>(keys), n,
         reinterpret_cast<unsigned long long*>(best));
}
hipError_t launch_fill_u64(hipStream_t s, uint64_t* p, size_t n, uint64_t v) {
  LAUNCH(n, k_fill_u64, reinterpret_cast<unsigned long long*>(p), n, (unsigned long long)v);
}
hipError_t launch_winners(hipStream_t s, const uint64_t* key, const uint64_t* best, size_t m,
                          uint8_t* win) {
  LAUNCH(m, k_winners, reinterpret_cast<const unsigned long long*>(key),
         reinterpret_cast<const unsigned long long*>(best), m, win);
}
hipError_t launch_occ_return(hipStream_t s, const int64_t* idx, const uint8_t* ret, size_t n,
                             const uint32_t* sel, uint8_t* occ) {
  LAUNCH(n, k_occ_return, idx, ret, n, sel, occ);
}
hipError_t launch_film_atomic(hipStream_t s, float* image, const int32_t* pix, size_t m, int ns,
                              const float* sw, const uint8_t* sv, const uint8_t* occ,
                              double scale, int stride, unsigned long long* tot,
                              const uint32_t* nsh, unsigned long long nrad) {
  if (ns == 0 && !tot) return hipSuccess;
  k_film_atomic<<<std::max(grid_for(m), 1u), kBlock, 0, s>>>(
      image, pix, m, ns, reinterpret_cast<const float4*>(sw), sv, occ, scale, stride, tot, nsh,
      nrad);
  return hipGetLastError();
}
hipError_t launch_record(hipStream_t s, const uint8_t* win, size_t m, int bounce, int ns,
                         const int32_t* sam, const spray_rt_hit* hits, const uint8_t* sv,
                         const uint8_t* occ, const spray_rt_insitu_rec& rec) {
  LAUNCH(m, k_record, win, m, bounce, ns, sam, hits, sv, occ, rec);
}
hipError_t launch_gather_next(hipStream_t s, const spray_rt_ray* rays, const float* w,
                              const int32_t* pix, const int32_t* sam, const uint32_t* sel,
                              size_t n, spray_rt_ray* orays, float* ow, int32_t* opix,
                              int32_t* osam) {
  LAUNCH(n, k_gather_next, reinterpret_cast<const float4*>(rays),
         reinterpret_cast<const float4*>(w), pix, sam, sel, n, reinterpret_cast<float4*>(orays),
         reinterpret_cast<float4*>(ow), opix, osam);
}
hipError_t launch_hit_flags(hipStream_t s, const uint8_t* valid, const spray_rt_hit* hits,
                            size_t n, uint8_t* win) {
  LAUNCH(n, k_hit_flags, valid, hits, n, win);
}
hipError_t launch_weights_one(hipStream_t s, float* w, size_t n) {
  LAUNCH(n, k_weights_one, reinterpret_cast<float4*>(w), n);
}
__global__ __launch_bounds__(kBlock) void k_bands_copy(uint4* __restrict__ image,
                                                       uint4* __restrict__ pk, int W, int bands,
                                                       size_t band16, int r0, size_t n,
                                                       int pack) {
  const size_t idx = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (idx >= n) return;
  const size_t seg = idx / band16, off = idx % band16;
  const size_t i = seg / size_t(bands), j = seg % size_t(bands);
  const size_t rank = size_t(r0) + i;
  const size_t io = (rank + j * size_t(W)) * band16 + off;
  if (pack)
    pk[j * band16 + off] = image[io];
  else
    image[io] = pk[(rank * size_t(bands) + j) * band16 + off];
}
hipError_t launch_bands_copy(hipStream_t s, float* image, void* pk, int W, int bands,
                             size_t band_bytes, int r0, int nr, int pack) {
  if (band_bytes % 16) return hipErrorInvalidValue;
  const size_t band16 = band_bytes / 16;
  const size_t n = size_t(nr) * size_t(bands) * band16;
  LAUNCH(n, k_bands_copy, reinterpret_cast<uint4*>(image), static_cast<uint4*>(pk), W, bands,
         band16, r0, n, pack);
}
__global__ __launch_bounds__(kBlock) void k_pack_rgb(CamTable T, int image_w,
                                                     const float* __restrict__ image,
                                                     float* __restrict__ out, int unpack) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= T.npix) return;
  int x, y, sm;
  size_t slot;
  cam_item(T, 1, j, x, y, sm, slot);
  const size_t px = 4 * (size_t(image_w) * size_t(y) + size_t(x));
  float* im = const_cast<float*>(image);
  if (unpack) {
    im[px] = out[3 * j];
    im[px + 1] = out[3 * j + 1];
    im[px + 2] = out[3 * j + 2];
  } else {
    out[3 * j] = image[px];
    out[3 * j + 1] = image[px + 1];
    out[3 * j + 2] = image[px + 2];
  }
}
hipError_t launch_pack_rgb(hipStream_t s, const CamTable& T, int image_w, const float* image,
                           float* out) {
  LAUNCH(size_t(T.npix), k_pack_rgb, T, image_w, image, out, 0);
}
hipError_t launch_unpack_rgb(hipStream_t s, const CamTable& T, int image_w, const float* in,
                             float* image) {
  LAUNCH(size_t(T.npix), k_pack_rgb, T, image_w, image, const_cast<float*>(in), 1);
}
__global__ void k_totals_of_stats(const unsigned long long* __restrict__ st,
                                  unsigned long long* __restrict__ tot) {
  if (threadIdx.x < 3) tot[threadIdx.x] = st[threadIdx.x == 0 ? 3 : threadIdx.x == 1 ? 1 : 0];
}
hipError_t launch_totals_of_stats(hipStream_t s, const unsigned long long* stats,
                                  unsigned long long* tot) {
  k_totals_of_stats<<<1, 64, 0, s>>>(stats, tot);
  return hipGetLastError();
}
hipError_t launch_rep_totals(hipStream_t s, uint8_t* tail, unsigned long long nrad,
                             const unsigned long long* nshadow) {
  k_rep_totals<<<1, 192, 0, s>>>(tail, nrad, nshadow);
  return hipGetLastError();
}

hipError_t launch_rep_cull(hipStream_t s, const spray_rt_ray* rays, size_t n, const SceneBox& b,
                           uint8_t* fc) {
  LAUNCH(n, k_rep_cull, reinterpret_cast<const float4*>(rays), n, b, fc);
}
hipError_t launch_rep_lp(hipStream_t s, const uint64_t* keys, const uint32_t* tmin, size_t nc,
                         uint8_t* lp) {
  LAUNCH(nc, k_rep_lp, keys, tmin, nc, lp);
}
hipError_t launch_rep_win(hipStream_t s, const uint64_t* keys, const uint32_t* tmin,
                          const uint8_t* lpmin, const uint64_t* kmin, const uint8_t* sv, size_t nc,
                          uint8_t* win, uint8_t* svw, unsigned long long* nshadow) {
  LAUNCH(nc, k_rep_win, keys, tmin, lpmin, kmin, sv, nc, win, svw, nshadow);
}
hipError_t launch_cam_lp(hipStream_t s, const CamTable& T, int spp, uint64_t* keys,
                        const uint32_t* tk, const uint32_t* tmin, uint8_t* lp,
                        const CamFrame* defer, const float* boxes, const BvhNode* tlas,
                        int ntlas) {
  if (defer && (!boxes || !tlas)) return hipErrorInvalidValue;
  Cam cam{};
  if (defer)
    for (int k = 0; k < 14; ++k) cam.p[k] = defer->cam[k];
  LAUNCH(size_t(T.npix) * uint32_t(spp), k_cam_lp, T, spp, keys, tk, tmin, lp, defer ? 1 : 0,
         cam, defer ? defer->image_w : 0, boxes, tlas, ntlas);
}
hipError_t launch_cam_win(hipStream_t s, const CamTable& T, int spp, const uint64_t* keys,
                         const uint32_t* tk, const uint32_t* tmin, const uint8_t* lpmin,
                         const uint64_t* kmin, const uint8_t* sv, uint8_t* win, uint8_t* svw,
                         unsigned long long* nshadow) {
  LAUNCH(size_t(T.npix) * uint32_t(spp), k_cam_win, T, spp, keys, tk, tmin, lpmin, kmin, sv, win,
         svw, nshadow);
}
hipError_t launch_cam_film(hipStream_t s, const CamTable& T, int spp, float* compact,
                          const float* sw, const uint8_t* svw, const uint8_t* occ, double scale) {
  LAUNCH(size_t(T.npix) * uint32_t(spp), k_cam_film, T, spp, compact,
         reinterpret_cast<const float4*>(sw), svw, occ, scale);
}
hipError_t launch_cam_expand(hipStream_t s, const CamTable& U, int image_w, const float* compact,
                            float* image) {
  LAUNCH(size_t(U.npix), k_cam_expand, U, image_w, compact, image);
}
hipError_t launch_cam_record(hipStream_t s, const CamTable& T, int spp, int image_w,
                            const uint8_t* win, const spray_rt_hit* hits, const uint8_t* svw,
                            const uint8_t* occ, const spray_rt_insitu_rec& rec) {
  LAUNCH(size_t(T.npix) * uint32_t(spp), k_cam_record, T, spp, image_w, win, hits, svw, occ, rec);
}
hipError_t launch_cam_eye_rays(hipStream_t s, const CamTable& T, const CamFrame& F,
                              spray_rt_ray* rays, int32_t* pixid, int32_t* samid) {
  Cam cam;
  for (int k = 0; k < 14; ++k) cam.p[k] = F.cam[k];
  LAUNCH(size_t(T.npix) * uint32_t(F.spp), k_cam_eye_rays, T, cam, F.image_w, F.spp,
         reinterpret_cast<float4*>(rays), pixid, samid);
}
hipError_t launch_tmin_from_keys(hipStream_t s, const uint64_t* kmin, size_t nc, uint32_t* tmin) {
  LAUNCH(nc, k_tmin_from_keys, kmin, nc, tmin);
}
hipError_t launch_gather_i32(hipStream_t s, const uint32_t* idx, size_t n, const int32_t* src,
                             int32_t* dst) {
  LAUNCH(n, k_gather_i32, idx, n, src, dst);
}
hipError_t launch_pix_max(hipStream_t s, const int32_t* pix, size_t n, uint32_t* bmax,
                          uint32_t* out) {
  if (n == 0) return hipMemsetAsync(out, 0, 4, s);
  k_pix_bmax<<<grid_for(n), kBlock, 0, s>>>(pix, n, bmax);
  k_max_u32<<<1, 1024, 0, s>>>(bmax, grid_for(n), out);
  return hipGetLastError();
}
hipError_t launch_rep_slots(hipStream_t s, const uint32_t* idx_c, const int32_t* pix, size_t nc,
                            uint32_t* incl, void* temp, size_t* temp_bytes,
                            int32_t* slot_c, int32_t* slot_pix, uint32_t* d_np) {
  // the run heads computed inside the scan's input (no heads pass)
  using Heads = hipcub::TransformInputIterator<uint32_t, RunHead,
                                               hipcub::CountingInputIterator<uint32_t>>;
  const Heads heads(hipcub::CountingInputIterator<uint32_t>(0u), RunHead{idx_c, pix});
  if (!temp) {
    size_t b = 0;
    const hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, b, heads, incl,
                                                          int(std::max<size_t>(nc, 1)), s);
    *temp_bytes = b;
    return e;
  }
  if (nc == 0) return hipMemsetAsync(d_np, 0, 4, s);
  hipError_t e = hipcub::DeviceScan::InclusiveSum(temp, *temp_bytes, heads, incl, int(nc), s);
  if (e != hipSuccess) return e;
  k_rep_slot_pix<<<grid_for(nc), kBlock, 0, s>>>(idx_c, pix, incl, nc, slot_c, slot_pix, d_np);
  return hipGetLastError();
}
hipError_t launch_rep_expand(hipStream_t s, float* image, const int32_t* slot_pix,
                             const float* compact, size_t np) {
  LAUNCH(np, k_rep_expand, image, slot_pix, compact, np);
}
hipError_t launch_rep_ao_publish(hipStream_t s, const RepAoArgs& a) {
  LAUNCH(a.nc, k_rep_ao_publish, a);
}
hipError_t launch_rep_ao_hits(hipStream_t s, const RepAoArgs& a) {
  LAUNCH(a.nc, k_rep_ao_hits, a);
}
hipError_t launch_pack_bits(hipStream_t s, const uint8_t* occ, size_t n, uint32_t* bits) {
  LAUNCH((n + 15) / 16, k_pack_bits, occ, n, bits);
}
hipError_t launch_rep_ao_film(hipStream_t s, const RepAoArgs& a, float* image, double scale) {
  LAUNCH(a.nc, k_rep_ao_film, a, image, scale);
}
hipError_t launch_rep_ao_film_pix(hipStream_t s, const RepAoArgs& a, int spp, size_t q0,
                                  size_t q1, float* compact, double scale) {
  if (spp > 0 && spp <= 64 && (spp & (spp - 1)) == 0) {
    LAUNCH(q1 > q0 ? (q1 - q0) * size_t(spp) : 0, k_rep_ao_film_slots, a, spp, q0, q1, compact,
           scale);
  }
  LAUNCH(q1 > q0 ? q1 - q0 : 0, k_rep_ao_film_pix, a, spp, q0, q1, compact, scale);
}
hipError_t launch_rep_ao_record(hipStream_t s, const RepAoArgs& a,
                                const spray_rt_insitu_rec& rec) {
  LAUNCH(a.nc, k_rep_ao_record, a, rec);
}

}  // namespace spray_rt

namespace spray_rt {
namespace {
__global__ void k_counts_from_starts(const int64_t* __restrict__ starts, int world,
                                     int64_t* __restrict__ counts) {
  const int r = threadIdx.x;
  if (r < world) counts[r] = starts[r + 1] - starts[r];
}
}  // namespace

hipError_t launch_counts_from_starts(hipStream_t s, const int64_t* starts, int world,
                                     int64_t* counts) {
  k_counts_from_starts<<<1, 64, 0, s>>>(starts, world, counts);
  return hipGetLastError();
}

}  // namespace spray_rt
