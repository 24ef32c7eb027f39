// ooc_kernels.hip -- gfx950 kernels of the out-of-core (streamed-domain) path.
//
// The reference's ooc tracer queues every ray to every domain on its sorted
// domain list (ooc_isector.h:116-174) and drains one resident domain at a
// time (ooc_tcontext.inl:28-101) while the LRU cache streams the next ones
// in (lru_cache.cc:65-171).  On the GPU the queues are built in bulk --
// domain masks, (domain, ray) pairs, one stable radix sort -- and each
// batch of resident domains drains its queues in one launch.  A ray's
// closest hit is combined across domains by the order of the sequential
// walk of its domain list, (t, then the list position), so the result is
// the whole-scene one whatever the drain order.
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include "rt_device.h"
#include "rt_kernels.h"

namespace spray_rt {
namespace {

template <int W>
__global__ __launch_bounds__(kBlock) void k_ooc_masks(
    const BvhNode* __restrict__ tlas, int ntlas, const spray_rt_ray* __restrict__ rays,
    const uint8_t* __restrict__ valid, size_t M, uint64_t* __restrict__ masks,
    uint32_t* __restrict__ npairs) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  __shared__ float4 stl[4 * 64 * W];
  for (int k = threadIdx.x; k < 4 * ntlas; k += kBlock) stl[k] = ld4(tlas, k);
  __syncthreads();
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  uint64_t m[W];
#pragma unroll
  for (int w = 0; w < W; ++w) m[w] = 0;
  if (!valid || valid[i]) {
    const float4* rp = reinterpret_cast<const float4*>(rays + i);
    const float4 o4 = rp[0], d4 = rp[1];
    const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
    tlas_mask_wave<W>(stl, ntlas, wstack + (threadIdx.x >> 6) * kStack, r, o4, d4, m);
  }
  uint32_t n = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    masks[i * W + w] = m[w];
    n += __popcll(m[w]);
  }
  npairs[i] = n;
}

// (domain, ray) pair j of ray i at off[i] + k, in ascending domain order
template <int W>
__global__ __launch_bounds__(kBlock) void k_ooc_pairs(const uint64_t* __restrict__ masks,
                                                      const uint32_t* __restrict__ off,
                                                      size_t M, uint16_t* __restrict__ key,
                                                      uint32_t* __restrict__ val) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  uint32_t o = off[i];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = masks[i * W + w];
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      key[o] = uint16_t(64 * w + j);
      val[o] = uint32_t(i);
      ++o;
    }
  }
}

// queue bounds: first[d] = first position of domain d in the sorted keys
__global__ void k_ooc_bounds(const uint16_t* __restrict__ key, uint32_t n, int ndom,
                             uint32_t* __restrict__ first) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d > ndom) return;
  uint32_t lo = 0, hi = n;  // lower_bound(d)
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (int(key[mid]) < d)
      lo = mid + 1;
    else
      hi = mid;
  }
  first[d] = lo;
}

__global__ __launch_bounds__(kBlock) void k_ooc_init(spray_rt_hit* __restrict__ hits,
                                                     uint64_t* __restrict__ key, size_t M) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  float4* hp = reinterpret_cast<float4*>(hits + i);
  hp[0] = make_float4(kInf, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu));
  hp[1] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
  hp[2] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  key[i] = kOocMissKey;
}

// The pair handled by this lane of a batch launch: the waves of segment s
// (one resident domain's queue) are wave0[s] .. wave0[s+1]-1, so a wave
// always walks one domain tree.  Returns the segment, or -1 past the end.
__device__ __forceinline__ int batch_pair(const OocBatch& B, uint32_t& pj, bool& valid) {
  const uint32_t gw = (blockIdx.x * kBlock + threadIdx.x) >> 6;
  if (gw >= B.wave0[B.count]) return -1;
  int s = 0;
  while (s + 1 < B.count && B.wave0[s + 1] <= gw) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  const uint32_t j = (gw - B.wave0[s]) * 64 + (threadIdx.x & 63);
  valid = j < B.n[s];
  pj = B.begin[s] + (valid ? j : 0u);
  return s;
}

// Position of domain `dom` in the ray's sorted domain list (ascending
// (intersectAabb entry t, id), rays.h:71-79): the tie-break of the key.
template <int W>
__device__ __forceinline__ uint32_t list_pos(const uint64_t* m, const float* boxes, int dom,
                                             const DRay& dr) {
  float tb;
  aabb_ref(boxes + 6 * dom, dr, tb);
  uint32_t p = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = m[w];
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      const int b = 64 * w + j;
      float tm;
      aabb_ref(boxes + 6 * b, dr, tm);
      if (tm < tb || (tm == tb && b < dom)) ++p;
    }
  }
  return p;
}

// Closest hit of the rays queued to up to kOocBatch resident domains in one
// launch.  Each (ray, domain) pair walks its domain tree as a packet (a
// queue holds its rays in ascending order: neighbouring pixels) with the
// ray's current best t as the cut, and a hit enters the ray's 64-bit key
// (t bits | list position | domain) by atomicMin.  The key order is the
// sequential walk's winner rule (nearer t, then the earlier list entry) and
// keys are unique per (ray, domain), so the result is the same in any drain
// order and any interleaving.  The pair's own key and winning triangle go
// to pkey / pleaf for k_ooc_ch_resolve.
template <int W>
__global__ __launch_bounds__(kBlock) void k_ooc_ch_batch(
    OocBatch B, const spray_rt_ray* __restrict__ rays, const uint32_t* __restrict__ idx,
    const uint64_t* __restrict__ masks, const float* __restrict__ boxes,
    uint64_t* __restrict__ key, uint64_t* __restrict__ pkey, uint32_t* __restrict__ pleaf) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  uint32_t pj;
  bool valid;
  const int s = batch_pair(B, pj, valid);
  if (s < 0) return;
  const OocDomain& D = B.d[s];
  const uint32_t i = valid ? idx[pj] : 0u;
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  uint64_t k0 = kOocMissKey;
  if (valid) {
    const float4* rp = reinterpret_cast<const float4*>(rays + i);
    o4 = rp[0];
    d4 = rp[1];
    k0 = __hip_atomic_load(key + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  // the domain's own nearest hit with t <= the ray's best so far (ties at
  // that t included: the list position decides them)
  const float tcur = k0 == kOocMissKey ? d4.w : __uint_as_float(uint32_t(k0 >> 32));
  Best best{tcur, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool act = valid, hit = false;
  trace_tree_packet<false>(reinterpret_cast<uint64_t>(D.nodes),
                           reinterpret_cast<uint64_t>(D.tris),
                           reinterpret_cast<uint64_t>(D.prims), r, o4.w, 0.f, best, act, hit,
                           wstack + (threadIdx.x >> 6) * kStack);
  if (!valid) return;
  uint64_t mine = kOocMissKey;
  if (best.leaf != 0xFFFFFFFFu) {
    uint64_t m[W];
#pragma unroll
    for (int w = 0; w < W; ++w) m[w] = masks[size_t(i) * W + w];
    const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
    mine = (uint64_t(__float_as_uint(best.t)) << 32) |
           (uint64_t(list_pos<W>(m, boxes, D.domain, dr)) << 16) | uint64_t(D.domain);
    atomicMin(reinterpret_cast<unsigned long long*>(key + i), (unsigned long long)mine);
  }
  pkey[pj] = mine;
  pleaf[pj] = best.leaf;
}

// Hit records of the batch's winners: the one pair whose key equals its
// ray's minimum runs updateIntersection (trimesh_buffer.cc:328-360) while
// its domain is still resident.  A later batch with a smaller key rewrites
// the record.
__global__ __launch_bounds__(kBlock) void k_ooc_ch_resolve(
    OocBatch B, const spray_rt_ray* __restrict__ rays, const uint32_t* __restrict__ idx,
    const uint64_t* __restrict__ key, const uint64_t* __restrict__ pkey,
    const uint32_t* __restrict__ pleaf, spray_rt_hit* __restrict__ hits) {
  uint32_t pj;
  bool valid;
  const int s = batch_pair(B, pj, valid);
  if (s < 0 || !valid) return;
  const uint64_t mine = pkey[pj];
  if (mine == kOocMissKey) return;
  const uint32_t i = idx[pj];
  if (key[i] != mine) return;
  const OocDomain& D = B.d[s];
  const float4* rp = reinterpret_cast<const float4*>(rays + i);
  const float4 o4 = rp[0], d4 = rp[1];
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  SlotDesc sd{};
  sd.tris = static_cast<const float*>(D.tris);
  sd.faces = D.faces;
  sd.colors = D.colors;
  sd.normals = D.normals;
  const uint32_t leaf = pleaf[pj];
  const uint32_t prim = reinterpret_cast<const GAS uint32_t*>(gptr(D.prims))[leaf];
  float hu, hv;
  const float4 c = hit_uv(sd, r, o4.w, leaf, hu, hv);
  uint32_t color;
  float nsx, nsy, nsz;
  epilogue(sd, prim, hu, hv, color, nsx, nsy, nsz);
  float4* hp = reinterpret_cast<float4*>(hits + i);
  hp[0] = make_float4(__uint_as_float(uint32_t(mine >> 32)), hu, hv, __uint_as_float(prim));
  hp[1] = make_float4(c.y, c.z, c.w, __uint_as_float(color));
  hp[2] = make_float4(nsx, nsy, nsz, __int_as_float(D.domain));
}

// Any hit of the rays queued to the batch's domains, OR-ed into occ (a ray
// already occluded by an earlier batch is skipped; same-batch writers all
// store 1).
__global__ __launch_bounds__(kBlock) void k_ooc_ah_batch(OocBatch B,
                                                         const spray_rt_ray* __restrict__ rays,
                                                         const uint32_t* __restrict__ idx,
                                                         uint8_t* __restrict__ occ) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  uint32_t pj;
  bool ok;
  const int s = batch_pair(B, pj, ok);
  if (s < 0) return;
  const OocDomain& D = B.d[s];
  const uint32_t i = ok ? idx[pj] : 0u;
  const bool valid = ok && !occ[i];
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  if (valid) {
    const float4* rp = reinterpret_cast<const float4*>(rays + i);
    o4 = rp[0];
    d4 = rp[1];
  }
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  Best best{0.f, 0u, 0u};
  bool act = valid, hit = false;
  if (__ballot(act))
    trace_tree_packet<true>(reinterpret_cast<uint64_t>(D.nodes),
                            reinterpret_cast<uint64_t>(D.tris),
                            reinterpret_cast<uint64_t>(D.prims), r, o4.w, d4.w, best, act, hit,
                            wstack + (threadIdx.x >> 6) * kStack);
  if (hit) occ[i] = 1;
}

__global__ __launch_bounds__(kBlock) void k_ooc_clear_occ(const uint8_t* __restrict__ valid,
                                                          uint8_t* __restrict__ occ, size_t M) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < M && (!valid || valid[i])) occ[i] = 0;
}

}  // namespace

hipError_t launch_ooc_queues(hipStream_t s, const BvhNode* tlas, int ntlas, int ndom,
                             const spray_rt_ray* rays, const uint8_t* valid, size_t M,
                             OocScratch& q, uint32_t* h_first) {
  if (ndom <= 0 || ndom > 256 || M > 0xFFFFFFFFull) return hipErrorInvalidValue;
  const int W = ndom <= 64 ? 1 : 4;
  const unsigned g = grid_for(M);
  hipError_t e0 = hipMemsetAsync(q.npairs + M, 0, sizeof(uint32_t), s);
  if (e0 != hipSuccess) return e0;
  if (W == 1)
    k_ooc_masks<1><<<g, kBlock, 0, s>>>(tlas, ntlas, rays, valid, M, q.masks, q.npairs);
  else
    k_ooc_masks<4><<<g, kBlock, 0, s>>>(tlas, ntlas, rays, valid, M, q.masks, q.npairs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // pair offsets: exclusive scan of the per-ray counts (+ total at [M])
  size_t tb = q.temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(q.temp, tb, q.npairs, q.poff, int(M + 1), s);
  if (e != hipSuccess) return e;
  uint32_t total = 0;
  e = hipMemcpyAsync(&total, q.poff + M, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  q.npair = total;
  if (total > q.pair_cap) return hipErrorOutOfMemory;  // caller grows and retries
  if (total) {
    if (W == 1)
      k_ooc_pairs<1><<<g, kBlock, 0, s>>>(q.masks, q.poff, M, q.key_in, q.val_in);
    else
      k_ooc_pairs<4><<<g, kBlock, 0, s>>>(q.masks, q.poff, M, q.key_in, q.val_in);
    int end_bit = 1;
    while ((1 << end_bit) < ndom) ++end_bit;
    tb = q.temp_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(q.temp, tb, q.key_in, q.key_out, q.val_in,
                                           q.val_out, int(total), 0, end_bit, s);
    if (e != hipSuccess) return e;
  }
  k_ooc_bounds<<<(ndom + 1 + 63) / 64, 64, 0, s>>>(q.key_out, total, ndom, q.first);
  e = hipMemcpyAsync(h_first, q.first, (ndom + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                     s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e;
}

size_t ooc_temp_bytes(size_t M, size_t pairs) {
  // size queries only; a failed query leaves 0, and the launch that needs the
  // scratch then reports its error
  size_t a = 0, b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, a, static_cast<uint32_t*>(nullptr),
                                       static_cast<uint32_t*>(nullptr),
                                       int(M + 1)) != hipSuccess)
    a = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, static_cast<uint16_t*>(nullptr),
                                         static_cast<uint16_t*>(nullptr),
                                         static_cast<uint32_t*>(nullptr),
                                         static_cast<uint32_t*>(nullptr), int(pairs), 0,
                                         8) != hipSuccess)
    b = 0;
  return a > b ? a : b;
}

hipError_t launch_ooc_init(hipStream_t s, spray_rt_hit* hits, uint64_t* key, size_t M) {
  if (M == 0) return hipSuccess;
  k_ooc_init<<<grid_for(M), kBlock, 0, s>>>(hits, key, M);
  return hipGetLastError();
}

static unsigned batch_grid(OocBatch& B) {
  B.wave0[0] = 0;
  for (int k = 0; k < B.count; ++k) B.wave0[k + 1] = B.wave0[k] + (B.n[k] + 63) / 64;
  return (B.wave0[B.count] + kBlock / 64 - 1) / (kBlock / 64);
}

hipError_t launch_ooc_ch_batch(hipStream_t s, OocBatch B, int W, const spray_rt_ray* rays,
                               const uint32_t* idx, const uint64_t* masks, const float* boxes,
                               uint64_t* key, uint64_t* pkey, uint32_t* pleaf,
                               spray_rt_hit* hits) {
  if (B.count <= 0 || B.count > kOocBatch) return hipErrorInvalidValue;
  const unsigned g = batch_grid(B);
  if (g == 0) return hipSuccess;
  if (W == 1)
    k_ooc_ch_batch<1><<<g, kBlock, 0, s>>>(B, rays, idx, masks, boxes, key, pkey, pleaf);
  else
    k_ooc_ch_batch<4><<<g, kBlock, 0, s>>>(B, rays, idx, masks, boxes, key, pkey, pleaf);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  k_ooc_ch_resolve<<<g, kBlock, 0, s>>>(B, rays, idx, key, pkey, pleaf, hits);
  return hipGetLastError();
}

hipError_t launch_ooc_ah_batch(hipStream_t s, OocBatch B, const spray_rt_ray* rays,
                               const uint32_t* idx, uint8_t* occ) {
  if (B.count <= 0 || B.count > kOocBatch) return hipErrorInvalidValue;
  const unsigned g = batch_grid(B);
  if (g == 0) return hipSuccess;
  k_ooc_ah_batch<<<g, kBlock, 0, s>>>(B, rays, idx, occ);
  return hipGetLastError();
}

hipError_t launch_ooc_clear_occ(hipStream_t s, const uint8_t* valid, uint8_t* occ, size_t M) {
  if (M == 0) return hipSuccess;
  k_ooc_clear_occ<<<grid_for(M), kBlock, 0, s>>>(valid, occ, M);
  return hipGetLastError();
}

}  // namespace spray_rt
