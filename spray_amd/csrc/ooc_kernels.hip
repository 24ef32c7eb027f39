// ooc_kernels.hip -- gfx950 kernels of the out-of-core (streamed-domain) path.
//
// The reference's ooc tracer queues every ray to every domain on its sorted
// domain list (ooc_isector.h:116-174) and drains one resident domain at a
// time (ooc_tcontext.inl:28-101) while the LRU cache streams the next ones
// in (lru_cache.cc:65-171).  On the GPU the queues are built in bulk --
// domain masks, (domain, ray) pairs, one stable radix sort -- and each
// resident domain drains its queue in one launch.  A ray's closest hit is
// combined across launches by the order of the sequential walk of its
// domain list, (t, then (entry t of the domain box, domain id)), so the
// result is the whole-scene one whatever the drain order.
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include "rt_device.h"
#include "rt_kernels.h"

namespace spray_rt {
namespace {

// orderable bits of a float (total order, -0 < +0)
__device__ __forceinline__ uint32_t ord_bits(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

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
                                                     uint64_t* __restrict__ tie, size_t M) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  float4* hp = reinterpret_cast<float4*>(hits + i);
  hp[0] = make_float4(kInf, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu));
  hp[1] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
  hp[2] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  tie[i] = ~0ull;
}

// Closest hit of the rays queued to one resident domain, merged into the
// running result of each ray: nearer t wins; an equal t goes to the earlier
// entry of the ray's domain list (smaller (box entry t, id)).
// The queue of one domain holds its rays in ascending ray order --
// neighbouring pixels -- so each wave walks the tree as a packet
// (trace_tree_packet: one scalar fetch per node per wave).
__global__ __launch_bounds__(kBlock) void k_ooc_ch(OocDomain D,
                                                   const spray_rt_ray* __restrict__ rays,
                                                   const uint32_t* __restrict__ idx,
                                                   uint32_t n, spray_rt_hit* __restrict__ hits,
                                                   uint64_t* __restrict__ tie) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (blockIdx.x * kBlock + (threadIdx.x & ~63u) >= n) return;  // whole wave idle
  const bool valid = j < n;
  const uint32_t i = valid ? idx[j] : 0u;
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  float4 h0 = make_float4(0.f, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu));
  if (valid) {
    const float4* rp = reinterpret_cast<const float4*>(rays + i);
    o4 = rp[0];
    d4 = rp[1];
    h0 = reinterpret_cast<const float4*>(hits + i)[0];
  }
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  float4* hp = reinterpret_cast<float4*>(hits + i);
  const bool have = __float_as_uint(h0.w) != 0xFFFFFFFFu;
  const float tcur = have ? h0.x : d4.w;
  // the domain's own nearest hit with t <= tcur (ties at tcur included)
  Best best{tcur, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool act = valid, hit = false;
  trace_tree_packet<false>(reinterpret_cast<uint64_t>(D.nodes),
                           reinterpret_cast<uint64_t>(D.tris),
                           reinterpret_cast<uint64_t>(D.prims), r, o4.w, 0.f, best, act, hit,
                           wstack + (threadIdx.x >> 6) * kStack);
  if (!valid || best.leaf == 0xFFFFFFFFu) return;
  const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  float tm;
  aabb_ref(D.box, dr, tm);
  const uint64_t mine = (uint64_t(ord_bits(tm)) << 32) | uint32_t(D.domain);
  if (have && !(best.t < tcur) && !(mine < tie[i])) return;
  SlotDesc s{};
  s.tris = static_cast<const float*>(D.tris);
  s.faces = D.faces;
  s.colors = D.colors;
  s.normals = D.normals;
  float hu, hv;
  const float4 c = hit_uv(s, r, o4.w, best.leaf, hu, hv);
  uint32_t color;
  float nsx, nsy, nsz;
  epilogue(s, best.prim, hu, hv, color, nsx, nsy, nsz);
  hp[0] = make_float4(best.t, hu, hv, __uint_as_float(best.prim));
  hp[1] = make_float4(c.y, c.z, c.w, __uint_as_float(color));
  hp[2] = make_float4(nsx, nsy, nsz, __int_as_float(D.domain));
  tie[i] = mine;
}

// Any hit of the rays queued to one resident domain, OR-ed into occ.
__global__ __launch_bounds__(kBlock) void k_ooc_ah(OocDomain D,
                                                   const spray_rt_ray* __restrict__ rays,
                                                   const uint32_t* __restrict__ idx,
                                                   uint32_t n, uint8_t* __restrict__ occ) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (blockIdx.x * kBlock + (threadIdx.x & ~63u) >= n) return;  // whole wave idle
  const uint32_t i = j < n ? idx[j] : 0u;
  const bool valid = j < n && !occ[i];  // else occluded by an earlier domain
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
  size_t a = 0, b = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, a, static_cast<uint32_t*>(nullptr),
                                   static_cast<uint32_t*>(nullptr), int(M + 1));
  hipcub::DeviceRadixSort::SortPairs(nullptr, b, static_cast<uint16_t*>(nullptr),
                                     static_cast<uint16_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr), int(pairs), 0, 8);
  return a > b ? a : b;
}

hipError_t launch_ooc_init(hipStream_t s, spray_rt_hit* hits, uint64_t* tie, size_t M) {
  if (M == 0) return hipSuccess;
  k_ooc_init<<<grid_for(M), kBlock, 0, s>>>(hits, tie, M);
  return hipGetLastError();
}

hipError_t launch_ooc_ch(hipStream_t s, const OocDomain& D, const spray_rt_ray* rays,
                         const uint32_t* idx, uint32_t n, spray_rt_hit* hits, uint64_t* tie) {
  if (n == 0) return hipSuccess;
  k_ooc_ch<<<grid_for(n), kBlock, 0, s>>>(D, rays, idx, n, hits, tie);
  return hipGetLastError();
}

hipError_t launch_ooc_ah(hipStream_t s, const OocDomain& D, const spray_rt_ray* rays,
                         const uint32_t* idx, uint32_t n, uint8_t* occ) {
  if (n == 0) return hipSuccess;
  k_ooc_ah<<<grid_for(n), kBlock, 0, s>>>(D, rays, idx, n, occ);
  return hipGetLastError();
}

hipError_t launch_ooc_clear_occ(hipStream_t s, const uint8_t* valid, uint8_t* occ, size_t M) {
  if (M == 0) return hipSuccess;
  k_ooc_clear_occ<<<grid_for(M), kBlock, 0, s>>>(valid, occ, M);
  return hipGetLastError();
}

}  // namespace spray_rt
