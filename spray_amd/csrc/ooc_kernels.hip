// ooc_kernels.hip -- gfx950 kernels of the out-of-core (streamed-domain) path.
//
// The reference's ooc tracer queues every ray to every domain on its sorted
// domain list (ooc_isector.h:116-174) and drains one resident domain at a
// time (ooc_tcontext.inl:28-101) while the LRU cache streams the next ones
// in (lru_cache.cc:65-171).  On the GPU the queues are built in bulk -- one
// pass over the rays computes the domain lists, the queue lengths and the
// DomainStats scores, a one-block scan places the queues, a second pass
// scatters the ray ids -- and each batch of resident domains drains its
// queues in one launch.  A ray's closest hit is combined across domains by
// the order of the sequential walk of its domain list, (t, then the list
// position), so the result is the whole-scene one whatever the drain order.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "rt_device.h"
#include "rt_kernels.h"

namespace spray_rt {
namespace {

constexpr int kWaves = kBlock / 64;
// blocks of the queue pass (k_ooc_masks): ~6 per CU resident at its LDS
#ifndef SPRAY_OOC_MASK_BLOCKS
#define SPRAY_OOC_MASK_BLOCKS 3072
#endif
constexpr unsigned kOocMaskBlocks = SPRAY_OOC_MASK_BLOCKS;
// waves per SIMD the any-hit drain is compiled for (register budget)
#ifndef SPRAY_OOC_AH_WAVES
#define SPRAY_OOC_AH_WAVES 1
#endif

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
  uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
  for (int off = 32; off > 0; off >>= 1) {
    lo |= __shfl_xor(lo, off);
    hi |= __shfl_xor(hi, off);
  }
  return (uint64_t(hi) << 32) | lo;
}

// A wave-uniform pointer as the packet walk's SGPR address: the segment's
// domain is the wave's, but the compiler cannot prove a pointer read through
// a dynamically indexed kernel argument uniform, and would fetch every node
// and triangle through the vector path into each lane.
__device__ __forceinline__ uint64_t uniform_ptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))));
  return (uint64_t(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t lanes_below() {
  const uint32_t l = threadIdx.x & 63;
  return l ? (~0ull >> (64 - l)) : 0ull;
}

// Position of domain `dom` (entry t `tb`) in the ray's sorted domain list
// (ascending (intersectAabb entry t, id), rays.h:71-79): the tie-break of
// the key and the DomainStats weight.
template <int W>
__device__ __forceinline__ uint32_t list_pos(const uint64_t* m, const float* boxes, int dom,
                                             float tb, const DRay& dr) {
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

// Ascending (t, id) over the first N of a lane's register entries: a
// bitonic sorting network, every index a compile-time constant.
template <int N, int R>
__device__ __forceinline__ void sort_entries(float (&t)[R], int (&id)[R]) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l <= i) continue;
        const bool up = (i & k) == 0;
        const bool gt = t[i] > t[l] || (t[i] == t[l] && id[i] > id[l]);
        if (gt == up) {
          const float tt = t[i];
          t[i] = t[l];
          t[l] = tt;
          const int ti = id[i];
          id[i] = id[l];
          id[l] = ti;
        }
      }
}

// Confirmed domains a lane keeps in LDS for its list positions (longer
// lists recompute positions from the mask).
constexpr int kLaneList = 8;

// Pass 1 over the rays.  The ray's domain list (ooc_isector.h:116-174: the
// domains whose box intersectAabb hits): the conservative top-level walk,
// each candidate then confirmed by the reference's box test (boxes staged
// in LDS).  Per block and domain: queued pairs (bc) and DomainStats::
// increment weights (sb; ooc_domain_stats.cc:60-111: SPRAY_RAY_DOMAIN_
// LIST_SIZE - list position, 1 past the list), summed in LDS, then stored
// block-major ([block * ndom + d], one coalesced row per block).  Also
// resets the per-ray results of the pass.
#ifndef SPRAY_OOC_MASK_WAVES
#define SPRAY_OOC_MASK_WAVES 6
#endif
template <int W>
__global__ __launch_bounds__(kBlock, W == 1 ? SPRAY_OOC_MASK_WAVES : 1) void k_ooc_masks(
    const BvhNode* __restrict__ tlas, int ntlas, const float* __restrict__ boxes, int ndom,
    const spray_rt_ray* __restrict__ rays, const uint8_t* __restrict__ valid, size_t M,
    uint32_t nrb, uint64_t* __restrict__ masks, uint64_t* __restrict__ key_init,
    uint8_t* __restrict__ occ_clear, uint32_t* __restrict__ bc, uint32_t* __restrict__ sb) {
  __shared__ int32_t wstack[kWaves * kStack];
  __shared__ float4 stl[4 * 64 * W];
  __shared__ float sbox[6 * 64 * W];
  __shared__ uint32_t cnt[64 * W], sc[64 * W];
  // up to 64 domains (W == 1): a lane's 16 nearest confirmed entries in
  // registers, sorted (a slot's index is its list position; LDS stays small
  // for the latency-bound walk's occupancy); wider scenes keep kLaneList
  // entries in LDS and look weights up by scanning them (the LDS entry
  // lists measured the same at W == 1)
  constexpr bool kTab = W == 1;
  __shared__ float lte[kTab ? 1 : kLaneList][kBlock];
  __shared__ int lid[kTab ? 1 : kLaneList][kBlock];
  // the top-level tree and the boxes are staged once per block, which then
  // walks ray blocks rb = blockIdx.x, + gridDim.x, ... (one launch-wide
  // staging of 5.5 KB per ray block of 256 rays was 180 MB of L2 reads per
  // 8 M rays)
  for (int q = threadIdx.x; q < 4 * ntlas; q += kBlock) stl[q] = ld4(tlas, q);
  for (int q = threadIdx.x; q < 6 * ndom; q += kBlock) sbox[q] = boxes[q];
  for (uint32_t rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    for (int q = threadIdx.x; q < 64 * W; q += kBlock) cnt[q] = sc[q] = 0;
    __syncthreads();
    const size_t i = size_t(rb) * kBlock + threadIdx.x;
    const bool in = i < M;
    const bool live = in && (!valid || valid[i]);
    uint64_t m[W];
#pragma unroll
    for (int w = 0; w < W; ++w) m[w] = 0;
    float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
    if (live) {
      const float4* rp = reinterpret_cast<const float4*>(rays + i);
      o4 = rp[0];
      d4 = rp[1];
      const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
      tlas_mask_wave<W>(stl, ntlas, wstack + (threadIdx.x >> 6) * kStack, r, o4, d4, m);
    }
    // confirm; the confirmed entry t's go to the lane's list (registers
    // for kTab: kReg slots filled by unrolled selects, no dynamic index)
    constexpr int kReg = 16;
    static_assert(kReg >= int(kDomainListSize), "positions past the list size weigh 1");
    float rte[kTab ? kReg : 1];
    int rid[kTab ? kReg : 1];
    uint32_t k = 0;
    const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
    if (live) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t bits = m[w];
        while (bits) {
          const int j = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          float te;
          if (aabb_ref(sbox + 6 * (64 * w + j), dr, te)) {
            if constexpr (kTab) {
              // the kReg nearest entries (te, id) stay; any other one is past
              // list position kReg - 1 >= kDomainListSize - 1: weight 1
              const int d = 64 * w + j;
              if (k < uint32_t(kReg)) {
#pragma unroll
                for (int q = 0; q < kReg; ++q)
                  if (uint32_t(q) == k) {
                    rte[q] = te;
                    rid[q] = d;
                  }
              } else {
                int qm = 0;
                float tm = rte[0];
                int im = rid[0];
#pragma unroll
                for (int q = 1; q < kReg; ++q)
                  if (rte[q] > tm || (rte[q] == tm && rid[q] > im)) {
                    qm = q;
                    tm = rte[q];
                    im = rid[q];
                  }
                if (te < tm || (te == tm && d < im)) {
#pragma unroll
                  for (int q = 0; q < kReg; ++q)
                    if (q == qm) {
                      rte[q] = te;
                      rid[q] = d;
                    }
                }
              }
            } else if (k < kLaneList) {
              lte[k][threadIdx.x] = te;
              lid[k][threadIdx.x] = 64 * w + j;
            }
            ++k;
          } else {
            m[w] &= ~(1ull << j);
          }
        }
      }
    }
    // list position of each confirmed domain = its rank by (entry t, id);
    // its DomainStats weight kDomainListSize - position (1 past the list)
    if constexpr (kTab) {
      // the wave's longest list bounds the unrolled loops (a scalar exit:
      // sky waves and dead slots skip them)
      uint32_t kmax = k;
      for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, uint32_t(__shfl_xor(int(kmax), o)));
      kmax = uint32_t(__builtin_amdgcn_readfirstlane(int(kmax)));
      if (kmax) {
        // sort the kept entries by (entry t, id) with a bitonic network in
        // registers (empty slots last); a slot's index is its list position
        const uint32_t nk = min(k, uint32_t(kReg));
#pragma unroll
        for (int q = 0; q < kReg; ++q)
          if (uint32_t(q) >= nk) {
            rte[q] = kInf;
            rid[q] = INT_MAX;
          }
        if (kmax <= 8)
          sort_entries<8>(rte, rid);
        else
          sort_entries<kReg>(rte, rid);
        // per list position a (the same weight in every lane): the lanes
        // holding the same domain there are counted together -- coherent
        // waves hold one or two domains per position
#pragma unroll
        for (int a = 0; a < kReg; ++a) {
          if (uint32_t(a) >= kmax) break;
          const int d = uint32_t(a) < nk ? rid[a] : -1;
          const uint32_t wt = uint32_t(a) < kDomainListSize ? kDomainListSize - uint32_t(a) : 1u;
          uint64_t todo = __ballot(d >= 0);
          while (todo) {
            const int dd = __builtin_amdgcn_readlane(d, __ffsll((long long)todo) - 1);
            const uint64_t same = __ballot(d == dd);
            todo &= ~same;
            if ((threadIdx.x & 63) == 0) {
              const uint32_t n = uint32_t(__popcll(same));
              atomicAdd(&cnt[dd], n);
              atomicAdd(&sc[dd], n * wt);
            }
          }
        }
        if (kmax > uint32_t(kReg)) {
          // lists longer than kReg: the entries past the kept ones weigh 1
          uint64_t extra = 0;
          if (k > uint32_t(kReg)) {
            extra = m[0];
#pragma unroll
            for (int q = 0; q < kReg; ++q) extra &= ~(1ull << (rid[q] & 63));
          }
          uint64_t u = wave_or64(extra);
          while (u) {
            const int j = __ffsll((long long)u) - 1;
            u &= u - 1;
            const uint32_t n = uint32_t(__popcll(__ballot((extra >> j) & 1ull)));
            if ((threadIdx.x & 63) == 0) {
              atomicAdd(&cnt[j], n);
              atomicAdd(&sc[j], n);
            }
          }
        }
      }
    } else {
      if (k <= kLaneList)
        for (uint32_t a = 0; a < k; ++a) {
          const float ta = lte[a][threadIdx.x];
          const int da = lid[a][threadIdx.x] & 0xFFFF;
          uint32_t pos = 0;
          for (uint32_t b = 0; b < k; ++b) {
            const float tb = lte[b][threadIdx.x];
            pos += (tb < ta || (tb == ta && (lid[b][threadIdx.x] & 0xFFFF) < da)) ? 1u : 0u;
          }
          lid[a][threadIdx.x] = da | int((pos < kDomainListSize ? kDomainListSize - pos : 1u) << 16);
        }
      // per domain of the wave: pairs and weights summed over the wave first
      // (a wave's rays mostly share domains: same-address LDS atomics serialise)
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t u = wave_or64(m[w]);
        while (u) {
          const int j = __ffsll((long long)u) - 1;
          u &= u - 1;
          const int dom = 64 * w + j;
          const bool has = (m[w] >> j) & 1;
          uint32_t add = 0;
          if (has) {
            if (k <= kLaneList) {
              for (uint32_t a = 0; a < k; ++a) {
                const int e = lid[a][threadIdx.x];
                if ((e & 0xFFFF) == dom) add = uint32_t(e) >> 16;
              }
            } else {  // long list: the position from the mask
              float te;
              aabb_ref(sbox + 6 * dom, dr, te);
              const uint32_t pos = list_pos<W>(m, sbox, dom, te, dr);
              add = pos < kDomainListSize ? kDomainListSize - pos : 1u;
            }
          }
          const uint32_t n = uint32_t(__popcll(__ballot(has)));
          for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o);
          if ((threadIdx.x & 63) == 0) {
            atomicAdd(&cnt[dom], n);
            atomicAdd(&sc[dom], add);
          }
        }
      }
    }
    if (in) {
#pragma unroll
      for (int w = 0; w < W; ++w) masks[i * W + w] = m[w];
      if (key_init) key_init[i] = kOocMissKey;
      if (occ_clear && live) occ_clear[i] = 0;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < ndom; q += kBlock) {
      bc[size_t(rb) * ndom + q] = cnt[q];
      sb[size_t(rb) * ndom + q] = sc[q];
    }
    __syncthreads();  // cnt / sc are cleared for the next ray block
  }
}

// The per-block counts of one domain form a column of bc; columns are cut
// into chunks of kOocChunk ray blocks, one 1024-thread block per (domain,
// chunk).  Pass a: chunk sums of counts and DomainStats weights; pass b:
// each chunk's exclusive scan from the sum of the chunks before it (off,
// domain-major: a ray block's place in its queue); then one block folds
// the chunk sums into queue lengths, scores and queue starts.
constexpr int kScanBlock = 1024;


__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < kScanBlock / 64; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(kScanBlock) void k_ooc_chunk_sums(
    const uint32_t* __restrict__ bc, const uint32_t* __restrict__ sb, uint32_t nb, int ndom,
    uint32_t* __restrict__ csum, uint32_t* __restrict__ cw) {
  __shared__ uint32_t red[2][kScanBlock / 64];
  const int d = blockIdx.x, c = blockIdx.y;
  uint32_t v = 0, w = 0;
  const uint32_t end = nb < (c + 1) * kOocChunk ? nb : (c + 1) * kOocChunk;
  for (uint32_t b = c * kOocChunk + threadIdx.x; b < end; b += kScanBlock) {
    v += bc[size_t(b) * ndom + d];
    w += sb[size_t(b) * ndom + d];
  }
  const uint32_t tv = block_sum_u32(v, red[0]);
  const uint32_t tw = block_sum_u32(w, red[1]);
  if (threadIdx.x == 0) {
    csum[size_t(d) * gridDim.y + c] = tv;
    cw[size_t(d) * gridDim.y + c] = tw;
  }
}

__global__ __launch_bounds__(kScanBlock) void k_ooc_chunk_scan(
    const uint32_t* __restrict__ bc, const uint32_t* __restrict__ csum, uint32_t nb, int ndom,
    uint32_t* __restrict__ off) {
  constexpr int kW = kScanBlock / 64;
  __shared__ uint32_t wsum[kW];
  __shared__ uint32_t carry;
  const int d = blockIdx.x, c = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int q = 0; q < c; ++q) t += csum[size_t(d) * gridDim.y + q];
    carry = t;
  }
  __syncthreads();
  const uint32_t end = nb < (c + 1) * kOocChunk ? nb : (c + 1) * kOocChunk;
  for (uint32_t b0 = c * kOocChunk; b0 < end; b0 += kScanBlock) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < end ? bc[size_t(b) * ndom + d] : 0u;
    uint32_t incl = v;  // inclusive scan within the wave
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o);
      if (lane >= o) incl += x;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = carry;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    if (b < end) off[size_t(d) * nb + b] = before + incl - v;
    __syncthreads();
    if (threadIdx.x == kScanBlock - 1) carry = before + incl;
    __syncthreads();
  }
}

// Queue bounds (one block): lengths and scores from the chunk sums, first =
// their exclusive scan; every pair starts live.
__global__ __launch_bounds__(256) void k_ooc_first(const uint32_t* __restrict__ csum,
                                                   const uint32_t* __restrict__ cw, int nch,
                                                   int ndom, uint32_t* __restrict__ first,
                                                   uint32_t* __restrict__ live,
                                                   unsigned long long* __restrict__ score) {
  __shared__ uint32_t sh[256];
  const int t = threadIdx.x;
  uint32_t v = 0;
  if (t < ndom) {
    unsigned long long w = 0;
    for (int q = 0; q < nch; ++q) {
      v += csum[size_t(t) * nch + q];
      w += cw[size_t(t) * nch + q];
    }
    score[t] = w;
  }
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t x = t >= o ? sh[t - o] : 0u;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  if (t < ndom) {
    first[t] = sh[t] - v;
    live[t] = v;
  }
  if (t == ndom - 1) first[ndom] = sh[t];
}

// Pass 2: ray i's id into the queue of every domain on its list, at its
// block's scanned offset plus its rank among the block's rays of that
// domain: every queue holds its rays in ascending order (packets of
// neighbouring rays), the same order every run.  Positions past cap are
// dropped (the host sees the total and grows).
template <int W>
__global__ __launch_bounds__(kBlock) void k_ooc_scatter(
    const uint64_t* __restrict__ masks, size_t M, const uint32_t* __restrict__ first,
    const uint32_t* __restrict__ off, uint32_t* __restrict__ val, size_t cap) {
  __shared__ uint32_t wc[kWaves][64 * W];
  for (int k = threadIdx.x; k < kWaves * 64 * W; k += kBlock) (&wc[0][0])[k] = 0;
  __syncthreads();
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const int wave = threadIdx.x >> 6;
  uint64_t m[W], u[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    m[w] = i < M ? masks[i * W + w] : 0ull;
    u[w] = wave_or64(m[w]);
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = u[w];
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      const uint64_t b = __ballot((m[w] >> j) & 1);
      if ((threadIdx.x & 63) == 0) wc[wave][64 * w + j] = uint32_t(__popcll(b));
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * W; k += kBlock) {  // exclusive over the waves
    uint32_t run = 0;
    for (int v = 0; v < kWaves; ++v) {
      const uint32_t c = wc[v][k];
      wc[v][k] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = u[w];
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      const bool has = (m[w] >> j) & 1;
      const uint64_t b = __ballot(has);
      if (has) {
        const int dom = 64 * w + j;
        const size_t pos = size_t(first[dom]) + off[size_t(dom) * gridDim.x + blockIdx.x] +
                           wc[wave][dom] + uint32_t(__popcll(b & lanes_below()));
        if (pos < cap) val[pos] = uint32_t(i);
      }
    }
  }
}

// The pair handled by this lane of a batch launch: the waves of segment s
// (one resident domain's queue) are wave0[s] .. wave0[s+1]-1, so a wave
// always walks one domain tree.  Returns the segment, or -1 past the end.
__device__ __forceinline__ int batch_pair(const OocBatch& B, uint32_t& pj, bool& valid,
                                          uint32_t blk) {
  const uint32_t gw = (blk * kBlock + threadIdx.x) >> 6;
  if (gw >= B.wave0[B.count]) return -1;
  int s = 0;
  while (s + 1 < B.count && B.wave0[s + 1] <= gw) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  const uint32_t j = (gw - B.wave0[s]) * 64 + (threadIdx.x & 63);
  valid = j < B.n[s];
  pj = B.begin[s] + (valid ? j : 0u);
  return s;
}

// Copy blocks of a launch (blockIdx >= B.copy0): the next batch's images,
// pinned host memory -> HBM slot, 16-B lanes, four loads in flight per lane.
__device__ __forceinline__ void prefetch_copy(const OocBatch& B, uint32_t blk) {
  const uint32_t nthreads = B.ncopy * kBlock;
  const uint32_t t = (blk - B.copy0) * kBlock + threadIdx.x;
  for (int e = 0; e < B.pf_count; ++e) {
    const uint4* __restrict__ src = B.pf_src[e];
    uint4* __restrict__ dst = B.pf_dst[e];
    const uint32_t n = B.pf_n16[e];
    uint32_t q = t;
    for (; q + 3 * nthreads < n; q += 4 * nthreads) {
      const uint4 a = src[q], b = src[q + nthreads], c = src[q + 2 * nthreads],
                  d = src[q + 3 * nthreads];
      dst[q] = a;
      dst[q + nthreads] = b;
      dst[q + 2 * nthreads] = c;
      dst[q + 3 * nthreads] = d;
    }
    for (; q < n; q += nthreads) dst[q] = src[q];
  }
}

// Liveness bookkeeping of the drains: live[d] counts the pairs of domain d's
// queue that can still change a result -- closest hit: the domain's entry t
// is not beyond the ray's best t (filterRqs, ooc_tcontext.inl:147: tdom <=
// the ray's t); any hit: the ray is not occluded yet (filterSqs, :165).  It
// starts at the queue length; a ray whose best t drops from `to` to `tn`
// kills exactly its pairs with entry t in (tn, to], and a ray's first
// occlusion kills all of its pairs, so each pair is counted down once.  A
// lane collects its killed domains as a mask; the wave sums the masks per
// domain (one ballot each) and adds once per domain in LDS -- the lanes of a
// wave mostly kill the same domains, and same-address LDS atomics
// serialise -- and the block adds once per domain globally.
template <int W>
__device__ __forceinline__ void death_mask(const uint64_t* m, const float* boxes,
                                           const DRay& dr, float tn, float to, uint64_t* dm) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = m[w];
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      float te;
      if (aabb_ref(boxes + 6 * (64 * w + j), dr, te) && te > tn && !(te > to))
        dm[w] |= 1ull << j;
    }
  }
}

// every lane of the wave calls this (converged)
template <int W>
__device__ __forceinline__ void wave_add_deaths(const uint64_t* dm, uint32_t* dead) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t u = wave_or64(dm[w]);
    while (u) {
      const int j = __ffsll((long long)u) - 1;
      u &= u - 1;
      const uint32_t n = uint32_t(__popcll(__ballot((dm[w] >> j) & 1ull)));
      if ((threadIdx.x & 63) == 0) atomicAdd(dead + 64 * w + j, n);
    }
  }
}

// A block's deaths go to one of kOocDeadShards counters per domain (by block
// index): a launch's blocks end at nearly the same time, and same-address
// atomics serialise in L2 -- one counter per domain, and one "last block"
// counter per launch, queued thousands of atomics behind each other.
template <int W>
__device__ __forceinline__ void flush_deaths(const uint32_t* dead, uint32_t* dshard) {
  __syncthreads();
  const uint32_t sh = blockIdx.x % kOocDeadShards;
  for (int k = threadIdx.x; k < 64 * W; k += kBlock)
    if (dead[k]) atomicAdd(dshard + size_t(k) * kOocDeadShards + sh, dead[k]);
}

// The live counts to the host (OocSnapshot): the launch's deaths summed out
// of their shards (which are cleared) and taken off live, the values, then
// the sequence number with system-scope release.  One block, after every
// drain block of the launch (a kernel boundary).
__device__ __forceinline__ void write_snapshot(uint32_t* live, uint32_t* dshard,
                                               const OocSnapshot& S, int ndom) {
  const unsigned long long g = (unsigned long long)S.gen << 32;
  for (int k = threadIdx.x; k < ndom; k += blockDim.x) {
    uint32_t* d = dshard + size_t(k) * kOocDeadShards;
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < kOocDeadShards; ++j) {
      sum += d[j];
      d[j] = 0;
    }
    const uint32_t v = live[k] - sum;
    live[k] = v;
    S.snap[k] = g | v;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(S.seq, g | (S.launch + 1u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Closest hit of the rays queued to up to kOocBatch resident domains in one
// launch.  Each live (ray, domain) pair walks its domain tree as a packet (a
// queue holds neighbouring rays) with the ray's current best t as the cut,
// and a hit enters the ray's 64-bit key (t bits | list position | domain) by
// atomicMin.  The key order is the sequential walk's winner rule (nearer t,
// then the earlier list entry) and keys are unique per (ray, domain), so the
// result is the same in any drain order and any interleaving.
//
// The hit record (updateIntersection, trimesh_buffer.cc:328-360) is made in
// the drain, while the domain is resident, by every pair whose atomicMin
// lowered the ray's key -- into the ray's record slot of the pair's batch
// position s (one pair per ray per position per launch).  The final winner
// lowered the key when it entered it (keys are unique, so the old value was
// larger), and a slot is written only by a pair that lowers the key:
// nothing after the winner overwrites its slot.  A domain is drained once
// per pass, at one batch position (dpos[domain], written by the launch), so
// k_ooc_finish reads the winner's slot from the final key's domain.  No
// pair reads another's record inside a launch, so no
// agent-scope acquire / release is needed (the round-5 in-drain resolve
// counted each ray's last pair and needed one: L2 write-back + invalidate
// per pair, 2.4x slower); every read is after a kernel boundary.
template <int W>
__device__ __forceinline__ void ch_pair(const OocDomain& D, int slot, uint32_t pj, bool valid,
                                        const spray_rt_ray* rays, const uint32_t* idx,
                                        const uint64_t* masks, const float* boxes,
                                        uint64_t* key, uint4* rec, int per, int32_t* stack,
                                        uint32_t* dead) {
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
  const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  // the domain's own nearest hit with t <= the ray's best so far (ties at
  // that t included: the list position decides them); a pair whose domain
  // starts beyond that t is dead and does not walk
  const float tcur = k0 == kOocMissKey ? d4.w : __uint_as_float(uint32_t(k0 >> 32));
  float te = 0.f;
  aabb_ref(boxes + 6 * D.domain, dr, te);
  Best best{tcur, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool act = valid && !(te > tcur), hit = false;
  if (__ballot(act))
    trace_tree_packet<false>(uniform_ptr(D.nodes), uniform_ptr(D.tris), uniform_ptr(D.prims), r,
                             o4.w, 0.f, best, act, hit, stack);
  uint64_t dm[W];
#pragma unroll
  for (int w = 0; w < W; ++w) dm[w] = 0;
  bool lowered = false;
  uint64_t mine = kOocMissKey;
  if (valid && best.leaf != 0xFFFFFFFFu) {
    uint64_t m[W];
#pragma unroll
    for (int w = 0; w < W; ++w) m[w] = masks[size_t(i) * W + w];
    mine = (uint64_t(__float_as_uint(best.t)) << 32) |
           (uint64_t(list_pos<W>(m, boxes, D.domain, te, dr)) << 16) | uint64_t(D.domain);
    const uint64_t old =
        atomicMin(reinterpret_cast<unsigned long long*>(key + i), (unsigned long long)mine);
    if (mine < old) {
      lowered = true;
      const float to = old == kOocMissKey ? kInf : __uint_as_float(uint32_t(old >> 32));
      if (best.t < to) death_mask<W>(m, boxes, dr, best.t, to, dm);
    }
  }
  if (lowered) {
    SlotDesc sd{};
    sd.tris = static_cast<const float*>(D.tris);
    sd.faces = D.faces;
    sd.colors = D.colors;
    sd.normals = D.normals;
    const uint32_t prim = reinterpret_cast<const GAS uint32_t*>(gptr(D.prims))[best.leaf];
    float hu, hv;
    const float4 c = hit_uv(sd, r, o4.w, best.leaf, hu, hv);
    uint32_t color;
    float nsx, nsy, nsz;
    epilogue(sd, prim, hu, hv, color, nsx, nsy, nsz);
    // the hit record (spray_rt_hit: t u v prim | Ng color | Ns domain)
    uint4* rp = rec + (size_t(i) * size_t(per) + size_t(slot)) * 3;
    rp[0] = make_uint4(__float_as_uint(best.t), __float_as_uint(hu), __float_as_uint(hv), prim);
    rp[1] = make_uint4(__float_as_uint(c.y), __float_as_uint(c.z), __float_as_uint(c.w), color);
    rp[2] = make_uint4(__float_as_uint(nsx), __float_as_uint(nsy), __float_as_uint(nsz),
                       uint32_t(D.domain));
  }
  wave_add_deaths<W>(dm, dead);
}

// The launch's deaths go to shard set S.launch & 1; its block 0 publishes
// the launch before it (set (S.launch - 1) & 1, complete at this kernel's
// start: block 0 is dispatched first), as the any-hit drains do -- the
// closest-hit pass needs no resolve launch of its own.  The drain and copy
// blocks follow at blockIdx.x - 1.
template <int W>
__global__ __launch_bounds__(kBlock) void k_ooc_ch_batch(
    OocBatch B, const spray_rt_ray* __restrict__ rays, const uint32_t* __restrict__ idx,
    const uint64_t* __restrict__ masks, const float* __restrict__ boxes,
    uint64_t* __restrict__ key, uint4* __restrict__ rec, int per, uint8_t* __restrict__ dpos,
    uint32_t* __restrict__ dshard, uint32_t* __restrict__ live, OocSnapshot S, int ndom) {
  const size_t set = size_t(ndom) * kOocDeadShards;
  if (blockIdx.x == 0) {  // the batch's positions, the previous launch's counts
    if (threadIdx.x < unsigned(B.count)) dpos[B.d[threadIdx.x].domain] = uint8_t(threadIdx.x);
    if (S.launch > 0) {
      OocSnapshot P = S;
      P.launch = S.launch - 1;
      write_snapshot(live, dshard + ((S.launch - 1) & 1u) * set, P, ndom);
    }
    return;
  }
  const uint32_t blk = blockIdx.x - 1;
  if (blk >= B.copy0) {
    prefetch_copy(B, blk);
    return;
  }
  dshard += (S.launch & 1u) * set;
  __shared__ int32_t wstack[kWaves * kStack];
  __shared__ uint32_t dead[64 * W];
  for (int k = threadIdx.x; k < 64 * W; k += kBlock) dead[k] = 0;
  __syncthreads();
  uint32_t pj;
  bool valid;
  const int s = batch_pair(B, pj, valid, blk);
  if (s >= 0)
    ch_pair<W>(B.d[s], s, pj, valid, rays, idx, masks, boxes, key, rec, per,
               wstack + (threadIdx.x >> 6) * kStack, dead);
  flush_deaths<W>(dead, dshard);
}

// The hit records of a closest-hit pass: a miss record where the key is
// still kOocMissKey, else the winner's record slot -- the batch position its
// domain had (dpos, k_ooc_ch_batch).  One lane per 16-B quarter of a
// record, so a wave stores whole lines.
__global__ __launch_bounds__(kBlock) void k_ooc_finish(const uint64_t* __restrict__ key,
                                                       const uint4* __restrict__ rec, int per,
                                                       const uint8_t* __restrict__ dpos,
                                                       spray_rt_hit* __restrict__ hits,
                                                       size_t M) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const size_t i = j / 3;
  if (i >= M) return;
  const int part = int(j - 3 * i);
  const uint64_t k = key[i];
  float4 v = part == 0   ? make_float4(kInf, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu))
             : part == 1 ? make_float4(0.f, 0.f, 0.f, __uint_as_float(0u))
                         : make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  if (k != kOocMissKey) {
    const uint32_t s = dpos[uint32_t(k) & 0xFFFFu];
    const uint4 q = rec[(size_t(i) * size_t(per) + s) * 3 + size_t(part)];
    v = make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z),
                    __uint_as_float(q.w));
  }
  reinterpret_cast<float4*>(hits)[j] = v;
}

// Any hit of the rays queued to the batch's domains, OR-ed into occ (a ray
// already occluded by an earlier batch is skipped).  PACKET: the wave walks
// the domain tree as a packet (trace_tree_packet<ANY>: one scalar fetch per
// node, a lane leaves at its first occluder) -- a queue holds neighbouring
// rays in ascending order, and point-light shadow rays of neighbouring
// pixels are coherent; else each lane walks its own ray (occluded_tree_ww,
// the in-core per-lane walk, for incoherent rays).  The OR is an atomic on
// the byte's word so that exactly one writer sees the ray's first occlusion
// and counts its pairs dead.
template <int W, int MODE>
__device__ __forceinline__ void ah_pair(const OocDomain& D, uint32_t pj, bool ok,
                                        const spray_rt_ray* rays, const uint32_t* idx,
                                        const uint64_t* masks, uint8_t* occ, int32_t* lstk,
                                        int32_t* wstk, uint32_t* dead) {
  const uint32_t i = ok ? idx[pj] : 0u;
  bool act = ok && !occ[i];
  bool hit = false;
  constexpr bool packet = MODE == 1;
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  if (act) {
    const float4* rp = reinterpret_cast<const float4*>(rays + i);
    o4 = rp[0];
    d4 = rp[1];
  }
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  if constexpr (packet) {
    Best best{0.f, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (__ballot(act))
      trace_tree_packet<true>(uniform_ptr(D.nodes), uniform_ptr(D.tris), uniform_ptr(D.prims), r,
                              o4.w, d4.w, best, act, hit, wstk);
  } else if (act) {
    hit = occluded_tree_ww(D.nodes, D.tris, r, o4.w, d4.w, lstk);
  }
  uint64_t dm[W];
#pragma unroll
  for (int w = 0; w < W; ++w) dm[w] = 0;
  if (hit) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(occ + i);
    const uint32_t sh = 8u * uint32_t(a & 3u);
    const uint32_t was = atomicOr(reinterpret_cast<uint32_t*>(a & ~uintptr_t(3)), 1u << sh);
    if (!((was >> sh) & 0xFFu)) {  // the first writer counts the ray's pairs dead
#pragma unroll
      for (int w = 0; w < W; ++w) dm[w] = masks[size_t(i) * W + w];
    }
  }
  wave_add_deaths<W>(dm, dead);
}

// The launch's deaths go to shard set S.launch & 1; its block 0 publishes
// the launch before it (set (S.launch - 1) & 1, complete at this kernel's
// start; block 0 is dispatched first, so the host, which chooses the batch
// after next from these counts, is not kept waiting for the drain) -- one
// launch per any-hit batch instead of a drain and a one-block snapshot
// kernel.  The drain and copy blocks follow at blockIdx.x - 1.  Launch 0 of
// a pass publishes nothing (the queue build cleared both sets); the pass's
// last launch is never published (no batch follows it).
template <int W, int MODE>
__global__ __launch_bounds__(kBlock, SPRAY_OOC_AH_WAVES) void k_ooc_ah_batch(
    OocBatch B, const spray_rt_ray* __restrict__ rays, const uint32_t* __restrict__ idx,
    const uint64_t* __restrict__ masks, uint8_t* __restrict__ occ,
    uint32_t* __restrict__ dshard, uint32_t* __restrict__ live, OocSnapshot S, int ndom) {
  // per lane: lane-interleaved stacks; packet: one stack per wave
  __shared__ int32_t stack[MODE != 1 ? kStack * kBlock : 1];
  __shared__ int32_t wstack[MODE != 0 ? kWaves * kStack : 1];
  __shared__ uint32_t dead[64 * W];
  const size_t set = size_t(ndom) * kOocDeadShards;
  if (blockIdx.x == 0) {  // the previous launch's counts
    if (S.launch > 0) {
      OocSnapshot P = S;
      P.launch = S.launch - 1;
      write_snapshot(live, dshard + ((S.launch - 1) & 1u) * set, P, ndom);
    }
    return;
  }
  dshard += (S.launch & 1u) * set;
  for (int k = threadIdx.x; k < 64 * W; k += kBlock) dead[k] = 0;
  __syncthreads();
  uint32_t pj;
  bool ok;
  const uint32_t blk = blockIdx.x - 1;
  const int s = blk >= B.copy0 ? -1 : batch_pair(B, pj, ok, blk);
  if (blk >= B.copy0) prefetch_copy(B, blk);
  if (s >= 0)
    ah_pair<W, MODE>(B.d[s], pj, ok, rays, idx, masks, occ, stack + (MODE != 1 ? threadIdx.x : 0),
                     wstack + (MODE != 0 ? (threadIdx.x >> 6) * kStack : 0), dead);
  flush_deaths<W>(dead, dshard);
}

}  // namespace

hipError_t launch_ooc_queues(hipStream_t s, const BvhNode* tlas, int ntlas, int ndom,
                             const float* boxes, const spray_rt_ray* rays, const uint8_t* valid,
                             size_t M, OocScratch& q, uint64_t* key_init, uint8_t* occ_clear,
                             uint32_t* h_first, unsigned long long* h_score) {
  if (ndom <= 0 || ndom > 256 || M == 0 || M > 0xFFFFFFFFull) return hipErrorInvalidValue;
  const int W = ndom <= 64 ? 1 : 4;
  const unsigned g = grid_for(M);
  const size_t n = size_t(ndom) * g;
  if (n > q.block_cap) return hipErrorInvalidValue;  // the caller sizes for M
  // a few ray blocks per block (the tree is staged once per block)
  const unsigned gm = g < kOocMaskBlocks ? g : kOocMaskBlocks;
  if (W == 1)
    k_ooc_masks<1><<<gm, kBlock, 0, s>>>(tlas, ntlas, boxes, ndom, rays, valid, M, g, q.masks,
                                         key_init, occ_clear, q.bc, q.sb);
  else
    k_ooc_masks<4><<<gm, kBlock, 0, s>>>(tlas, ntlas, boxes, ndom, rays, valid, M, g, q.masks,
                                         key_init, occ_clear, q.bc, q.sb);
  const unsigned nch = (g + kOocChunk - 1) / kOocChunk;
  if (size_t(ndom) * nch > q.chunk_cap) return hipErrorInvalidValue;  // the caller sizes for M
  k_ooc_chunk_sums<<<dim3(ndom, nch), kScanBlock, 0, s>>>(q.bc, q.sb, g, ndom, q.csum, q.cw);
  k_ooc_chunk_scan<<<dim3(ndom, nch), kScanBlock, 0, s>>>(q.bc, q.csum, g, ndom, q.off);
  k_ooc_first<<<1, 256, 0, s>>>(q.csum, q.cw, int(nch), ndom, q.first, q.live, q.score);
  // both shard sets at the drains' stride: the drain kernels index them by
  // 64 * W queues (the any-hit launches alternate sets 64 * W * shards apart),
  // not by the scene's ndom -- a set left dirty by a pass's unpublished last
  // launch would be added into the next pass's snapshots
  if (hipMemsetAsync(q.dshard, 0, 2 * size_t(64 * W) * kOocDeadShards * sizeof(uint32_t), s) !=
      hipSuccess)
    return hipGetLastError();
  if (W == 1)
    k_ooc_scatter<1><<<g, kBlock, 0, s>>>(q.masks, M, q.first, q.off, q.val, q.pair_cap);
  else
    k_ooc_scatter<4><<<g, kBlock, 0, s>>>(q.masks, M, q.first, q.off, q.val, q.pair_cap);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(h_first, q.first, (ndom + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h_score, q.score, ndom * sizeof(unsigned long long),
                       hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  q.npair = h_first[ndom];
  return q.npair > q.pair_cap ? hipErrorOutOfMemory : hipSuccess;  // caller grows, redoes
}

static unsigned batch_grid(OocBatch& B) {
  B.ncopy = kOocCopyBlocks;
  B.wave0[0] = 0;
  for (int k = 0; k < B.count; ++k) B.wave0[k + 1] = B.wave0[k] + (B.n[k] + 63) / 64;
  const unsigned g = (B.wave0[B.count] + kWaves - 1) / kWaves;
  B.copy0 = g;
  return g;
}

hipError_t launch_ooc_ch_batch(hipStream_t s, OocBatch B, int W, const spray_rt_ray* rays,
                               const OocScratch& q, const float* boxes, uint64_t* key,
                               spray_rt_hit* hits, OocSnapshot snap) {
  (void)hits;  // the records go to q.rec; k_ooc_finish writes hits
  if (B.count <= 0 || B.count > kOocBatch || B.count > q.rec_per) return hipErrorInvalidValue;
  const int ndom = 64 * W;
  unsigned g = batch_grid(B);
  g += B.pf_count ? B.ncopy : 0;
  g += 1;  // block 0 publishes the previous launch's counts
  if (W == 1)
    k_ooc_ch_batch<1><<<g, kBlock, 0, s>>>(B, rays, q.val, q.masks, boxes, key, q.rec, q.rec_per,
                                           q.dpos, q.dshard, q.live, snap, ndom);
  else
    k_ooc_ch_batch<4><<<g, kBlock, 0, s>>>(B, rays, q.val, q.masks, boxes, key, q.rec, q.rec_per,
                                           q.dpos, q.dshard, q.live, snap, ndom);
  return hipGetLastError();
}

hipError_t launch_ooc_finish(hipStream_t s, const uint64_t* key, const OocScratch& q,
                             spray_rt_hit* hits, size_t M) {
  if (M == 0) return hipSuccess;
  k_ooc_finish<<<grid_for(3 * M), kBlock, 0, s>>>(key, q.rec, q.rec_per, q.dpos, hits, M);
  return hipGetLastError();
}

hipError_t launch_ooc_ah_batch(hipStream_t s, OocBatch B, int W, const spray_rt_ray* rays,
                               const OocScratch& q, uint8_t* occ, OocSnapshot snap,
                               int coherence) {
  if (B.count <= 0 || B.count > kOocBatch) return hipErrorInvalidValue;
  const int ndom = 64 * W;
  unsigned g = batch_grid(B);
  g += B.pf_count ? B.ncopy : 0;
  g += 1;  // block 0 publishes the previous launch's counts
#define SPRAY_AH_LAUNCH(WW, MM)                                                              \
  k_ooc_ah_batch<WW, MM><<<g, kBlock, 0, s>>>(B, rays, q.val, q.masks, occ, q.dshard, q.live, \
                                              snap, ndom)
  // the context's coherence setting: incoherent -> per lane, else packets
  // (measured on configs[3]'s PT shadows, one box: packets 4.08, per lane
  // 4.60, a per-wave choice 4.72 ms per frame -- the choice's direction
  // loads and the two walks' registers and stacks cost more than it saves
  // on queues of neighbouring rays)
  const bool per_lane = coherence == SPRAY_RT_RAYS_INCOHERENT;
  if (W == 1) {
    if (per_lane) SPRAY_AH_LAUNCH(1, 0);
    else SPRAY_AH_LAUNCH(1, 1);
  } else {
    if (per_lane) SPRAY_AH_LAUNCH(4, 0);
    else SPRAY_AH_LAUNCH(4, 1);
  }
#undef SPRAY_AH_LAUNCH
  return hipGetLastError();
}

}  // namespace spray_rt
