// rt_kernels.hip -- gfx950 kernels of the intersect / occluded hot path.
//
// One lane = one ray.  Per lane: a short traversal stack in LDS laid out
// [depth][lane] (consecutive lanes hit consecutive banks), BVH2 nodes read as
// four 16-B loads, triangles as three 16-B loads.  Compiled with
// -ffp-contract=off: every fused multiply-add below is an explicit fmaf(), so
// t/u/v/Ng are bit-identical to the CPU oracle (oracle/oracle.c) and to every
// other kernel here -- VBuf compares t with == (ooc_vbuf.cc:41-52).
#include <hip/hip_runtime.h>

#include <type_traits>

#include <hipcub/block/block_reduce.hpp>
#include <hipcub/block/block_scan.hpp>

#include <climits>
#include <cstdint>

#include "cam_device.h"
#include "rt_device.h"
#include "shade_device.h"

namespace spray_rt {
namespace {

// Work distribution of the scene kernels (measured, profiles/): closest hit
// = persistent waves dequeuing 256-ray chunks (four neighbouring packets,
// which share the scalar cache) from per-XCD band queues (1.02 -> 0.71 ms:
// no block-coupled wave lifetimes, band-local L2; 128 -> 256 with the
// dequeue during the last packet, SPRAY_DEQ_AHEAD: fused launch 0.759 ->
// 0.744 ms, DESIGN §4 "Launch tail"); any hit
// = one ray per lane over a plain grid for batches below kPersistAhRays
// (shadow batches: the persistent tail costs more than it saves, 0.27 vs
// 0.33 ms), persistent above it (AO-16 batches, 36.6 M rays: 6.23 -> 5.71 ms
// per AO step).  SPRAY_PERSIST_*/SPRAY_CHUNK_* select the other forms in
// diagnostic builds.
#ifndef SPRAY_CHUNK_CH
#define SPRAY_CHUNK_CH 256
#endif
#ifndef SPRAY_CHUNK_AH
#define SPRAY_CHUNK_AH 128
#endif
#ifndef SPRAY_PERSIST_CH
#define SPRAY_PERSIST_CH 1
#endif
#ifndef SPRAY_PERSIST_AH
#define SPRAY_PERSIST_AH 0
#endif
constexpr size_t kPersistAhRays = size_t(16) << 20;  // any-hit batches this large persist

// Minimum resident waves per SIMD the register allocator must allow (the
// second __launch_bounds__ operand); 1 = unconstrained.
// Per-lane any hit: 1 = while-while walk with postponed leaves, 0 = the
// canonical closest-child-first walk.
#ifndef SPRAY_AH_WW
#define SPRAY_AH_WW 1
#endif
// Per-lane while-while any hit over the 64-B 4-wide quantized node copy
// (QNode4) of scene slots: 1 = quantized 4-wide nodes, 0 = the fp32 BVH2.
#ifndef SPRAY_AH_QNODES
#define SPRAY_AH_QNODES 1
#endif
#ifndef SPRAY_WAVES_CH
#define SPRAY_WAVES_CH 6
#endif
// the keyed closest hit + shading of in-situ frames (5 / 4 waves per SIMD:
// rank launches at N = 8 0.185 / 0.188 vs 0.195 ms, at N = 2 0.319 / 0.328
// vs 0.311 ms -- within the run-to-run spread)
#ifndef SPRAY_WAVES_KEYED
#define SPRAY_WAVES_KEYED 6
#endif
#ifndef SPRAY_WAVES_SHADOW
#define SPRAY_WAVES_SHADOW 6
#endif
#ifndef SPRAY_WAVES_AH
#define SPRAY_WAVES_AH 1
#endif
// LDS entries of the AO any hit's per-lane stack (the rest of kQ4Stack is
// private): 8 instead of the launch's 16 leaves LDS for 8 blocks per CU, and
// the register budget of 8 waves per SIMD (64 VGPRs) holds the 4-wide walk
// (measured: AO any hit 4.12 / 4.14 ms at 6 waves with 16 entries -> 3.93 /
// 3.94 at 7 waves with 12 or 8 -> 3.85 / 3.85 at 8 waves with 8; same bits)
#ifndef SPRAY_AOGEN_LSTK
#define SPRAY_AOGEN_LSTK 8
#endif
#ifndef SPRAY_WAVES_AOGEN
#define SPRAY_WAVES_AOGEN 8
#endif

// ---------------------------------------------------------------------------
// Embree-layout streams (RTCRayIntersection / RTCRay, byte stride)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int find_segment(const size_t* off, int nseg,
                                            size_t i) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {  // last segment with off[seg] <= i
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kBlock) void k_rtc_intersect(
    const SlotDesc* __restrict__ slots, const int* __restrict__ seg_slot,
    const size_t* __restrict__ seg_off, int nseg, char* __restrict__ rays,
    size_t stride, size_t M) {
  __shared__ int32_t stack[kStack * kBlock];
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  const int seg = nseg == 1 ? 0 : find_segment(seg_off, nseg, i);
  const int slot = seg_slot[seg];
  const SlotDesc s = slots[slot];
  char* rec = rays + i * stride;
  const float* f = reinterpret_cast<const float*>(rec);
  const Ray r = make_ray(f[0], f[1], f[2], f[4], f[5], f[6]);
  const float tnear = f[8];
  Best best{f[9], 0xFFFFFFFFu, 0u};
  unsigned a = 0, b = 0;
  if (s.nnodes)
    trace_slot<false, false>(s, r, tnear, 0.f, best, stack + threadIdx.x, a, b);
  if (best.prim == 0xFFFFFFFFu) return;  // miss: record untouched
  float hu, hv;
  const float4 c = hit_uv(s, r, tnear, best.leaf, hu, hv);
  uint32_t color;
  float nsx, nsy, nsz;
  epilogue(s, best.prim, hu, hv, color, nsx, nsy, nsz);
  float* o = reinterpret_cast<float*>(rec);
  uint32_t* ou = reinterpret_cast<uint32_t*>(rec);
  o[9] = best.t;          // tfar
  o[12] = c.y;            // Ng
  o[13] = c.z;
  o[14] = c.w;
  ou[15] = color;         // color (offset 60)
  o[16] = hu;
  o[17] = hv;
  ou[18] = 0u;            // geomID (one mesh per slot)
  ou[19] = best.prim;     // primID
  o[21] = nsx;            // Ns (offset 84)
  o[22] = nsy;
  o[23] = nsz;
}

// TriMeshBuffer::updateIntersection (src/render/trimesh_buffer.cc:328-360)
// on its own: color and Ns of every record whose geomID says hit, from its
// primID, u and v -- the epilogue k_rtc_intersect fuses, same operations.
__global__ __launch_bounds__(kBlock) void k_rtc_update(
    const SlotDesc* __restrict__ slots, const int* __restrict__ seg_slot,
    const size_t* __restrict__ seg_off, int nseg, char* __restrict__ rays,
    size_t stride, size_t M) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  const int seg = nseg == 1 ? 0 : find_segment(seg_off, nseg, i);
  const SlotDesc s = slots[seg_slot[seg]];
  char* rec = rays + i * stride;
  uint32_t* ou = reinterpret_cast<uint32_t*>(rec);
  float* o = reinterpret_cast<float*>(rec);
  if (ou[18] == 0xFFFFFFFFu || ou[19] >= s.ntris) return;  // no hit / not this mesh
  uint32_t color;
  float nsx, nsy, nsz;
  epilogue(s, ou[19], o[16], o[17], color, nsx, nsy, nsz);
  ou[15] = color;
  o[21] = nsx;
  o[22] = nsy;
  o[23] = nsz;
}

__global__ __launch_bounds__(kBlock) void k_rtc_occluded(
    const SlotDesc* __restrict__ slots, const int* __restrict__ seg_slot,
    const size_t* __restrict__ seg_off, int nseg, char* __restrict__ rays,
    size_t stride, size_t M) {
  __shared__ int32_t stack[kStack * kBlock];
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  const int seg = nseg == 1 ? 0 : find_segment(seg_off, nseg, i);
  const SlotDesc s = slots[seg_slot[seg]];
  char* rec = rays + i * stride;
  const float* f = reinterpret_cast<const float*>(rec);
  const Ray r = make_ray(f[0], f[1], f[2], f[4], f[5], f[6]);
  Best best{0.f, 0u, 0u};
  unsigned a = 0, b = 0;
  if (s.nnodes &&
      trace_slot<true, false>(s, r, f[8], f[9], best, stack + threadIdx.x, a, b))
    reinterpret_cast<uint32_t*>(rec)[18] = 0u;  // geomID = 0: occluded
}

// ---------------------------------------------------------------------------
// domain lists (WbvhEmbree::intersect + DomainList::sort)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_domains(
    const float* __restrict__ boxes, int ndom, const float* __restrict__ org,
    const float* __restrict__ dir, size_t M, int* __restrict__ ids,
    float* __restrict__ ts, int* __restrict__ counts, int maxhits) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  const DRay r = make_dray(org[3 * i], org[3 * i + 1], org[3 * i + 2],
                           dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
  // selection: k-th entry = smallest (t, id) strictly after the previous one
  float pt = -kInf;
  int pid = -1;
  int n = 0;
  for (; n < maxhits; ++n) {
    float bt = kInf;
    int bid = -1;
    for (int b = 0; b < ndom; ++b) {
      float tm;
      if (!aabb_ref(boxes + 6 * b, r, tm)) continue;
      const bool after = tm > pt || (tm == pt && b > pid);
      if (!after) continue;
      if (bid < 0 || tm < bt) {
        bt = tm;
        bid = b;
      }
    }
    if (bid < 0) break;
    ids[i * maxhits + n] = bid;
    ts[i * maxhits + n] = bt;
    pt = bt;
    pid = bid;
  }
  counts[i] = n;
}


// ---------------------------------------------------------------------------
// fused scene path
// ---------------------------------------------------------------------------
// Domains of a ray are visited in (tmin, id) order (DomainList::sort); the
// closest hit is carried across domains, a later domain replacing it only
// when strictly nearer -- the earlier list entry wins a tie.
// The domain mask comes from the top-level tree (exact union boxes, exact
// intersectAabb at every node: monotone, so it equals the brute-force test).
struct SceneArgs {
  const SlotDesc* slots;
  const int* dom2slot;
  const DomTrav* domtrav;
  const float* boxes;
  int ndom;
  const BvhNode* tlas;
  int ntlas;
  const spray_rt_ray* rays;
  size_t M;
  const uint32_t* d_count;  // device ray count (spawned rays) or null
  spray_rt_hit* hits;
  uint8_t* occ;
  unsigned long long* counters;
  uint32_t* heads;  // kQueues queue heads, 32 words apart (persistent launch)
  int persist;      // any hit: persistent waves (set by the launcher)
  int heads_ready;  // heads zeroed by the caller (no memset before the launch)
  int count_ready;  // sh_count zeroed by the caller
  // fused PT shadow spawn (closest hit): positional output
  ShadePt shade;
  spray_rt_ray* sh_out;  // [M] shadow ray of source i (valid entries only)
  uint8_t* sh_valid;     // [M] 1 if source i spawned a shadow ray
  uint32_t* sh_count;    // optional total
  float4* sw;            // kEpiShadowFrame: light weight of source i's shadow ray
  // indexed input: slot j traces ray idx[j] (e.g. a selected sparse subset)
  const uint32_t* idx;
  // kEpiKeys: composite key per ray
  uint64_t* keys;
  // positional mask: only rays with valid[i] != 0 are traced (occ / hits of
  // the others untouched)
  const uint8_t* valid;
  // kEpiAoGen: ray k is AO sample (ao_pairs[k] & 31) of source ray
  // ao_pairs[k] >> 5, generated in the lane (ooc::ShaderAo's spawn) instead
  // of read from rays
  const uint32_t* ao_pairs;
  const float4* ao_rec;  // per source ray: (origin, pixel), normal, tangent frame
  const float4* ao_lv;   // local hemisphere sample of (pixel, l) at pixel * ao_ns + l
  int ao_ns;
  // replicated AO frames: an occluded pair also sets its count field (fb
  // bits at (source, sample) position source * ao_ns + sample) here
  uint32_t* ao_fields;
  int ao_fb;
  // replicated frames: t bits per slot (kEpiKeysShade), the group's minimum
  // t bits per slot (kEpiShadowGen; 0xFFFFFFFF: no hit)
  uint32_t* tkeys;
  const uint32_t* tmin;
  size_t nrays;  // index lists: ray ids idx[j] < nrays (0: < M)
  // replicated frames from the camera (cam_runs != null): work item j is
  // sample j of table cam's pixels, generated in the lane, results at its
  // U slot (cam_item)
  CamTable cam_tab;
  Cam cam;
  int cam_w, cam_spp;
  // camera frames of a rank holding few domains: a lane's domain list is its
  // test of the rank's resident boxes (no top-level walk); keyed launches
  // leave the list-position byte of the key 0 (launch_cam_lp fills it in)
  int direct_res;
};

// Packet path ray loads / hit stores: 1 = non-temporal, so the 671 MB of
// rays and records streamed through a frame do not evict BVH nodes from L2
// (measured: fused step 0.848 / 0.828 vs 0.868 / 0.843 ms on one box).
#ifndef SPRAY_NT_IO
#define SPRAY_NT_IO 1
#endif
// Packet path hit records of a full wave of consecutive rays: 1 = three
// wave-wide 1-KB stores (records transposed across the lanes), 0 = three
// strided 16-B stores per lane.
#ifndef SPRAY_HIT_TRANSPOSE
#define SPRAY_HIT_TRANSPOSE 1
#endif
// Closest-hit packet walks of plain ray buffers: 1 = the next packet of the
// chunk is copied global -> LDS (global_load_lds, no VGPRs) while the
// current packet walks, so its rays are waiting in LDS when it starts.
#ifndef SPRAY_RAY_PREFETCH
#define SPRAY_RAY_PREFETCH 1
#endif
// cache policy of those copies (gfx950 CPol: 2 = nt, the non-temporal hint
// of the plain ray loads, SPRAY_NT_IO)
#ifndef SPRAY_GLDS_AUX
#define SPRAY_GLDS_AUX 0
#endif
typedef __attribute__((address_space(1))) const void* glds_src_t;
typedef __attribute__((address_space(3))) void* glds_dst_t;
// The same for the per-lane path's ray loads and the AO rays' stores
// (measured: AO step 6.27 vs 6.41 ms).
#ifndef SPRAY_NT_IO_LANE
#define SPRAY_NT_IO_LANE 1
#endif

// Closest-hit epilogue variants of the scene kernels.
constexpr int kEpiNone = 0;   // hit records only
constexpr int kEpiSpawn = 1;  // + fused PT shadow spawn (positional)
constexpr int kEpiKeys = 2;   // + 64-bit composite key (t, list position, domain)
constexpr int kEpiShadow = 3; // + PT spawn and the shadow ray's any hit, same launch
// kEpiShadow for a frame's camera rays: the spawn rule and the light weight of
// ooc::ShaderPt's shading pass (k_shade, one point light, path weight 1),
// the weight written to sw[i] for the film
constexpr int kEpiShadowFrame = 4;
// any hit of AO rays generated in the lane from (source ray, sample) pairs
constexpr int kEpiAoGen = 5;
// kEpiAoGen for replicated AO frames: an occluded pair also sets its count
// field (A.ao_fields) -- its own instantiation, so the one-GPU AO kernel
// carries none of it
constexpr int kEpiAoGenF = 8;
constexpr bool ao_epi(int e) { return e == kEpiAoGen || e == kEpiAoGenF; }
// replicated in-situ frames (insitu.cpp trace_replicated): slot j traces ray
// idx[j] and writes its results at j.  kEpiKeysShade: the keyed closest hit
// over the rank's domains + the t bits (tkeys) + the point-light shading of
// the rank's own hit (sw / sh_valid, shade_pt_point); kEpiShadowGen (any
// hit): the shadow ray of the group's minimum t (tmin), built in the lane
// with shade_pt_point's operations, occ[j].
constexpr int kEpiKeysShade = 6;
constexpr int kEpiShadowGen = 7;
constexpr bool rep_epi(int e) { return e == kEpiKeysShade || e == kEpiShadowGen; }

// Band q of M rays = [q*S, min((q+1)*S, M)), S = band_size(M): one work
// queue of the persistent launches; bands 8x .. 8x+7 (a contiguous eighth of
// the rays) are the home queues of XCD x.
__device__ __host__ __forceinline__ size_t band_size(size_t M) {
  return (((M + kQueues - 1) / kQueues) + 63) / 64 * 64;
}

// LDS written by some lanes of a wave and read by others: ordered within
// the wave (no block barrier)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// AO ray k of a fused spawn + any hit: sample l of source ray i, (i, l) =
// (ao_pairs[k] >> 5, ao_pairs[k] & 31) -- the rotation of
// k_spawn_ao_write_hits on the same values: the hit's origin, normal and
// tangent frame from its record and the local hemisphere sample (the double
// sincos) from the (pixel, l) table, both written by k_spawn_ao_index, so
// the same bits as the written ray.
// the pair's operands: its source's record (origin + pixel, normal, tangent
// frame) and its hemisphere sample
struct AoSrc {
  float4 op, n4, x4, y4, l4;
};
__device__ __forceinline__ AoSrc ao_load(const SceneArgs& A, uint32_t pr) {
  const uint32_t i = pr >> 5, l = pr & 31u;
  const float4* rec = A.ao_rec + 4 * size_t(i);
  AoSrc o;
  o.op = rec[0];
  o.n4 = rec[1];
  o.x4 = rec[2];
  o.y4 = rec[3];
  o.l4 = A.ao_lv[size_t(__float_as_uint(o.op.w)) * uint32_t(A.ao_ns) + l];
  return o;
}
__device__ __forceinline__ void ao_ray(const AoSrc& o, v4f& a, v4f& b) {
  const float N[3] = {o.n4.x, o.n4.y, o.n4.z}, ax[3] = {o.x4.x, o.x4.y, o.x4.z},
              ay[3] = {o.y4.x, o.y4.y, o.y4.z};
  const float lv[3] = {o.l4.x, o.l4.y, o.l4.z};
  float w[3], pdf;
  hemisphere_apply(lv, N, ax, ay, w, pdf);
  a = v4f{o.op.x, o.op.y, o.op.z, kRayEpsilon};
  b = v4f{w[0], w[1], w[2], kInf};
}
__device__ __forceinline__ void ao_gen(const SceneArgs& A, size_t k, v4f& a, v4f& b) {
  ao_ray(ao_load(A, A.ao_pairs[k]), a, b);
}
// the count field of occluded pair k (the fields are zeroed per frame; the
// group's SUM of their bytes counts the ranks that found an occluder)
__device__ __forceinline__ void ao_field(const SceneArgs& A, size_t k) {
  const uint32_t pr = A.ao_pairs[k];
  const size_t pos = size_t(pr >> 5) * uint32_t(A.ao_ns) + (pr & 31u);
  const uint32_t per = 32u / uint32_t(A.ao_fb);
  atomicOr(A.ao_fields + pos / per, 1u << (uint32_t(pos % per) * uint32_t(A.ao_fb)));
}

// whether AO ray k enters a resident domain's box (replicated AO frames):
// the exact test (the top-level tree's leaf test), each box first through
// the fast slab on its kTopPad-padded copy (spad) -- the pair the top-level
// walk itself uses for its internal boxes, a superset of the exact test --
// so most boxes cost no double-precision test
// sun: the union of the resident padded boxes, tested first -- its slab
// accepts every ray a resident padded box accepts (the slab is monotone in
// the bounds), so a ray it rejects enters no resident box; the exact test's
// inverse direction is formed only once a padded box passes
__device__ __forceinline__ bool ao_own(const AoSrc& o, const float* sbox, const float* spad,
                                       const float* sun, const uint8_t* sres, int nres) {
  v4f a, b;
  ao_ray(o, a, b);
  const Ray r = make_ray(a.x, a.y, a.z, b.x, b.y, b.z);
  float tm;
  if (!slab(r, sun[0], sun[1], sun[2], sun[3], sun[4], sun[5], 0.f, kInf, tm)) return false;
  for (int q = 0; q < nres; ++q) {
    const int d = int(sres[q]);
    const float* pb = spad + 6 * d;
    if (!slab(r, pb[0], pb[1], pb[2], pb[3], pb[4], pb[5], 0.f, kInf, tm)) continue;
    const DRay dr = make_dray(a.x, a.y, a.z, b.x, b.y, b.z);
    if (aabb_ref(sbox + 6 * d, dr, tm)) return true;
  }
  return false;
}

template <int W, bool ANY, bool COUNT, int EPI, int STK>
__device__ __forceinline__ void scene_ray(const SceneArgs& A, size_t i,
                                          const float4* stl, const float* sbox,
                                          const float4* sdom, int32_t* stk, int32_t* wstk,
                                          unsigned& nnode, unsigned& ntri,
                                          unsigned& nvisit, bool& spawn, float* pos,
                                          float* wi, const float* rin = nullptr) {
  constexpr bool kKeysL = EPI == kEpiKeys || EPI == kEpiKeysShade;
  const SlotDesc* __restrict__ slots = A.slots;
  const int* __restrict__ dom2slot = A.dom2slot;
  const int ntlas = A.ntlas;
  spray_rt_hit* __restrict__ hits = A.hits;
  uint8_t* __restrict__ occ = A.occ;
  {
    v4f a, b;
    if (ao_epi(EPI)) {
      ao_gen(A, i, a, b);
    } else if (rin) {  // a replicated frame's ray (rep_ray), results at i
      a = v4f{rin[0], rin[1], rin[2], kRayEpsilon};
      b = v4f{rin[3], rin[4], rin[5], kInf};
    } else {
      const v4f* rp = reinterpret_cast<const v4f*>(A.rays + i);
      if (SPRAY_NT_IO_LANE) {
        a = __builtin_nontemporal_load(rp);
        b = __builtin_nontemporal_load(rp + 1);
      } else {
        a = rp[0];
        b = rp[1];
      }
    }
    const float4 o4 = make_float4(a.x, a.y, a.z, a.w), d4 = make_float4(b.x, b.y, b.z, b.w);
    const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
    uint64_t m[W];
#pragma unroll
    for (int w = 0; w < W; ++w) m[w] = 0;
    tlas_mask_wave<W>(stl, ntlas, wstk, r, o4, d4, m);
    // Closest hit keeps (t, prim, leaf) of the running winner in place.  A
    // later domain may only win with a strictly smaller t (the earlier
    // entry of the sorted domain list wins ties): its traversal starts with
    // the tie-break key at 0, and leaf at a sentinel tells whether it won.
    Best best{ANY ? 0.f : d4.w, 0xFFFFFFFFu, 0xFFFFFFFFu};
    int best_dom = -1;
    uint32_t it = 0, best_it = 0;  // list positions (kEpiKeys only)
    bool occluded = false;
    for (;;) {
      float st = kInf;
      int sb = -1;
      bool any_left = false;
#pragma unroll
      for (int w = 0; w < W; ++w) any_left |= m[w] != 0;
      if (!any_left) break;
      {
        // the reference's domain ray (division-based inverse), rebuilt per
        // selection: keeping it live through trace_slot costs occupancy
        float dx = r.dx, dy = r.dy, dz = r.dz;
        asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz));
        const DRay dr = make_dray(r.ox, r.oy, r.oz, dx, dy, dz);
#pragma unroll
        for (int w = 0; w < W; ++w) {
          uint64_t bits = m[w];
          while (bits) {
            const int j = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            const int b = 64 * w + j;
            float tm;
            aabb_ref(sbox + 6 * b, dr, tm);
            if (sb < 0 || tm < st) {
              st = tm;
              sb = b;
            }
          }
        }
      }
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (w == (sb >> 6)) m[w] &= ~(1ull << (sb & 63));
      const uint32_t pos_sb = it;
      if (kKeysL) ++it;
      const float4 dt = sdom[sb];
      const char* nodes = reinterpret_cast<const char*>(
          (uint64_t(__float_as_uint(dt.y)) << 32) | __float_as_uint(dt.x));
      if (!nodes) continue;  // not resident here (or empty)
      const void* tris = nodes + __float_as_uint(dt.z);
      const uint32_t* prims = reinterpret_cast<const uint32_t*>(nodes + __float_as_uint(dt.w));
      if (COUNT) ++nvisit;
      if (ANY) {
        // the counting build walks in the canonical order the byte formula
        // is defined on; the fast build postpones leaves (same result)
        const bool o = (COUNT || SPRAY_AH_WW == 0)
                           ? trace_tree<true, COUNT>(nodes, tris, prims, r, o4.w, d4.w, best,
                                                     stk, nnode, ntri)
                           : SPRAY_AH_QNODES ? occluded_tree_q4<STK>(nodes, tris, r, o4.w, d4.w, stk)
                                             : occluded_tree_ww(nodes, tris, r, o4.w, d4.w, stk);
        if (o) {
          occluded = true;
          break;
        }
      } else {
        const uint32_t keep_prim = best.prim, keep_leaf = best.leaf;
        if (best_dom >= 0) best.prim = 0u;  // strictly nearer from now on
        best.leaf = 0xFFFFFFFFu;
        trace_tree<false, COUNT>(nodes, tris, prims, r, o4.w, 0.f, best, stk, nnode,
                                 ntri);
        if (best.leaf != 0xFFFFFFFFu) {
          best_dom = sb;
          if (kKeysL) best_it = pos_sb;
        } else {
          best.prim = keep_prim;
          best.leaf = keep_leaf;
        }
      }
    }
    if (ANY) {
      occ[i] = occluded ? 1 : 0;
      if (EPI == kEpiAoGenF && occluded) ao_field(A, i);
    } else {
      float4 h0, h1, h2;
      if (best_dom < 0) {
        h0 = make_float4(kInf, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu));
        h1 = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
        h2 = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
      } else {
        const SlotDesc s = slots[dom2slot[best_dom]];
        float hu, hv;
        const float4 c = hit_uv(s, r, o4.w, best.leaf, hu, hv);
        uint32_t color;
        float nsx, nsy, nsz;
        epilogue(s, best.prim, hu, hv, color, nsx, nsy, nsz);
        h0 = make_float4(best.t, hu, hv, __uint_as_float(best.prim));
        h1 = make_float4(c.y, c.z, c.w, __uint_as_float(color));
        h2 = make_float4(nsx, nsy, nsz, __int_as_float(best_dom));
      }
      if (!((EPI == kEpiKeysShade || EPI == kEpiShadowFrame) && !hits)) {
        float4* hp = reinterpret_cast<float4*>(hits + i);
        hp[0] = h0;
        hp[1] = h1;
        hp[2] = h2;
      }
      if (kKeysL) {
        // in-situ compositing key: the order of the sequential domain walk
        // (t, then the earlier entry of the sorted domain list), unique per
        // domain; misses sort last
        A.keys[i] = best_dom < 0 ? 0x7FFFFFFFFFFFFFFFull
                                 : (uint64_t(__float_as_uint(best.t)) << 32) |
                                       (uint64_t(best_it) << 16) | uint64_t(best_dom);
      }
      if (EPI == kEpiKeysShade) {  // the replicated frame (one round, per lane)
        A.tkeys[i] = best_dom >= 0 ? __float_as_uint(best.t) : 0xFFFFFFFFu;
        if (A.sh_valid) {
          bool sp = false;
          if (best_dom >= 0) {
            spray_rt_hit h;
            h.t = h0.x;
            h.color = __float_as_uint(h1.w);
            h.ns[0] = h2.x;
            h.ns[1] = h2.y;
            h.ns[2] = h2.z;
            const float d3[3] = {d4.x, d4.y, d4.z}, o3[3] = {o4.x, o4.y, o4.z};
            float L[3];
            sp = shade_pt_point(o3, d3, h, A.shade, pos, wi, L);
            if (sp) A.sw[i] = make_float4(L[0], L[1], L[2], 0.f);
          }
          A.sh_valid[i] = sp;
        }
      }
      if (EPI == kEpiSpawn && best_dom >= 0) {
        spray_rt_hit h;
        h.t = h0.x;
        h.color = __float_as_uint(h1.w);
        h.ns[0] = h2.x;
        h.ns[1] = h2.y;
        h.ns[2] = h2.z;
        h.domain = best_dom;
        spray_rt_ray ray;
        ray.org[0] = o4.x;
        ray.org[1] = o4.y;
        ray.org[2] = o4.z;
        ray.dir[0] = d4.x;
        ray.dir[1] = d4.y;
        ray.dir[2] = d4.z;
        spawn = shadow_pt(ray, h, A.shade, pos, wi);
      }
    }
  }
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

// A wave's rays are coherent when every direction is within ~8 degrees of
// the first valid lane's (camera rays of neighbouring pixels, shadow rays
// toward one point light); hemisphere-sampled AO rays are not, and walk
// per lane.
__device__ __forceinline__ bool wave_coherent(const SceneArgs& A, size_t i, bool valid) {
  float dx = 0.f, dy = 0.f, dz = 0.f;
  if (valid) {
    const float4 d4 = reinterpret_cast<const float4*>(A.rays + i)[1];
    dx = d4.x;
    dy = d4.y;
    dz = d4.z;
  }
  const uint64_t vb = __ballot(valid);
  if (!vb) return true;
  const int lead = __ffsll((long long)vb) - 1;
  const float lx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dx), lead));
  const float ly = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dy), lead));
  const float lz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), lead));
  const float c = (dx * lx + dy * ly) + dz * lz;
  return __ballot(valid && !(c >= 0.99f)) == 0;
}

// The fast (non-counting) form of scene_ray, run by the whole wave: rays of
// lanes with valid == false only take part in the collective steps.  The
// wave walks the union of its lanes' domain lists, one domain at a time --
// the nearest remaining domain of the first lane that still has one -- and
// traverses each domain tree as a packet (trace_tree_packet).  Lanes meet
// their domains out of list order, so a lane's running hit is replaced by a
// nearer t, or by an equal t of an earlier list entry (smaller (box entry
// t, id)); that is exactly the sequential walk's result.
// rin (optional): the lane's ray as org[3], dir[3] (a shadow ray queued in
// LDS, tnear = SPRAY_RAY_EPSILON, tfar = +inf) instead of A.rays[i]; i is
// then only the index its result is written at.
struct NoPost {
  __device__ void operator()() const {}
};
// post (optional): called once the lane's ray has arrived -- a vector-memory
// operation it issues (the steal scheduler's next-packet claim) then
// overlaps the walk, whose node and triangle fetches are scalar loads and
// whose stack is LDS: no vmcnt wait until the epilogue's gathers.  (Issued
// before the ray loads' wait it would be waited for with them: vector
// memory returns in order.)
template <int W, bool ANY, int EPI, typename Post = NoPost>
__device__ __forceinline__ void scene_ray_packet(const SceneArgs& A, size_t i, bool valid,
                                                 const float4* stl, const float* sbox,
                                                 const float4* sdom, int32_t* wstk,
                                                 bool& spawn, float* pos, float* wi,
                                                 const float* rin = nullptr,
                                                 const Post& post = Post(),
                                                 const uint8_t* sres = nullptr, int nres = 0,
                                                 const float4* lray = nullptr) {
  const SlotDesc* __restrict__ slots = A.slots;
  const int* __restrict__ dom2slot = A.dom2slot;
  const int lane = threadIdx.x & 63;
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  if (lray) {
    // the wave's rays copied to LDS by the previous packet (global_load_lds:
    // lane l's 32 B at lray[l], lray[64 + l]); the copy is a vector-memory
    // operation hipcc does not count, so wait for it here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (valid) {
      o4 = lray[lane];
      d4 = lray[64 + lane];
    }
  } else if (valid && rin) {
    o4 = make_float4(rin[0], rin[1], rin[2], kRayEpsilon);
    d4 = make_float4(rin[3], rin[4], rin[5], kInf);
  } else if (valid) {
    const v4f* rp = reinterpret_cast<const v4f*>(A.rays + i);
    v4f a, b;
    if (SPRAY_NT_IO) {  // streamed once: keep L2 for the BVH
      a = __builtin_nontemporal_load(rp);
      b = __builtin_nontemporal_load(rp + 1);
    } else {
      a = rp[0];
      b = rp[1];
    }
    o4 = make_float4(a.x, a.y, a.z, a.w);
    d4 = make_float4(b.x, b.y, b.z, b.w);
  }
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  if constexpr (!std::is_same<Post, NoPost>::value) {
    // the ray registers are consumed here, so their wait is emitted before
    // the hook's operation (the compiler would otherwise schedule the hook
    // first and wait for both together)
    asm volatile("" ::"v"(o4.x), "v"(d4.x));
    post();
  }
  uint64_t m[W];
#pragma unroll
  for (int w = 0; w < W; ++w) m[w] = 0;
  const bool direct = sres && A.direct_res;  // wave-uniform
  if (valid && direct) {
    // exactly the mask's resident bits: tlas_mask_wave's leaf test is this
    // intersectAabb on the same box
    const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
    for (int k = 0; k < nres; ++k) {
      const int d = int(sres[k]);
      float tm;
      if (aabb_ref(sbox + 6 * d, dr, tm)) {
#pragma unroll
        for (int w = 0; w < W; ++w)
          if (w == (d >> 6)) m[w] |= 1ull << (d & 63);
      }
    }
  } else if (valid) {
    tlas_mask_wave<W>(stl, A.ntlas, wstk, r, o4, d4, m);
  }
  constexpr bool kKeys = EPI == kEpiKeys || EPI == kEpiKeysShade;
  uint64_t m0[kKeys ? W : 1];
  if (kKeys) {
#pragma unroll
    for (int w = 0; w < W; ++w) m0[w] = m[w];
  }
  Best best{ANY ? 0.f : d4.w, 0xFFFFFFFFu, 0xFFFFFFFFu};
  int best_dom = -1;
  bool occluded = false;
  for (;;) {
    bool has = false;
#pragma unroll
    for (int w = 0; w < W; ++w) has |= m[w] != 0;
    const uint64_t hb = __ballot(has);
    if (!hb) break;
    const int lead = __ffsll((long long)hb) - 1;
    int sb = 0;
    if (lane == lead) {
      // the lead lane's nearest remaining domain by the fast slab entry
      // distance: the order only steers culling, the merge below is exact
      float st = kInf;
      sb = -1;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t bits = m[w];
        while (bits) {
          const int j = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          const int b = 64 * w + j;
          const float* bx = sbox + 6 * b;
          float tm;
          slab(r, bx[0], bx[1], bx[2], bx[3], bx[4], bx[5], -kInf, kInf, tm);
          if (sb < 0 || tm < st) {
            st = tm;
            sb = b;
          }
        }
      }
    }
    const int d = __builtin_amdgcn_readlane(sb, lead);
    bool act = false;
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (w == (d >> 6)) {
        act = (m[w] >> (d & 63)) & 1ull;
        m[w] &= ~(1ull << (d & 63));
      }
    if (ANY) act = act && !occluded;
    if (!__ballot(act)) continue;
    const float4 dt = sdom[d];
    const uint32_t nlo = __builtin_amdgcn_readfirstlane(__float_as_uint(dt.x));
    const uint32_t nhi = __builtin_amdgcn_readfirstlane(__float_as_uint(dt.y));
    const uint64_t nodes = (uint64_t(nhi) << 32) | nlo;
    if (!nodes) continue;  // not resident here (or empty)
    const uint64_t tris = nodes + __builtin_amdgcn_readfirstlane(__float_as_uint(dt.z));
    const uint64_t prims = nodes + __builtin_amdgcn_readfirstlane(__float_as_uint(dt.w));
    if (ANY) {
      bool hit = false;
      trace_tree_packet<true>(nodes, tris, prims, r, o4.w, d4.w, best, act, hit, wstk);
      if (hit) {
        occluded = true;
#pragma unroll
        for (int w = 0; w < W; ++w) m[w] = 0;
      }
    } else {
      Best loc{best_dom == -1 ? d4.w : best.t, 0xFFFFFFFFu, 0xFFFFFFFFu};
      bool hit = false;
      trace_tree_packet<false>(nodes, tris, prims, r, o4.w, 0.f, loc, act, hit, wstk);
      if (loc.leaf != 0xFFFFFFFFu) {
        bool take = best_dom == -1 || loc.t < best.t;
        if (!take && loc.t == best.t && best_dom >= 0) {  // exact tie: the earlier list entry
          const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
          float tmd, tme;
          aabb_ref(sbox + 6 * d, dr, tmd);
          aabb_ref(sbox + 6 * best_dom, dr, tme);
          take = tmd < tme || (tmd == tme && d < best_dom);
        }
        if (take) {
          best = loc;
          best_dom = d;
        }
      }
    }
  }
  if (ANY) {
    if (valid) A.occ[i] = occluded ? 1 : 0;
    if (EPI == kEpiAoGenF && valid && occluded) ao_field(A, i);
    return;
  }
  float4 h0, h1, h2;  // invalid lanes: best_dom < 0, never stored
  if (best_dom < 0) {
    h0 = make_float4(kInf, 0.f, 0.f, __uint_as_float(0xFFFFFFFFu));
    h1 = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
    h2 = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  } else {
    const SlotDesc s = slots[dom2slot[best_dom]];
    float hu, hv;
    const float4 c = hit_uv(s, r, o4.w, best.leaf, hu, hv);
    uint32_t color;
    float nsx, nsy, nsz;
    epilogue(s, best.prim, hu, hv, color, nsx, nsy, nsz);
    h0 = make_float4(best.t, hu, hv, __uint_as_float(best.prim));
    h1 = make_float4(c.y, c.z, c.w, __uint_as_float(color));
    h2 = make_float4(nsx, nsy, nsz, __int_as_float(best_dom));
  }
  // A whole wave of consecutive records (64 x 48 B = 24 full 128-B lines)
  // goes out as three wave-wide 1-KB stores: lane l of store s writes 16-B
  // chunk g = 64 s + l of the wave's region, chunk g % 3 of record g / 3,
  // pulled from that record's lane (3 x 12 cross-lane reads).  The three
  // strided 16-B stores per lane left lines partially written between
  // instructions (WRITE_SIZE 1.25x the records).
  const size_t i0 = size_t(__builtin_amdgcn_readfirstlane(uint32_t(i))) |
                    (size_t(__builtin_amdgcn_readfirstlane(uint32_t(i >> 32))) << 32);
  if ((EPI == kEpiKeysShade || EPI == kEpiShadowFrame) && !A.hits) {
    // no hit records (the replicated frame keeps keys and shading only; an
    // in-situ frame without per-sample records keeps shading and shadows)
  } else if (SPRAY_HIT_TRANSPOSE && (i0 & 63) == 0 &&
      __ballot(valid && i == i0 + size_t(lane)) == ~0ull) {
    const float hv[12] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w,
                          h2.x, h2.y, h2.z, h2.w};
    v4f* wp = reinterpret_cast<v4f*>(A.hits + i0);
#pragma unroll
    for (int st = 0; st < 3; ++st) {
      const int g = 64 * st + lane;
      const int src = g / 3, ch = g - 3 * src;
      float o[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const float a0 = __shfl(hv[d], src), a1 = __shfl(hv[4 + d], src),
                    a2 = __shfl(hv[8 + d], src);
        o[d] = ch == 0 ? a0 : (ch == 1 ? a1 : a2);
      }
      if (SPRAY_NT_IO)
        __builtin_nontemporal_store(v4f{o[0], o[1], o[2], o[3]}, wp + g);
      else
        wp[g] = v4f{o[0], o[1], o[2], o[3]};
    }
  } else if (valid) {
    if (SPRAY_NT_IO) {
      v4f* hp = reinterpret_cast<v4f*>(A.hits + i);
      __builtin_nontemporal_store(v4f{h0.x, h0.y, h0.z, h0.w}, hp);
      __builtin_nontemporal_store(v4f{h1.x, h1.y, h1.z, h1.w}, hp + 1);
      __builtin_nontemporal_store(v4f{h2.x, h2.y, h2.z, h2.w}, hp + 2);
    } else {
      float4* hp = reinterpret_cast<float4*>(A.hits + i);
      hp[0] = h0;
      hp[1] = h1;
      hp[2] = h2;
    }
  }
  if (!valid) return;
  if (kKeys) {
    uint64_t key = 0x7FFFFFFFFFFFFFFFull;
    if (best_dom >= 0 && direct) {  // the position is filled in by launch_cam_lp
      key = (uint64_t(__float_as_uint(best.t)) << 32) | uint64_t(best_dom);
    } else if (best_dom >= 0) {  // position of best_dom in the ray's sorted list
      const DRay dr = make_dray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
      float tb;
      aabb_ref(sbox + 6 * best_dom, dr, tb);
      uint32_t p = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t bits = m0[w];
        while (bits) {
          const int j = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          const int b = 64 * w + j;
          float tm;
          aabb_ref(sbox + 6 * b, dr, tm);
          if (tm < tb || (tm == tb && b < best_dom)) ++p;
        }
      }
      key = (uint64_t(__float_as_uint(best.t)) << 32) | (uint64_t(p) << 16) |
            uint64_t(best_dom);
    }
    A.keys[i] = key;
    if (EPI == kEpiKeysShade) {
      A.tkeys[i] = best_dom >= 0 ? __float_as_uint(best.t) : 0xFFFFFFFFu;
      // no shading arrays: keys only (the replicated AO frame)
      if (!A.sh_valid) return;
      bool sp = false;
      if (best_dom >= 0) {
        spray_rt_hit h;
        h.t = h0.x;
        h.color = __float_as_uint(h1.w);
        h.ns[0] = h2.x;
        h.ns[1] = h2.y;
        h.ns[2] = h2.z;
        const float d3[3] = {d4.x, d4.y, d4.z}, o3[3] = {o4.x, o4.y, o4.z};
        float L[3];
        sp = shade_pt_point(o3, d3, h, A.shade, pos, wi, L);
        if (sp) A.sw[i] = make_float4(L[0], L[1], L[2], 0.f);
      }
      A.sh_valid[i] = sp;
    }
  }
  if (EPI == kEpiShadowFrame && best_dom >= 0) {
    spray_rt_hit h;
    h.t = h0.x;
    h.color = __float_as_uint(h1.w);
    h.ns[0] = h2.x;
    h.ns[1] = h2.y;
    h.ns[2] = h2.z;
    const float d3[3] = {d4.x, d4.y, d4.z}, o3[3] = {o4.x, o4.y, o4.z};
    float L[3];
    spawn = shade_pt_point(o3, d3, h, A.shade, pos, wi, L);
    if (spawn) A.sw[i] = make_float4(L[0], L[1], L[2], 0.f);
  }
  if ((EPI == kEpiSpawn || EPI == kEpiShadow) && best_dom >= 0) {
    spray_rt_hit h;
    h.t = h0.x;
    h.color = __float_as_uint(h1.w);
    h.ns[0] = h2.x;
    h.ns[1] = h2.y;
    h.ns[2] = h2.z;
    h.domain = best_dom;
    spray_rt_ray ray;
    ray.org[0] = o4.x;
    ray.org[1] = o4.y;
    ray.org[2] = o4.z;
    ray.dir[0] = d4.x;
    ray.dir[1] = d4.y;
    ray.dir[2] = d4.z;
    spawn = shadow_pt(ray, h, A.shade, pos, wi);
  }
}

// The ray slot j of a replicated-frame launch traces (rep_epi): eye ray
// idx[j] (kEpiKeysShade), or the point-light shadow ray of the group's
// minimum t of it (kEpiShadowGen: RTCRayUtil::hitPosition + PointLight::
// sample, the operations of shade_pt_point / k_rep_shadows, so the bits of
// the winner's own shadow ray); false: no ray (no hit anywhere).
// A lane whose ray enters none of the resident domains' boxes (the exact
// test of the top-level tree's leaves: its list holds no domain of this
// rank) is dropped before any walk: kEpiKeysShade writes its miss key, t
// bits and "no shading" here (every slot of C' is written by its lane, no
// prefill); kEpiShadowGen leaves its occlusion byte at the prefilled 0.
template <int EPI>
__device__ __forceinline__ bool rep_ray(const SceneArgs& A, size_t j, size_t i, bool ok, bool inb,
                                        size_t& at, float* r6, const float* sbox,
                                        const uint8_t* sres, int nres) {
  const bool cam = A.cam_tab.runs != nullptr;
  at = j;
  // a dropped slot of C' gets the miss results (every slot of C' is written
  // by its lane, no prefill); camera slots are prefilled (the memset of U)
  const auto miss = [&]() {
    if (EPI == kEpiKeysShade && !cam && inb) {
      A.keys[j] = 0x7FFFFFFFFFFFFFFFull;  // the epilogue's miss key (kInsituMissKey)
      A.tkeys[j] = 0xFFFFFFFFu;
      if (A.sh_valid) A.sh_valid[j] = 0;
    }
    return false;
  };
  float o[3], d[3];
  if (cam) {
    if (!inb) return false;
    int x, y, s;
    cam_item(A.cam_tab, A.cam_spp, j, x, y, s, at);
    float fx, fy;
    insitu_jitter(A.cam_w, A.cam_spp, x, y, s, fx, fy);
    cam_dir(A.cam, fx, fy, d);
    o[0] = A.cam.p[0];
    o[1] = A.cam.p[1];
    o[2] = A.cam.p[2];
  } else {
    if (!ok) return miss();
    const float4* rp = reinterpret_cast<const float4*>(A.rays + i);
    const float4 o4 = rp[0], d4 = rp[1];
    o[0] = o4.x;
    o[1] = o4.y;
    o[2] = o4.z;
    d[0] = d4.x;
    d[1] = d4.y;
    d[2] = d4.z;
  }
  if (EPI == kEpiKeysShade) {
    r6[0] = o[0];
    r6[1] = o[1];
    r6[2] = o[2];
    r6[3] = d[0];
    r6[4] = d[1];
    r6[5] = d[2];
  } else {
    const uint32_t tb = A.tmin[at];
    if (tb == 0xFFFFFFFFu) return false;
    const float t = __uint_as_float(tb);
    r6[0] = d[0] * t + o[0];
    r6[1] = d[1] * t + o[1];
    r6[2] = d[2] * t + o[2];
    float w[3] = {A.shade.lp[0] - r6[0], A.shade.lp[1] - r6[1], A.shade.lp[2] - r6[2]};
    gnorm3(w);
    r6[3] = w[0];
    r6[4] = w[1];
    r6[5] = w[2];
  }
  const DRay dr = make_dray(r6[0], r6[1], r6[2], r6[3], r6[4], r6[5]);
  for (int k = 0; k < nres; ++k) {
    float tm;
    if (aabb_ref(sbox + 6 * int(sres[k]), dr, tm)) return true;
  }
  return miss();
}

// When a wave takes its next chunk: packet kernels during the walk of the
// chunk's last packet, once that packet's rays have landed
// (scene_ray_packet's post hook: the atomic overlaps the walk and nothing
// waits in a wave's hands for longer than one packet; measured against
// dequeuing before / after the chunk, DESIGN.md section 4 "Launch tail");
// per-lane kernels after the chunk.

// Persistent launch: each wave dequeues kChunk-ray chunks from kQueues
// queues, each owning a contiguous band of the rays.  XCD x's waves start on
// its eight bands (an eighth of the image: its L2 holds the BVH nodes of that
// region), spread over them by block index so that no head counter sees more
// than 1/kQueues of the dequeues (same-address atomics serialise in L2), and
// then steal -- first within the XCD, then from the others.  A drained queue
// is recognised by a plain load of its head, so the end of the launch costs
// no atomics.  No wave waits on another.  The heads are zeroed by a memset
// before every launch.
// Positional spawn output: the shadow ray of source i goes to sh_out[i],
// sh_valid[i] says whether it exists; one atomic per wave for the total.
__device__ __forceinline__ void store_shadow(const SceneArgs& A, bool active,
                                             bool flag, size_t i,
                                             const float* pos, const float* wi,
                                             uint32_t& wcount) {
  if (active) {
    A.sh_valid[i] = flag ? 1 : 0;
    if (flag) {
      float4* op = reinterpret_cast<float4*>(A.sh_out + i);
      op[0] = make_float4(pos[0], pos[1], pos[2], kRayEpsilon);
      op[1] = make_float4(wi[0], wi[1], wi[2], kInf);
    }
  }
  wcount += uint32_t(__popcll(__ballot(flag)));
}

// The closest-hit register target (SPRAY_WAVES_CH) applies to the 16-entry
// stack over <= 64 domains; the 24-entry stack and the 256-domain tables
// are LDS-bound below it anyway.
// Fused shadow tracing (kEpiShadow): a per-wave LDS queue of the spawned
// point-light shadow rays.  A wave's chunks append their shadow rays until
// 64 are waiting, which then walk the scene as one any-hit packet -- right
// after their primary rays, while the nodes those just visited are still in
// the caches -- and the rest is traced when the wave runs out of work.
// occ[i] / sh_valid[i] are positional by source ray, as the two-launch form
// (spawn, select, any hit) writes them.
// capacity; a packet of min(waiting, 64) rays is traced once kShadowT wait
// (kShadowT - 1 waiting + 64 new fit): 128 / 64 = full packets only;
// smaller queues trade packet fill for LDS (more resident blocks)
#ifndef SPRAY_SHADOW_Q
#define SPRAY_SHADOW_Q 104
#endif
constexpr uint32_t kShadowQ = SPRAY_SHADOW_Q;
constexpr uint32_t kShadowT = kShadowQ - 64;
static_assert(kShadowQ > 64 && kShadowQ <= 128, "shadow queue capacity in (64, 128]");
struct ShadowQueue {
  float* ray;     // [kShadowQ][6]: org, dir
  uint32_t* src;  // [kShadowQ]: source ray index
  uint32_t n;     // waiting (wave-uniform)
};

template <int W>
__device__ __forceinline__ void shadow_trace(const SceneArgs& A, const ShadowQueue& q,
                                             uint32_t cnt, const float4* stl, const float* sbox,
                                             const float4* sdom, int32_t* wstk) {
  const uint32_t lane = threadIdx.x & 63;
  const bool v = lane < cnt;
  const size_t s = v ? q.src[lane] : 0;
  bool f = false;
  float p[3], w[3];
  scene_ray_packet<W, true, kEpiNone>(A, s, v, stl, sbox, sdom, wstk, f, p, w, q.ray + 6 * lane);
}

template <int W>
__device__ __forceinline__ void shadow_push(const SceneArgs& A, ShadowQueue& q, bool active,
                                            bool flag, size_t i, const float* pos,
                                            const float* wi, const float4* stl,
                                            const float* sbox, const float4* sdom,
                                            int32_t* wstk, uint32_t& wcount) {
  const uint32_t lane = threadIdx.x & 63;
  if (active) A.sh_valid[i] = flag ? 1 : 0;
  const unsigned long long bal = __ballot(flag);
  if (!bal) return;
  wcount += uint32_t(__popcll(bal));
  if (flag) {
    const uint32_t k = q.n + uint32_t(__popcll(bal & ((1ull << lane) - 1ull)));
    float* e = q.ray + 6 * k;
    e[0] = pos[0];
    e[1] = pos[1];
    e[2] = pos[2];
    e[3] = wi[0];
    e[4] = wi[1];
    e[5] = wi[2];
    q.src[k] = uint32_t(i);
  }
  q.n += uint32_t(__popcll(bal));
  if (q.n < kShadowT) return;
  wave_lds_sync();
  const uint32_t cnt = q.n < 64 ? q.n : 64u;
  shadow_trace<W>(A, q, cnt, stl, sbox, sdom, wstk);
  // the remainder (< 64) moves to the front
  const uint32_t rest = q.n - cnt;
  const bool mv = lane < rest;
  float e[6];
  uint32_t si = 0;
  if (mv) {
#pragma unroll
    for (int k = 0; k < 6; ++k) e[k] = q.ray[6 * (cnt + lane) + k];
    si = q.src[cnt + lane];
  }
  wave_lds_sync();
  if (mv) {
#pragma unroll
    for (int k = 0; k < 6; ++k) q.ray[6 * lane + k] = e[k];
    q.src[lane] = si;
  }
  wave_lds_sync();
  q.n = rest;
}


// STK: traversal-stack entries per lane, >= the depth of every resident
// slot tree and of the top-level tree (a node at depth k has at most k
// pending siblings).  LDS = STK KiB + 4 KiB per 64 domains, so STK 16 lets 8
// blocks (32 waves) share a CU where 24 allowed 5.
// TRAV: 0 per-lane walk, 1 packet walk, 2 packet walk for coherent waves
// and per-lane for the others (any-hit only; the counting variants always
// walk per lane, the canonical order the counts are defined on).
template <int W, bool ANY, bool COUNT, int EPI, int STK, int TRAV>
__global__ __launch_bounds__(kBlock, ANY ? (ao_epi(EPI) ? SPRAY_WAVES_AOGEN : SPRAY_WAVES_AH)
                                     : (W == 1 && STK == 16
                                            ? (EPI == kEpiShadow || EPI == kEpiShadowFrame ? SPRAY_WAVES_SHADOW
                                               : EPI == kEpiKeysShade ? SPRAY_WAVES_KEYED
                                                                 : SPRAY_WAVES_CH)
                                            : 1)) void k_scene(
    SceneArgs A) {
  // packet form for the non-counting kernels; any-hit waves fall back to
  // the per-lane walk when their rays are not coherent (AO hemispheres)
  constexpr bool kPacket = TRAV != 0 && !COUNT;
  constexpr bool kAdaptive = kPacket && TRAV == 2;
  constexpr bool kLaneStack = !kPacket || kAdaptive;
  // the AO any hit's 4-wide walk keeps kLStk entries in LDS and the rest of
  // its kQ4Stack in private memory (LDS for more resident blocks)
  constexpr int kLStk = (ANY && ao_epi(EPI) && !COUNT && SPRAY_AH_QNODES &&
                         SPRAY_AH_WW && SPRAY_AOGEN_LSTK < STK)
                            ? SPRAY_AOGEN_LSTK
                            : STK;
  __shared__ int32_t stack[(kLaneStack ? kLStk : 1) * kBlock];
  __shared__ float4 stl[4 * 64 * W];   // top-level tree
  __shared__ float sbox[6 * 64 * W];   // domain boxes (exact, for the sort)
  __shared__ float4 sdom[64 * W];      // DomTrav per domain
  // top-level / packet stacks, one per wave: STK entries suffice (the launch
  // picks STK >= every resident tree's depth and the top-level tree's), and
  // at STK 16 the any-hit kernels' 23.3 KB of LDS let 7 blocks share a CU
  __shared__ int32_t wstack[(kBlock / 64) * STK];
  constexpr bool kShadow = EPI == kEpiShadow || EPI == kEpiShadowFrame;
  __shared__ float sq_ray[kShadow ? (kBlock / 64) * kShadowQ * 6 : 1];
  // the next packet's rays, per wave (SPRAY_RAY_PREFETCH)
  constexpr bool kPre = SPRAY_RAY_PREFETCH && kPacket && !kAdaptive && !ANY && !rep_epi(EPI);
  __shared__ float4 spre[kPre ? (kBlock / 64) * 128 : 1];
  __shared__ uint32_t sq_src[kShadow ? (kBlock / 64) * kShadowQ : 1];
  ShadowQueue sq{sq_ray + (kShadow ? (threadIdx.x >> 6) * kShadowQ * 6 : 0),
                 sq_src + (kShadow ? (threadIdx.x >> 6) * kShadowQ : 0), 0u};
  size_t M = A.M;
  if (A.d_count) {  // ray count produced on the device
    const size_t dc = *A.d_count;
    M = dc < M ? dc : M;
  }
  const size_t S = band_size(M);
  // (camera launches testing the resident boxes directly never walk it)
  if (!(rep_epi(EPI) && A.direct_res))
    for (int k = threadIdx.x; k < 4 * A.ntlas; k += kBlock) stl[k] = ld4(A.tlas, k);
  for (int k = threadIdx.x; k < 6 * A.ndom; k += kBlock) sbox[k] = A.boxes[k];
  for (int k = threadIdx.x; k < A.ndom; k += kBlock) sdom[k] = ld4(A.domtrav, k);
  // replicated frames: the resident domains, whose boxes cull the lanes
  constexpr bool kRes = rep_epi(EPI);
  __shared__ uint8_t sres[kRes ? 64 * W : 1];
  __shared__ int nres;
  if (kRes) {
    __syncthreads();
    if (threadIdx.x == 0) {
      int k = 0;
      for (int d = 0; d < A.ndom; ++d)
        if (__float_as_uint(sdom[d].x) | __float_as_uint(sdom[d].y)) sres[k++] = uint8_t(d);
      nres = k;
    }
  }
  __syncthreads();
  unsigned nnode = 0, ntri = 0, nvisit = 0;
  int32_t* stk = stack + threadIdx.x;
  int32_t* wstk = wstack + (threadIdx.x >> 6) * STK;
  bool flag = false;
  float pos[3], wi[3];
  // spawned shadow rays of the wave, added to *sh_count once at its end (a
  // same-address atomic per chunk queued ~10^5 atomics behind each other)
  uint32_t wcount = 0;
  // persistent waves dequeue chunks; a launch of at most one packet per
  // resident wave runs one packet per wave instead (set by the launcher)
  const bool persist = A.persist != 0;
  const int lane = threadIdx.x & 63;
  const uint32_t* __restrict__ idx = A.idx;
  if (!persist) {
    const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
    const size_t i = (idx && j < M) ? idx[j] : j;
    // an index list entry past the ray buffer is skipped, never read
    const bool ok = j < M && i < (A.nrays ? A.nrays : A.M) && (!A.valid || A.valid[i]);
    if constexpr (rep_epi(EPI)) {
      float r6[6];
      size_t at;
      const bool okr = rep_ray<EPI>(A, j, i, ok, j < M, at, r6, sbox, sres, nres);
      scene_ray_packet<W, ANY, EPI == kEpiShadowGen ? kEpiNone : EPI>(
          A, at, okr, stl, sbox, sdom, wstk, flag, pos, wi, r6, NoPost(), sres, nres);
    } else if (kPacket && (!kAdaptive || wave_coherent(A, i, ok)))
      scene_ray_packet<W, ANY, EPI>(A, i, ok, stl, sbox, sdom, wstk, flag, pos, wi);
    else if (ok)
      scene_ray<W, ANY, COUNT, EPI, kLStk>(A, i, stl, sbox, sdom, stk, wstk, nnode, ntri,
                                      nvisit, flag, pos, wi);
    if (EPI == kEpiSpawn) store_shadow(A, j < M, flag, i, pos, wi, wcount);
    if (kShadow) shadow_push<W>(A, sq, j < M, flag, i, pos, wi, stl, sbox, sdom, wstk, wcount);
  } else {
    constexpr uint32_t kChunk = ANY ? SPRAY_CHUNK_AH : SPRAY_CHUNK_CH;
    constexpr uint32_t kPerXcd = kQueues / 8;
    // a batch of fewer than four kChunk chunks per wave (a rank's share of
    // a replicated frame) is dealt one packet per dequeue: with kChunk a few
    // waves take two chunks and walk their packets one after another while
    // the rest of the grid idles (measured: 331 K rays in 0.24 ms, the
    // latency of four packet walks in a row)
    const bool small = M < size_t(gridDim.x) * (kBlock / 64) * kChunk * 4;
    const uint32_t csz = small ? 64u : kChunk;
    // plain ray buffers: the chunk's next packet is prefetched into LDS
    const bool pre_on = kPre && !idx && !A.valid && !A.nrays;
    float4* wpre = spre + (kPre ? (threadIdx.x >> 6) * 128 : 0);
    bool have = false;  // wave-uniform: the next packet's rays are in wpre
    const uint32_t xcd = xcc_id() & 7u;
    const uint32_t sub = (blockIdx.x >> 3) % kPerXcd;
    for (uint32_t k = 0; k < uint32_t(kQueues); ++k) {
      const uint32_t q = ((xcd + k / kPerXcd) & 7u) * kPerXcd + (sub + k) % kPerXcd;
      const size_t begin = size_t(q) * S;
      const size_t end = begin + S < M ? begin + S : M;
      if (begin >= end) continue;
      uint32_t* head = &A.heads[32 * q];
      uint32_t base = 0;
      if (lane == 0) {
        base = __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (begin + base < end) base = atomicAdd(head, csz);
      }
      base = __builtin_amdgcn_readfirstlane(base);
      while (begin + base < end) {
        uint32_t next = 0;
        const size_t cbeg = begin + base;
        for (uint32_t c = 0; c < csz; c += 64) {
          const size_t j = cbeg + c + lane;
          const size_t i = (idx && j < end) ? idx[j] : j;
          const bool ok = j < end && i < (A.nrays ? A.nrays : A.M) && (!A.valid || A.valid[i]);
          flag = false;
          if (kPacket && !kAdaptive) {
            // the next chunk is dequeued by the chunk's last packet once its
            // rays have landed: the atomic overlaps that packet's walk, and
            // no chunk waits in a wave's hands while another is traced
            const bool last = c + 64 >= csz;
            float r6[6];
            size_t at = i;
            const bool okr =
                rep_epi(EPI) ? rep_ray<EPI>(A, j, i, ok, j < end, at, r6, sbox, sres, nres) : ok;
            // the chunk's next packet, copied to LDS during this one's walk
            const bool pre = pre_on && !last && cbeg + c + 64 < end;
            scene_ray_packet<W, ANY, EPI == kEpiShadowGen ? kEpiNone : EPI>(
                A, at, okr, stl, sbox, sdom, wstk, flag, pos, wi,
                rep_epi(EPI) ? r6 : nullptr,
                [&]() {
                  if (last && lane == 0) next = atomicAdd(head, csz);
                  if (kPre && pre && j + 64 < end) {
                    const spray_rt_ray* src = A.rays + (j + 64);
                    __builtin_amdgcn_global_load_lds((glds_src_t)src, (glds_dst_t)wpre, 16, 0, SPRAY_GLDS_AUX);
                    __builtin_amdgcn_global_load_lds(
                        (glds_src_t)(reinterpret_cast<const char*>(src) + 16),
                        (glds_dst_t)(wpre + 64), 16, 0, SPRAY_GLDS_AUX);
                  }
                },
                rep_epi(EPI) ? sres : nullptr, kRes ? nres : 0, kPre && have ? wpre : nullptr);
            // the next chunk's first packet: its head came back during this
            // walk; copied to LDS beside the epilogue and the shadow packets
            bool pre_next = false;
            if (kPre && last && pre_on) {
              const uint32_t nb = __builtin_amdgcn_readfirstlane(next);
              if (begin + nb < end) {
                const size_t jn = begin + nb + lane;
                if (jn < end) {
                  const spray_rt_ray* src = A.rays + jn;
                  __builtin_amdgcn_global_load_lds((glds_src_t)src, (glds_dst_t)wpre, 16, 0, SPRAY_GLDS_AUX);
                  __builtin_amdgcn_global_load_lds(
                      (glds_src_t)(reinterpret_cast<const char*>(src) + 16),
                      (glds_dst_t)(wpre + 64), 16, 0, SPRAY_GLDS_AUX);
                }
                pre_next = true;
              }
            }
            have = pre || pre_next;
          } else if (kPacket && wave_coherent(A, i, ok)) {
            scene_ray_packet<W, ANY, EPI>(A, i, ok, stl, sbox, sdom, wstk, flag, pos, wi);
          } else if (ok) {
            scene_ray<W, ANY, COUNT, EPI, kLStk>(A, i, stl, sbox, sdom, stk, wstk, nnode,
                                            ntri, nvisit, flag, pos, wi);
          }
          if (EPI == kEpiSpawn) store_shadow(A, j < end, flag, i, pos, wi, wcount);
          if (kShadow)
            shadow_push<W>(A, sq, j < end, flag, i, pos, wi, stl, sbox, sdom, wstk, wcount);
        }
        if (!(kPacket && !kAdaptive) && lane == 0) next = atomicAdd(head, csz);
        base = __builtin_amdgcn_readfirstlane(next);
      }
    }
  }
  if (kShadow && sq.n) {  // the wave's last shadow rays (fewer than 64)
    wave_lds_sync();
    shadow_trace<W>(A, sq, sq.n, stl, sbox, sdom, wstk);
  }
  if ((EPI == kEpiSpawn || kShadow) && A.sh_count && wcount && lane == 0)
    atomicAdd(A.sh_count, wcount);
  if (COUNT) {
    atomicAdd(&A.counters[0], (unsigned long long)nnode);
    atomicAdd(&A.counters[1], (unsigned long long)ntri);
    atomicAdd(&A.counters[2], (unsigned long long)nvisit);
  }
}

// In-situ routing (insitu::Isector::intersect, src/insitu/insitu_isector.h:
// 164-224, + InsituPartition::rank, src/render/data_partition.h:48-56): the
// set of ranks owning a domain on the ray's list, as a bitmask.
template <int W>
__global__ __launch_bounds__(kBlock) void k_route(const BvhNode* __restrict__ tlas,
                                                  int ntlas, const int* __restrict__ owner,
                                                  int ndom, const spray_rt_ray* __restrict__ rays,
                                                  const uint32_t* __restrict__ sel,
                                                  size_t M, uint64_t* __restrict__ out,
                                                  const uint8_t* __restrict__ valid,
                                                  unsigned long long* __restrict__ nvalid) {
  __shared__ int32_t wstack[(kBlock / 64) * kStack];
  __shared__ float4 stl[4 * 64 * W];
  __shared__ int sown[64 * W];
  for (int k = threadIdx.x; k < 4 * ntlas; k += kBlock) stl[k] = ld4(tlas, k);
  for (int k = threadIdx.x; k < ndom; k += kBlock) sown[k] = owner[k];
  __syncthreads();
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  // valid (optional): slot i holds a ray only where valid[i] (its mask is 0
  // otherwise; the wave still walks the top-level tree together)
  const bool live = !valid || valid[i];
  if (nvalid) {
    const uint64_t b = __ballot(live);
    if ((threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1)
      atomicAdd(nvalid, (unsigned long long)__popcll(b));
  }
  float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = make_float4(0.f, 0.f, 1.f, 0.f);
  if (live) {
    const float4* rp = reinterpret_cast<const float4*>(rays + (sel ? sel[i] : i));
    o4 = rp[0];
    d4 = rp[1];
  }
  uint64_t m[W];
  const Ray r = make_ray(o4.x, o4.y, o4.z, d4.x, d4.y, d4.z);
  tlas_mask_wave<W>(stl, ntlas, wstack + (threadIdx.x >> 6) * kStack, r, o4, d4, m);
  uint64_t ranks = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t bits = live ? m[w] : 0ull;
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      const int o = sown[64 * w + j];
      if (o >= 0) ranks |= 1ull << o;
    }
  }
  out[i] = ranks;
}

// ---------------------------------------------------------------------------
// ray sources
// ---------------------------------------------------------------------------

// ooc::Tracer::genMultiEyes (src/ooc/ooc_tracer.inl:124-172) + Camera::
// generateRay (camera.h:168-209), glm operand order: ray `bufid` of tile
// (tx, ty, tw), written at out[0] (pixid / samid optional).
__device__ __forceinline__ void eye_ray_ooc_xy(const Cam& cam, int image_w, int spp, int x, int y,
                                               size_t bufid, spray_rt_ray* out, int32_t* pixid,
                                               int32_t* samid) {
  float fx = float(x), fy = float(y);
  if (spp > 1) {
    uint32_t st = mm_fin(mm_mix(0u, uint32_t(bufid)));
    fx = float(x) + sampler_1d(st);
    fy = float(y) + sampler_1d(st);
  }
  const float* c = cam.p;
  const float u = fx / c[12], v = fy / c[13];
  float dx = ((c[3] + c[6] * u) + c[9] * v) - c[0];
  float dy = ((c[4] + c[7] * u) + c[10] * v) - c[1];
  float dz = ((c[5] + c[8] * u) + c[11] * v) - c[2];
  const float inv = 1.0f / sqrtf((dx * dx + dy * dy) + dz * dz);
  dx = dx * inv;
  dy = dy * inv;
  dz = dz * inv;
  float4* rp = reinterpret_cast<float4*>(out);
  rp[0] = make_float4(c[0], c[1], c[2], kRayEpsilon);
  rp[1] = make_float4(dx, dy, dz, kInf);
  if (pixid) *pixid = y * image_w + x;
  if (samid) *samid = int32_t(bufid);
}
__device__ __forceinline__ void eye_ray_ooc(const Cam& cam, int image_w, int spp, int tx, int ty,
                                            int tw, size_t bufid, spray_rt_ray* out,
                                            int32_t* pixid, int32_t* samid) {
  const int p = int(bufid / spp);
  eye_ray_ooc_xy(cam, image_w, spp, tx + p % tw, ty + p / tw, bufid, out, pixid, samid);
}

__global__ __launch_bounds__(kBlock) void k_eye_rays_ooc(
    Cam cam, int image_w, int spp, int tx, int ty, int tw, int th,
    spray_rt_ray* __restrict__ rays, int32_t* __restrict__ pixid,
    int32_t* __restrict__ samid) {
  const size_t bufid = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const size_t n = size_t(tw) * th * spp;
  if (bufid >= n) return;
  eye_ray_ooc(cam, image_w, spp, tx, ty, tw, bufid, rays + bufid, pixid ? pixid + bufid : nullptr,
              samid ? samid + bufid : nullptr);
}

// The eye rays of up to kEyeTiles tiles in one launch, tile k's at off[k]
// (each with its tile-local seeds, as one launch per tile writes them).
constexpr int kEyeTiles = 32;
struct EyeTiles {
  int n;
  int t[kEyeTiles][4];
  uint32_t off[kEyeTiles + 1];
};
__global__ __launch_bounds__(kBlock) void k_eye_rays_ooc_tiles(
    Cam cam, int image_w, int spp, EyeTiles T, spray_rt_ray* __restrict__ rays,
    int32_t* __restrict__ pixid, int32_t* __restrict__ samid) {
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= T.off[T.n]) return;
  int lo = 0, hi = T.n - 1;  // the last tile with off <= j
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (T.off[mid] <= j)
      lo = mid;
    else
      hi = mid - 1;
  }
  eye_ray_ooc(cam, image_w, spp, T.t[lo][0], T.t[lo][1], T.t[lo][2], j - T.off[lo], rays + j,
              pixid ? pixid + j : nullptr, samid ? samid + j : nullptr);
}

// The eye rays of run table T's pixels (render_tiles' footprint-culled
// frame): each run's ubase is the tile-local pixel id of its first pixel,
// so the slot cam_item returns is eye_ray_ooc's tile-local sample id and
// the ray, pixel and sample ids are the tile launch's, at compact index j.
__global__ __launch_bounds__(kBlock) void k_eye_rays_ooc_table(
    Cam cam, int image_w, int spp, CamTable T, spray_rt_ray* __restrict__ rays,
    int32_t* __restrict__ pixid, int32_t* __restrict__ samid) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= size_t(T.npix) * uint32_t(spp)) return;
  int x, y, s;
  size_t slot;
  cam_item(T, spp, j, x, y, s, slot);
  eye_ray_ooc_xy(cam, image_w, spp, x, y, slot, rays + j, pixid + j, samid + j);
}

// insitu::genMultiSampleEyeRays / genSingleSampleEyeRays (src/insitu/
// insitu_ray.h:103-182): stripe (tx, ty, tw, th) of blocking tile
// (bx, by, bw, bh); jitter seeded by (pixid, s); samid = blocking-tile-local
// sample id (the VBuf index).
__global__ __launch_bounds__(kBlock) void k_eye_rays_insitu(
    Cam cam, int image_w, int spp, int bx, int by, int bw, int tx, int ty, int tw,
    int th, spray_rt_ray* __restrict__ rays, int32_t* __restrict__ pixid,
    int32_t* __restrict__ samid) {
  const size_t bufid = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const size_t n = size_t(tw) * th * spp;
  if (bufid >= n) return;
  const int s = int(bufid % spp);
  const int p = int(bufid / spp);
  const int x = tx + p % tw, y = ty + p / tw;
  const int pid = image_w * y + x;
  float fx, fy;
  insitu_jitter(image_w, spp, x, y, s, fx, fy);
  float d[3];
  cam_dir(cam, fx, fy, d);
  const float* c = cam.p;
  float4* rp = reinterpret_cast<float4*>(rays + bufid);
  rp[0] = make_float4(c[0], c[1], c[2], kRayEpsilon);
  rp[1] = make_float4(d[0], d[1], d[2], kInf);
  if (pixid) pixid[bufid] = pid;
  if (samid)
    samid[bufid] = spp > 1 ? (bw * (y - by) + (x - bx)) * spp + s : bw * (y - by) + (x - bx);
}

__device__ __forceinline__ uint32_t block_prefix(bool flag, uint32_t& total) {
  // exclusive prefix of `flag` over the block (4 waves), in lane order
  __shared__ uint32_t wsum[kBlock / 64];
  const unsigned long long bal = __ballot(flag);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t in_wave =
      __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
  if (lane == 0) wsum[wave] = __popcll(bal);
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w) {
    if (w < wave) before += wsum[w];
    total += wsum[w];
  }
  return before + in_wave;
}

// single-block exclusive scan over nb block counts (coalesced 1024-wide
// chunks, hipCUB block scan); writes the total to *d_count
__global__ __launch_bounds__(1024) void k_scan_blocks(uint32_t* __restrict__ c,
                                                      uint32_t nb,
                                                      uint32_t* __restrict__ d_count) {
  using Scan = hipcub::BlockScan<uint32_t, 1024>;
  __shared__ typename Scan::TempStorage tmp;
  uint32_t run = 0;
  for (uint32_t base = 0; base < nb; base += 1024) {
    const uint32_t k = base + threadIdx.x;
    const uint32_t x = k < nb ? c[k] : 0u;
    uint32_t ex, agg;
    Scan(tmp).ExclusiveSum(x, ex, agg);
    if (k < nb) c[k] = run + ex;
    run += agg;
    __syncthreads();
  }
  if (threadIdx.x == 0) *d_count = run;
}

constexpr int kSelPer = 16;  // flags / masks per thread of the selection kernels
constexpr int kSelTile = kBlock * kSelPer;

// Exchange plan of a routed batch: for every destination rank d, the
// ascending indices of the rays whose mask has bit d, concatenated in rank
// order.  One wave owns kPlanWave consecutive rays (coalesced 8-B mask loads,
// 64 rays per step) and counts / places every rank's entries from the same
// load (one ballot per rank): count -> one exclusive scan over the
// [rank][wave tile] counts (rank-major, so the concatenation falls out) ->
// ordered write.  Lane d of a wave keeps rank d's running count / offset.
constexpr int kPlanSteps = 16;
constexpr size_t kPlanWave = 64 * kPlanSteps;

__global__ __launch_bounds__(kBlock) void k_plan_count(const uint64_t* __restrict__ m,
                                                       size_t n, int world, size_t wtiles,
                                                       uint32_t* __restrict__ tc) {
  const int lane = threadIdx.x & 63;
  const size_t wt = size_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  if (wt >= wtiles) return;  // whole waves
  const size_t base = wt * kPlanWave;
  uint32_t acc = 0;
  for (int p = 0; p < kPlanSteps; ++p) {
    const size_t i = base + size_t(p) * 64 + lane;
    const uint64_t v = i < n ? m[i] : 0ull;
    if (__ballot(v != 0ull) == 0ull) continue;
    for (int d = 0; d < world; ++d) {
      const uint32_t c = uint32_t(__popcll(__ballot((v >> d) & 1ull)));
      if (lane == d) acc += c;
    }
  }
  if (lane < world) tc[size_t(lane) * wtiles + wt] = acc;
}

__global__ __launch_bounds__(kBlock) void k_plan_write(const uint64_t* __restrict__ m,
                                                       size_t n, int world, size_t wtiles,
                                                       const uint32_t* __restrict__ tc,
                                                       int64_t* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const size_t wt = size_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  if (wt >= wtiles) return;
  const size_t base = wt * kPlanWave;
  uint32_t off = lane < world ? tc[size_t(lane) * wtiles + wt] : 0u;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int p = 0; p < kPlanSteps; ++p) {
    const size_t i = base + size_t(p) * 64 + lane;
    const uint64_t v = i < n ? m[i] : 0ull;
    if (__ballot(v != 0ull) == 0ull) continue;
    for (int d = 0; d < world; ++d) {
      const bool mine = (v >> d) & 1ull;
      const uint64_t b = __ballot(mine);
      if (!b) continue;
      const uint32_t o = uint32_t(__builtin_amdgcn_readlane(int(off), d));
      if (mine) idx[o + uint32_t(__popcll(b & below))] = int64_t(i);
      if (lane == d) off += uint32_t(__popcll(b));
    }
  }
}

// starts[d] = first position of rank d's list (d <= world: starts[world] = total)
__global__ void k_plan_bounds(const uint32_t* __restrict__ tc, uint32_t tiles, int world,
                              const uint32_t* __restrict__ total,
                              int64_t* __restrict__ starts) {
  const int d = threadIdx.x;
  if (d < world) starts[d] = tc[size_t(d) * tiles];
  if (d == world) starts[d] = *total;
}

// Row gather dst[j] = src[idx[j]] for rows of 4 / 8 / 16 / 32 / 48 bytes
// (the in-situ exchange packing); 16-B rows move as one 16-B load/store.
template <int WORDS>
__global__ __launch_bounds__(kBlock) void k_gather_rows(const uint32_t* __restrict__ src,
                                                        const int64_t* __restrict__ idx,
                                                        size_t n, uint32_t* __restrict__ dst) {
  const size_t j = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const size_t i = size_t(idx[j]);
  if (WORDS % 4 == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src + i * WORDS);
    uint4* d4 = reinterpret_cast<uint4*>(dst + j * WORDS);
#pragma unroll
    for (int k = 0; k < WORDS / 4; ++k) d4[k] = s4[k];
  } else {
#pragma unroll
    for (int k = 0; k < WORDS; ++k) dst[j * WORDS + k] = src[i * WORDS + k];
  }
}

// Ordered selection of the flagged positions (the masked any hit's index
// list): tiles of kSelTile flags, 16 per thread through one 16-B load;
// count -> scan of the tile counts -> ordered write.

__device__ __forceinline__ uint32_t flags16(const uint8_t* f, size_t M, size_t base,
                                            uint32_t& mask) {
  // bit k of mask = flags[base + k] != 0
  mask = 0;
  if (base + kSelPer <= M && (reinterpret_cast<uintptr_t>(f + base) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(f + base);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((w[q] >> (8 * b)) & 0xffu) mask |= 1u << (4 * q + b);
  } else {
    for (int k = 0; k < kSelPer; ++k)
      if (base + k < M && f[base + k]) mask |= 1u << k;
  }
  return __popc(mask);
}

__global__ __launch_bounds__(kBlock) void k_select_count(const uint8_t* __restrict__ f,
                                                         size_t M,
                                                         uint32_t* __restrict__ tile_counts) {
  using Reduce = hipcub::BlockReduce<uint32_t, kBlock>;
  __shared__ typename Reduce::TempStorage tmp;
  uint32_t mask;
  const size_t base = size_t(blockIdx.x) * kSelTile + size_t(threadIdx.x) * kSelPer;
  const uint32_t c = base < M ? flags16(f, M, base, mask) : 0u;
  const uint32_t total = Reduce(tmp).Sum(c);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(kBlock) void k_select_write(const uint8_t* __restrict__ f,
                                                         size_t M,
                                                         const uint32_t* __restrict__ tile_off,
                                                         uint32_t* __restrict__ out) {
  using Scan = hipcub::BlockScan<uint32_t, kBlock>;
  __shared__ typename Scan::TempStorage tmp;
  uint32_t mask = 0;
  const size_t base = size_t(blockIdx.x) * kSelTile + size_t(threadIdx.x) * kSelPer;
  const uint32_t c = base < M ? flags16(f, M, base, mask) : 0u;
  uint32_t k, total;
  Scan(tmp).ExclusiveSum(c, k, total);
  k += tile_off[blockIdx.x];
  while (mask) {
    const int b = __ffs(mask) - 1;
    mask &= mask - 1;
    out[k++] = uint32_t(base + b);
  }
}

// The PT shadow spawn (shadow_pt) compacted in ray order in one pass (a
// decoupled look-back scan): blocks take ordered tickets, publish their
// count (aggregate) at once, then sum their predecessors' published values
// back to the first inclusive prefix and publish their own inclusive prefix.  A block only
// waits on blocks with earlier tickets, which are already running and
// publish without waiting, so every wait ends; the values travel inside the
// 64-bit status words, so relaxed atomics order everything.  Same output
// order (ray order) as the two-pass form, one read of the rays and hits.
constexpr unsigned long long kLbAgg = 1ull << 62, kLbInc = 2ull << 62;
constexpr unsigned long long kLbVal = (1ull << 62) - 1;
// rays per thread: a block covers kBlock * kSpawnPer rays (OOC frame with
// 1 / 2 / 4 / 8: 3.06 / 2.89 / 2.84-2.85 / 2.89-2.91 ms, the two-pass form
// 2.86-2.87 ms: fewer blocks shorten the look-back chain, more rays per
// thread cost registers)
constexpr int kSpawnPer = 4;
__global__ __launch_bounds__(kBlock) void k_spawn_pt_onepass(
    const spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits, size_t M,
    ShadePt sh, unsigned long long* __restrict__ state, uint32_t nb,
    spray_rt_ray* __restrict__ out, int32_t* __restrict__ src, uint32_t* __restrict__ d_count) {
  __shared__ uint32_t s_b;
  __shared__ unsigned long long s_excl;
  if (threadIdx.x == 0) s_b = uint32_t(atomicAdd(state, 1ull));
  __syncthreads();
  const uint32_t b = s_b;
  // ray base + kBlock j + t: coalesced loads, ray order = (j, t) order
  const size_t base = size_t(b) * (kBlock * kSpawnPer) + threadIdx.x;
  float pos[kSpawnPer][3], wi[kSpawnPer][3];
  uint32_t fm = 0;
#pragma unroll
  for (int j = 0; j < kSpawnPer; ++j) {
    const size_t i = base + size_t(j) * kBlock;
    pos[j][0] = pos[j][1] = pos[j][2] = 0.f;
    wi[j][0] = wi[j][1] = wi[j][2] = 0.f;
    if (i < M && shadow_pt(rays[i], hits[i], sh, pos[j], wi[j])) fm |= 1u << j;
  }
  uint32_t k[kSpawnPer], run = 0;
#pragma unroll
  for (int j = 0; j < kSpawnPer; ++j) {
    uint32_t tot;
    k[j] = run + block_prefix((fm >> j) & 1u, tot);
    run += tot;
    __syncthreads();  // block_prefix's partial sums are reused by the next j
  }
  if (threadIdx.x < 64) {
    // the look-back by the first wave: lane l reads predecessor pend - l, so
    // one round trip covers 64 predecessors
    const int lane = int(threadIdx.x);
    unsigned long long* st = state + 1;
    unsigned long long excl = 0;
    if (b == 0) {
      if (lane == 0)
        __hip_atomic_store(st, kLbInc | run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(st + b, kLbAgg | run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t pend = int64_t(b) - 1;
      for (;;) {
        const int64_t p = pend - lane;
        // before the first block: an inclusive prefix of 0
        const unsigned long long v =
            p >= 0 ? __hip_atomic_load(st + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : kLbInc;
        const uint64_t inc = __ballot((v & kLbInc) != 0);
        const uint64_t ready = __ballot((v >> 62) != 0);
        const int first = inc ? __ffsll((long long)inc) - 1 : 63;
        const uint64_t need = first == 63 ? ~0ull : ((2ull << first) - 1);
        if ((ready & need) != need) continue;  // a predecessor has not published yet
        unsigned long long add = lane <= first ? (v & kLbVal) : 0ull;
        for (int o = 32; o > 0; o >>= 1) {
          const uint32_t lo = uint32_t(__shfl_xor(int(uint32_t(add)), o));
          const uint32_t hi = uint32_t(__shfl_xor(int(uint32_t(add >> 32)), o));
          add += (uint64_t(hi) << 32) | lo;
        }
        excl += add;
        if (inc) break;
        pend -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(st + b, kLbInc | (excl + run), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      if (b == nb - 1) *d_count = uint32_t(excl + run);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSpawnPer; ++j)
    if ((fm >> j) & 1u) {
      const size_t o = size_t(s_excl) + k[j];
      float4* op = reinterpret_cast<float4*>(out + o);
      op[0] = make_float4(pos[j][0], pos[j][1], pos[j][2], kRayEpsilon);
      op[1] = make_float4(wi[j][0], wi[j][1], wi[j][2], kInf);
      if (src) src[o] = int32_t(base + size_t(j) * kBlock);
    }
}

// ao_sample / ao_ok: shade_device.h

// One lane per (hit, sample) pair q = i * ns + l (32-bit: the API bounds
// M * ns), kAoPer pairs per thread in block-strided rounds: each round
// covers kBlock consecutive pairs, so the 32-B ray stores of a round are
// contiguous and the lanes of one hit share its record loads.  Output order
// is q ascending -- the reference's (hits in order, samples l = 0..ns-1):
// count pass (ao_ok), one scan of the tile totals, write pass.
constexpr int kAoPer = 16;
constexpr int kAoTile = kBlock * kAoPer;
// source rays per sample-major trace-order block (divides kBlock)
constexpr uint32_t kAoGroup = 8;
static_assert(kBlock % kAoGroup == 0, "trace-order blocks must not straddle tiles");

__global__ __launch_bounds__(kBlock) void k_spawn_ao_count(
    const spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    const int32_t* __restrict__ pixid, uint32_t npairs, uint32_t ns,
    uint32_t* __restrict__ tile_counts) {
  using Reduce = hipcub::BlockReduce<uint32_t, kBlock>;
  __shared__ typename Reduce::TempStorage tmp;
  const uint32_t base = blockIdx.x * uint32_t(kAoTile) + threadIdx.x;
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kAoPer; ++r) {  // independent rounds: the loads overlap
    const uint32_t q = base + uint32_t(r * kBlock);
    const uint32_t i = q < npairs ? q / ns : 0u;
    const spray_rt_hit h = hits[i];
    if (q < npairs && h.domain >= 0 && ao_ok(rays + i, h, pixid[i], int(q - i * ns), int(ns)))
      ++c;
  }
  const uint32_t total = Reduce(tmp).Sum(c);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

// Write pass: the ok flags of all rounds first (independent loads, one
// barrier for the whole tile's prefix), then the samples and stores, with
// no further synchronisation.
__global__ __launch_bounds__(kBlock) void k_spawn_ao_write(
    const spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    const int32_t* __restrict__ pixid, uint32_t npairs, uint32_t ns,
    const uint32_t* __restrict__ tile_off, spray_rt_ray* __restrict__ out,
    int32_t* __restrict__ src) {
  __shared__ uint32_t wcnt[kAoPer][kBlock / 64];
  __shared__ uint32_t spre[kAoPer][kBlock];  // each thread's output slot per round
  const uint32_t base = blockIdx.x * uint32_t(kAoTile) + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  uint32_t okm = 0;
#pragma unroll
  for (int r = 0; r < kAoPer; ++r) {
    const uint32_t q = base + uint32_t(r * kBlock);
    const uint32_t i = q < npairs ? q / ns : 0u;
    const spray_rt_hit h = hits[i];
    const bool ok =
        q < npairs && h.domain >= 0 && ao_ok(rays + i, h, pixid[i], int(q - i * ns), int(ns));
    const unsigned long long bal = __ballot(ok);
    spre[r][threadIdx.x] = __popcll(bal & below);
    if (lane == 0) wcnt[r][wave] = __popcll(bal);
    okm |= ok ? 1u << r : 0u;
  }
  __syncthreads();
  uint32_t run = tile_off[blockIdx.x];
#pragma unroll
  for (int r = 0; r < kAoPer; ++r) {
    uint32_t before = run;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      const uint32_t x = wcnt[r][w];
      before += w < wave ? x : 0u;
      run += x;
    }
    spre[r][threadIdx.x] += before;
  }
#pragma unroll 1
  for (int r = 0; r < kAoPer; ++r) {
    if (!((okm >> r) & 1u)) continue;
    const uint32_t q = base + uint32_t(r * kBlock);
    const uint32_t i = q / ns;
    const uint32_t k = spre[r][threadIdx.x];
    const AoOut a = ao_sample(rays[i], hits[i], pixid[i], int(q - i * ns), int(ns));
    float4* op = reinterpret_cast<float4*>(out + k);
    op[0] = make_float4(a.o[0], a.o[1], a.o[2], kRayEpsilon);
    op[1] = make_float4(a.w[0], a.w[1], a.w[2], kInf);
    if (src) src[k] = int32_t(i);
  }
}

// ns <= 32: the ok flags per hit first (one thread per hit: the hit record,
// the normalised N and the colour test once, then ns cheap sampler draws),
// as a sample mask plus the hit's exclusive prefix within its tile of kBlock
// hits; the write pass (one lane per pair, coalesced stores) then needs no
// prefix work: slot = tile offset + prefix + popcount of the mask below l.
// rec (optional): the origin, normal and tangent frame of every hit that
// spawns (ao_sample's prologue; 4 float4, the pixel in the first's w), read
// by the any-hit lanes that generate the AO rays (kEpiAoGen).
__global__ __launch_bounds__(kBlock) void k_spawn_ao_hitmask(
    const spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    const int32_t* __restrict__ pixid, uint32_t M, uint32_t ns, uint2* __restrict__ meta,
    uint32_t* __restrict__ tile_counts, float4* __restrict__ rec, uint32_t npix) {
  using Scan = hipcub::BlockScan<uint32_t, kBlock>;
  __shared__ typename Scan::TempStorage tmp;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  uint32_t mask = 0;
  if (i < M) {
    const spray_rt_hit h = hits[i];
    if (h.domain >= 0) {
      const int32_t px = pixid[i];
      // pairs form: the (pixel, sample) table holds npix pixels; a ray of a
      // pixel outside it spawns nothing (its table entries do not exist)
      if (!rec || uint32_t(px) < npix)
        for (uint32_t l = 0; l < ns; ++l)
          if (ao_ok(rays + i, h, px, int(l), int(ns))) mask |= 1u << l;
      if (rec && mask) {
        const spray_rt_ray r = rays[i];
        const float ht = h.t;
        float N[3] = {h.ns[0], h.ns[1], h.ns[2]};
        const float o[3] = {r.dir[0] * ht + r.org[0], r.dir[1] * ht + r.org[1],
                            r.dir[2] * ht + r.org[2]};
        const float wo[3] = {-r.dir[0], -r.dir[1], -r.dir[2]};
        if (!(gdot3(wo, N) > 0.0f)) {
          N[0] = -N[0];
          N[1] = -N[1];
          N[2] = -N[2];
        }
        gnorm3(N);
        float ax[3], ay[3];
        hemisphere_frame(N, ax, ay);
        float4* q = rec + 4 * size_t(i);
        q[0] = make_float4(o[0], o[1], o[2], __uint_as_float(uint32_t(px)));
        q[1] = make_float4(N[0], N[1], N[2], 0.f);
        q[2] = make_float4(ax[0], ax[1], ax[2], 0.f);
        q[3] = make_float4(ay[0], ay[1], ay[2], 0.f);
      }
    }
  }
  uint32_t pre, total;
  Scan(tmp).ExclusiveSum(uint32_t(__popc(mask)), pre, total);
  if (i < M) meta[i] = make_uint2(mask, pre);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

// The write pass, one thread per hit: its set samples in order, each at
// its compaction slot k (ascending from the hit's prefix) and its trace
// position (the masks of the hit's aligned group of kAoGroup neighbours,
// taken from the group's lanes: the group's rays of samples below l, then
// the group's earlier rays of sample l).  traced: the ray and its source
// go to the trace position, where the lanes of one sample write
// neighbouring slots; else to k, with order[pos] = k.
//
// The work of ao_sample, split by what it depends on: the hit's origin,
// normal and tangent frame once per hit; the local hemisphere sample
// (sampler seed pixid * (l + 1) -> concentric disk, the double sincos) once
// per (pixel, sample) -- the group's lanes compute samples l = me, me + 8,
// ... of the group leader's pixel and pass them round; a lane of another
// pixel draws its own -- and the rotation per (hit, sample).  The same
// operations on the same values as ao_sample, so the same bits.
__global__ __launch_bounds__(kBlock) void k_spawn_ao_write_hits(
    const spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    const int32_t* __restrict__ pixid, uint32_t M, uint32_t ns,
    const uint2* __restrict__ meta, const uint32_t* __restrict__ tile_off,
    spray_rt_ray* __restrict__ out, int32_t* __restrict__ src, uint32_t* __restrict__ order,
    int traced) {
  static_assert(kBlock % kAoGroup == 0 && 64 % kAoGroup == 0, "groups stay inside a wave");
  constexpr int kPer = 32 / int(kAoGroup);  // local samples per lane (ns <= 32)
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool in = i < M;
  const uint2 m = in ? meta[i] : make_uint2(0u, 0u);
  const int lane = threadIdx.x & 63, g0 = lane & ~int(kAoGroup - 1), me = lane - g0;
  uint32_t gm[kAoGroup];
#pragma unroll
  for (int t = 0; t < int(kAoGroup); ++t) gm[t] = __shfl(m.x, g0 + t);
  const uint32_t tile = in ? tile_off[blockIdx.x] : 0u;
  const uint32_t gpos = tile + __shfl(m.y, g0);
  const int32_t px = in ? pixid[i] : 0;
  const int32_t lead = __shfl(px, g0);
  if (__ballot(m.x != 0) == 0) return;  // the whole wave spawns nothing
  // the group leader's local samples l = me + kAoGroup * c (those some lane
  // of the group spawns)
  uint32_t gor = 0;
#pragma unroll
  for (int t = 0; t < int(kAoGroup); ++t) gor |= gm[t];
  float lvs[kPer][3];
#pragma unroll
  for (int c = 0; c < kPer; ++c) {
    const uint32_t l = uint32_t(me + int(kAoGroup) * c);
    lvs[c][0] = lvs[c][1] = lvs[c][2] = 0.f;
    if (l < ns && ((gor >> l) & 1u)) {
      uint32_t st = sampler_init1(lead * int32_t(l + 1));
      const float u1 = sampler_1d(st), u2 = sampler_1d(st);
      hemisphere_local(u1, u2, lvs[c]);
    }
  }
  // per hit (ao_sample's prologue)
  float o[3] = {0.f, 0.f, 0.f}, N[3] = {0.f, 0.f, 1.f}, ax[3] = {1.f, 0.f, 0.f},
        ay[3] = {0.f, 1.f, 0.f};
  if (m.x) {
    const spray_rt_ray r = rays[i];
    const spray_rt_hit h = hits[i];
    o[0] = r.dir[0] * h.t + r.org[0];
    o[1] = r.dir[1] * h.t + r.org[1];
    o[2] = r.dir[2] * h.t + r.org[2];
    const float wo[3] = {-r.dir[0], -r.dir[1], -r.dir[2]};
    N[0] = h.ns[0];
    N[1] = h.ns[1];
    N[2] = h.ns[2];
    if (!(gdot3(wo, N) > 0.0f)) {
      N[0] = -N[0];
      N[1] = -N[1];
      N[2] = -N[2];
    }
    gnorm3(N);
    hemisphere_frame(N, ax, ay);
  }
  uint32_t k = tile + m.y, run = 0;
#pragma unroll
  for (int c = 0; c < kPer; ++c) {
    for (int q = 0; q < int(kAoGroup); ++q) {
      const uint32_t l = uint32_t(int(kAoGroup) * c + q);
      if (l >= ns) break;  // uniform
      float lv[3] = {__shfl(lvs[c][0], g0 + q), __shfl(lvs[c][1], g0 + q),
                     __shfl(lvs[c][2], g0 + q)};
      uint32_t col = 0, before = 0;
#pragma unroll
      for (int t = 0; t < int(kAoGroup); ++t) {
        const uint32_t b = (gm[t] >> l) & 1u;
        col += b;
        before += t < me ? b : 0u;
      }
      if ((m.x >> l) & 1u) {
        if (px != lead) {  // another pixel than the group's leader
          uint32_t st = sampler_init1(px * int32_t(l + 1));
          const float u1 = sampler_1d(st), u2 = sampler_1d(st);
          hemisphere_local(u1, u2, lv);
        }
        float w[3], pdf;
        hemisphere_apply(lv, N, ax, ay, w, pdf);
        const uint32_t pos = gpos + run + before;
        const uint32_t dst = traced ? pos : k;
        if (order && !traced) order[pos] = k;
        ++k;
        if (SPRAY_NT_IO_LANE) {
          v4f* op = reinterpret_cast<v4f*>(out + dst);
          __builtin_nontemporal_store(v4f{o[0], o[1], o[2], kRayEpsilon}, op);
          __builtin_nontemporal_store(v4f{w[0], w[1], w[2], kInf}, op + 1);
        } else {
          float4* op = reinterpret_cast<float4*>(out + dst);
          op[0] = make_float4(o[0], o[1], o[2], kRayEpsilon);
          op[1] = make_float4(w[0], w[1], w[2], kInf);
        }
        if (src) src[dst] = int32_t(i);
      }
      run += col;
    }
  }
}

// 8x8 bit-matrix transpose: bit c of byte r <-> bit r of byte c
__device__ __forceinline__ uint64_t transpose8x8(uint64_t x) {
  uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  return x ^ t ^ (t << 28);
}

// The trace order of k_spawn_ao_write_hits (traced), as (source ray, sample)
// pairs only: pairs[pos] = i << 5 | l -- for the fused spawn + any hit,
// whose lanes generate the rays themselves (kEpiAoGen).
__global__ __launch_bounds__(kBlock) void k_spawn_ao_index(uint32_t M, uint32_t ns,
                                                           const uint2* __restrict__ meta,
                                                           const uint32_t* __restrict__ tile_off,
                                                           uint32_t* __restrict__ pairs,
                                                           const int32_t* __restrict__ pixid,
                                                           float4* __restrict__ lv) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool in = i < M;
  const uint2 m = in ? meta[i] : make_uint2(0u, 0u);
  const int lane = threadIdx.x & 63, g0 = lane & ~int(kAoGroup - 1), me = lane - g0;
  if (__ballot(m.x != 0) == 0) return;
  uint32_t gm[kAoGroup];
#pragma unroll
  for (int t = 0; t < int(kAoGroup); ++t) gm[t] = __shfl(m.x, g0 + t);
  // the local hemisphere samples of the group's pixels, lv[pixel * ns + l]:
  // the group's lanes share its leader pixel's (samples l = me, me + 8, ...,
  // the union of that pixel's masks in the group); the first lane of any
  // other pixel's run in the group draws the samples of its own and every
  // later lane of that pixel -- whether or not its own ray spawns (a run's
  // first sample may miss while the next hits: runs need not align with
  // the groups, e.g. a compacted subset of a frame's rays).  A pixel spread
  // over groups is written by each, with the same values.
  {
    const int32_t px = in ? pixid[i] : -1;
    int32_t gpx[kAoGroup];  // every lane takes part in the shuffles
#pragma unroll
    for (int t = 0; t < int(kAoGroup); ++t) gpx[t] = __shfl(px, g0 + t);
    const int32_t lead = gpx[0];
    uint32_t lor = 0, ror = 0;
    int32_t prev = -2;
#pragma unroll
    for (int t = 0; t < int(kAoGroup); ++t) {
      if (gpx[t] == lead) lor |= gm[t];
      if (t >= me && gpx[t] == px) ror |= gm[t];
      if (t == me - 1) prev = gpx[t];
    }
    for (uint32_t l = uint32_t(me); l < ns; l += kAoGroup)
      if ((lor >> l) & 1u) {
        uint32_t st = sampler_init1(lead * int32_t(l + 1));
        const float u1 = sampler_1d(st), u2 = sampler_1d(st);
        float v[3];
        hemisphere_local(u1, u2, v);
        lv[size_t(lead) * ns + l] = make_float4(v[0], v[1], v[2], 0.f);
      }
    if (in && px != lead && prev != px)
      for (uint32_t l = 0; l < ns; ++l)
        if ((ror >> l) & 1u) {
          uint32_t st = sampler_init1(px * int32_t(l + 1));
          const float u1 = sampler_1d(st), u2 = sampler_1d(st);
          float v[3];
          hemisphere_local(u1, u2, v);
          lv[size_t(px) * ns + l] = make_float4(v[0], v[1], v[2], 0.f);
        }
  }
  const uint32_t tile = in ? tile_off[blockIdx.x] : 0u;
  const uint32_t gpos = tile + __shfl(m.y, g0);
  // the group's masks as columns: byte l of cols[q] = the group members
  // with sample 8q + l (an 8x8 bit transpose per 8 samples), so each
  // sample's count and this lane's rank are two popcounts
  static_assert(kAoGroup == 8, "one byte per group member");
  uint64_t cols[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint64_t x = 0;
#pragma unroll
    for (int t = 0; t < int(kAoGroup); ++t) x |= uint64_t((gm[t] >> (8 * q)) & 0xFFu) << (8 * t);
    cols[q] = transpose8x8(x);
  }
  const uint32_t below = (1u << me) - 1u;
  uint32_t run = 0;
  for (uint32_t l = 0; l < ns; ++l) {
    const uint32_t b = uint32_t(cols[l >> 3] >> (8 * (l & 7))) & 0xFFu;
    if ((m.x >> l) & 1u) pairs[gpos + run + uint32_t(__popc(b & below))] = (i << 5) | l;
    run += uint32_t(__popc(b));
  }
}

// frame counters of a fused bounce: live slots (= radiance rays) and shadows
__global__ void k_frame_stats_add(unsigned long long* __restrict__ stats, int stripes, size_t M,
                                  const uint32_t* __restrict__ d_count) {
  if (threadIdx.x == 0) {
    stats[3 * stripes] += (unsigned long long)M;
    stats[1 * stripes] += (unsigned long long)*d_count;
  }
}

__global__ __launch_bounds__(kBlock) void k_iota(uint32_t* __restrict__ out, uint32_t n) {
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j < n) out[j] = j;
}

}  // namespace


// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_rtc_intersect(hipStream_t s, const SlotDesc* slots,
                                const int* seg_slot, const size_t* seg_off,
                                int nseg, char* rays, size_t stride, size_t M) {
  if (M == 0) return hipSuccess;
  k_rtc_intersect<<<grid_for(M), kBlock, 0, s>>>(slots, seg_slot, seg_off, nseg,
                                                 rays, stride, M);
  return hipGetLastError();
}

hipError_t launch_rtc_occluded(hipStream_t s, const SlotDesc* slots,
                               const int* seg_slot, const size_t* seg_off,
                               int nseg, char* rays, size_t stride, size_t M) {
  if (M == 0) return hipSuccess;
  k_rtc_occluded<<<grid_for(M), kBlock, 0, s>>>(slots, seg_slot, seg_off, nseg,
                                                rays, stride, M);
  return hipGetLastError();
}

hipError_t launch_rtc_update(hipStream_t s, const SlotDesc* slots, const int* seg_slot,
                             const size_t* seg_off, int nseg, char* rays, size_t stride,
                             size_t M) {
  if (M == 0) return hipSuccess;
  k_rtc_update<<<grid_for(M), kBlock, 0, s>>>(slots, seg_slot, seg_off, nseg, rays, stride, M);
  return hipGetLastError();
}

hipError_t launch_domains(hipStream_t s, const float* boxes, int ndom,
                          const float* org, const float* dir, size_t M,
                          int* ids, float* ts, int* counts, int maxhits) {
  if (M == 0) return hipSuccess;
  k_domains<<<grid_for(M), kBlock, 0, s>>>(boxes, ndom, org, dir, M, ids, ts,
                                           counts, maxhits);
  return hipGetLastError();
}

template <int W, bool ANY, bool COUNT, int EPI, int STK, int TRAV>
static hipError_t launch_scene_t(hipStream_t s, SceneArgs a) {
  bool kPersist = ANY ? (SPRAY_PERSIST_AH != 0 || a.M >= kPersistAhRays) : SPRAY_PERSIST_CH != 0;
  static int grid = 0;  // resident blocks (per process; gfx950 only)
  if (kPersist && !grid) {
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess)
      e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, k_scene<W, ANY, COUNT, EPI, STK, TRAV>, kBlock, 0);
    if (e != hipSuccess) return e;
    grid = cus * (per_cu > 0 ? per_cu : 1);
  }
  // No more packets than the persistent grid has waves (a rank's share of a
  // camera frame, a small batch): one packet per wave, no queue.  Every
  // wave of a persistent grid dequeues from the few non-empty queues at once
  // and then sweeps the drained ones -- ~45-55 us for a launch of one
  // packet, against one block's walk here.
  if (kPersist && !a.d_count && (a.M + 63) / 64 <= size_t(grid) * (kBlock / 64)) kPersist = false;
  a.persist = kPersist ? 1 : 0;
  // the queue heads and the spawn count zeroed in one launch
  ClearSeg cs[2];
  int ncs = 0;
  if (kPersist && !a.heads_ready) cs[ncs++] = {a.heads, kHeadsBytes, 0};
  if ((EPI == kEpiSpawn || EPI == kEpiShadow || EPI == kEpiShadowFrame) && a.sh_count &&
      !a.count_ready)
    cs[ncs++] = {a.sh_count, sizeof(uint32_t), 0};
  if (ncs) {
    const hipError_t e = launch_clear(s, cs, ncs);
    if (e != hipSuccess) return e;
  }
  const unsigned g = kPersist ? unsigned(grid) : grid_for(a.M);
  k_scene<W, ANY, COUNT, EPI, STK, TRAV><<<g, kBlock, 0, s>>>(a);
  return hipGetLastError();
}

// counting variants walk per lane; the fused closest-hit forms walk
// packets; plain closest hit and any hit follow the context's ray-coherence
// setting
template <int W, bool ANY, int EPI, int STK>
static hipError_t launch_scene_c(hipStream_t s, const SceneArgs& a, int coherence) {
  if (a.counters) return launch_scene_t<W, ANY, true, EPI, STK, 0>(s, a);
  // the fused spawn / keyed closest-hit forms serve camera rays: packets;
  // generated AO rays (hemispheres) walk per lane
  if constexpr (ANY && ao_epi(EPI)) {
    return launch_scene_t<W, ANY, false, EPI, STK, 0>(s, a);
  } else if constexpr (rep_epi(EPI)) {  // camera rays and point-light shadows
    return launch_scene_t<W, ANY, false, EPI, STK, 1>(s, a);
  } else if constexpr (!ANY && EPI != kEpiNone) {
    return launch_scene_t<W, ANY, false, EPI, STK, 1>(s, a);
  } else {
    switch (coherence) {
      case SPRAY_RT_RAYS_COHERENT:
        return launch_scene_t<W, ANY, false, EPI, STK, 1>(s, a);
      case SPRAY_RT_RAYS_INCOHERENT:
        return launch_scene_t<W, ANY, false, EPI, STK, 0>(s, a);
      default:
        return launch_scene_t<W, ANY, false, EPI, STK, 2>(s, a);
    }
  }
}

template <bool ANY, int EPI>
static hipError_t launch_scene_w(hipStream_t s, const SceneArgs& a, const SceneView& v) {
  if (v.max_depth > kStack) return hipErrorInvalidValue;
  if (a.ndom <= 64)
    return v.max_depth <= 16 ? launch_scene_c<1, ANY, EPI, 16>(s, a, v.coherence)
                             : launch_scene_c<1, ANY, EPI, kStack>(s, a, v.coherence);
  return v.max_depth <= 16 ? launch_scene_c<4, ANY, EPI, 16>(s, a, v.coherence)
                           : launch_scene_c<4, ANY, EPI, kStack>(s, a, v.coherence);
}

static SceneArgs scene_args(const SceneView& v, const spray_rt_ray* rays, size_t M) {
  SceneArgs a{};
  a.slots = v.slots;
  a.dom2slot = v.dom2slot;
  a.domtrav = v.domtrav;
  a.boxes = v.boxes;
  a.ndom = v.ndom;
  a.tlas = v.tlas;
  a.ntlas = v.ntlas;
  a.heads = v.heads;
  a.rays = rays;
  a.M = M;
  return a;
}

static ShadePt shade_from10(const float* s10) {
  ShadePt sh{};
  for (int k = 0; k < 3; ++k) {
    sh.lp[k] = s10[k];
    sh.lr[k] = s10[3 + k];
    sh.ks[k] = s10[6 + k];
  }
  sh.shininess = s10[9];
  return sh;
}

hipError_t launch_scene_intersect(hipStream_t s, const SceneView& v,
                                  const spray_rt_ray* rays, size_t M,
                                  spray_rt_hit* hits, unsigned long long* counters) {
  if (M == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.hits = hits;
  a.counters = counters;
  return launch_scene_w<false, kEpiNone>(s, a, v);
}

hipError_t launch_scene_occluded(hipStream_t s, const SceneView& v,
                                 const spray_rt_ray* rays, size_t M,
                                 const uint32_t* d_count, uint8_t* occluded,
                                 unsigned long long* counters) {
  if (M == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.d_count = d_count;
  a.occ = occluded;
  a.counters = counters;
  return launch_scene_w<true, kEpiNone>(s, a, v);
}

hipError_t launch_select_flagged(hipStream_t s, const uint8_t* flags, size_t M,
                                 uint32_t* idx_out, uint32_t* d_num, void* temp,
                                 size_t* temp_bytes) {
  const size_t tiles = (M + kSelTile - 1) / kSelTile;
  if (!temp) {
    *temp_bytes = (tiles + 1) * sizeof(uint32_t);
    return hipSuccess;
  }
  if (M == 0) return hipMemsetAsync(d_num, 0, sizeof(uint32_t), s);
  uint32_t* tc = static_cast<uint32_t*>(temp);
  k_select_count<<<unsigned(tiles), kBlock, 0, s>>>(flags, M, tc);
  k_scan_blocks<<<1, 1024, 0, s>>>(tc, uint32_t(tiles), d_num);
  k_select_write<<<unsigned(tiles), kBlock, 0, s>>>(flags, M, tc, idx_out);
  return hipGetLastError();
}

hipError_t launch_scene_occluded_masked(hipStream_t s, const SceneView& v,
                                       const spray_rt_ray* rays, size_t M,
                                       const uint8_t* valid, uint8_t* occluded) {
  if (M == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.valid = valid;
  a.occ = occluded;
  return launch_scene_w<true, kEpiNone>(s, a, v);
}

hipError_t launch_scene_occluded_indexed(hipStream_t s, const SceneView& v,
                                        const spray_rt_ray* rays, size_t max_n,
                                        const uint32_t* idx, const uint32_t* d_num,
                                        uint8_t* occluded,
                                        unsigned long long* counters) {
  if (max_n == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, max_n);
  a.idx = idx;
  a.d_count = d_num;
  a.occ = occluded;
  a.counters = counters;
  return launch_scene_w<true, kEpiNone>(s, a, v);
}

hipError_t launch_scene_intersect_indexed(hipStream_t s, const SceneView& v,
                                          const spray_rt_ray* rays, size_t max_n,
                                          const uint32_t* idx, const uint32_t* d_num,
                                          spray_rt_hit* hits) {
  if (max_n == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, max_n);
  a.idx = idx;
  a.d_count = d_num;
  a.hits = hits;
  return launch_scene_w<false, kEpiNone>(s, a, v);
}

hipError_t launch_scene_intersect_pt(hipStream_t s, const SceneView& v,
                                     const spray_rt_ray* rays, size_t M,
                                     spray_rt_hit* hits, const float* shade10,
                                     spray_rt_ray* out_rays, uint8_t* out_valid,
                                     uint32_t* d_count) {
  if (M == 0) return d_count ? hipMemsetAsync(d_count, 0, sizeof(uint32_t), s) : hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.hits = hits;
  for (int k = 0; k < 3; ++k) {
    a.shade.lp[k] = shade10[k];
    a.shade.lr[k] = shade10[3 + k];
    a.shade.ks[k] = shade10[6 + k];
  }
  a.shade.shininess = shade10[9];
  a.sh_out = out_rays;
  a.sh_valid = out_valid;
  a.sh_count = d_count;
  return launch_scene_w<false, kEpiSpawn>(s, a, v);
}

hipError_t launch_scene_intersect_shadow_pt(hipStream_t s, const SceneView& v,
                                            const spray_rt_ray* rays, size_t M,
                                            spray_rt_hit* hits, const float* shade10,
                                            uint8_t* occluded, uint8_t* sh_valid,
                                            uint32_t* d_count) {
  if (M == 0) return d_count ? hipMemsetAsync(d_count, 0, sizeof(uint32_t), s) : hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.hits = hits;
  for (int k = 0; k < 3; ++k) {
    a.shade.lp[k] = shade10[k];
    a.shade.lr[k] = shade10[3 + k];
    a.shade.ks[k] = shade10[6 + k];
  }
  a.shade.shininess = shade10[9];
  a.occ = occluded;
  a.sh_valid = sh_valid;
  a.sh_count = d_count;
  return launch_scene_w<false, kEpiShadow>(s, a, v);
}

hipError_t launch_scene_frame_pt(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                 size_t M, spray_rt_hit* hits, const float* shade10,
                                 uint8_t* occluded, uint8_t* sh_valid, float* sw,
                                 uint32_t* d_count, uint32_t* heads) {
  if (M == 0)
    return d_count && !heads ? hipMemsetAsync(d_count, 0, sizeof(uint32_t), s) : hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  if (heads) {  // the caller zeroed them and the count in one launch
    a.heads = heads;
    a.heads_ready = 1;
    a.count_ready = 1;
  }
  a.hits = hits;
  for (int k = 0; k < 3; ++k) {
    a.shade.lp[k] = shade10[k];
    a.shade.lr[k] = shade10[3 + k];
    a.shade.ks[k] = shade10[6 + k];
  }
  a.shade.shininess = shade10[9];
  a.occ = occluded;
  a.sh_valid = sh_valid;
  a.sw = reinterpret_cast<float4*>(sw);
  a.sh_count = d_count;
  return launch_scene_w<false, kEpiShadowFrame>(s, a, v);
}

hipError_t launch_frame_stats_add(hipStream_t s, unsigned long long* stats, int stripes,
                                  size_t M, const uint32_t* d_count) {
  k_frame_stats_add<<<1, 64, 0, s>>>(stats, stripes, M, d_count);
  return hipGetLastError();
}

hipError_t launch_scene_intersect_keyed(hipStream_t s, const SceneView& v,
                                        const spray_rt_ray* rays, size_t M,
                                        spray_rt_hit* hits, uint64_t* keys) {
  if (M == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, M);
  a.hits = hits;
  a.keys = keys;
  return launch_scene_w<false, kEpiKeys>(s, a, v);
}

hipError_t launch_scene_intersect_keyed_indexed(hipStream_t s, const SceneView& v,
                                                const spray_rt_ray* rays, size_t max_n,
                                                const uint32_t* idx, const uint32_t* d_num,
                                                spray_rt_hit* hits, uint64_t* keys) {
  if (max_n == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, max_n);
  a.idx = idx;
  a.d_count = d_num;
  a.hits = hits;
  a.keys = keys;
  return launch_scene_w<false, kEpiKeys>(s, a, v);
}

hipError_t launch_route(hipStream_t s, const SceneView& v, const int* owner,
                        const spray_rt_ray* rays, size_t M, uint64_t* out, const uint32_t* sel,
                        const uint8_t* valid, unsigned long long* nvalid) {
  if (M == 0) return hipSuccess;
  if (v.ndom <= 64)
    k_route<1><<<grid_for(M), kBlock, 0, s>>>(v.tlas, v.ntlas, owner, v.ndom, rays, sel, M, out,
                                              valid, nvalid);
  else
    k_route<4><<<grid_for(M), kBlock, 0, s>>>(v.tlas, v.ntlas, owner, v.ndom, rays, sel, M, out,
                                              valid, nvalid);
  return hipGetLastError();
}

hipError_t launch_eye_rays_insitu(hipStream_t s, const float* cam14, int image_w,
                                  int spp, int bx, int by, int bw, int tx, int ty,
                                  int tw, int th, spray_rt_ray* rays, int32_t* pixid,
                                  int32_t* samid) {
  const size_t n = size_t(tw) * th * spp;
  if (n == 0) return hipSuccess;
  Cam c;
  for (int k = 0; k < 14; ++k) c.p[k] = cam14[k];
  k_eye_rays_insitu<<<grid_for(n), kBlock, 0, s>>>(c, image_w, spp, bx, by, bw, tx, ty,
                                                   tw, th, rays, pixid, samid);
  return hipGetLastError();
}

size_t plan_temp_bytes(size_t n, int world) {
  const size_t tiles = (n + kPlanWave - 1) / kPlanWave;
  return (tiles * size_t(world) + 2) * sizeof(uint32_t);
}

hipError_t launch_plan(hipStream_t s, const uint64_t* masks, size_t n, int world,
                       int64_t* idx, int64_t* starts, void* temp) {
  const size_t tiles = (n + kPlanWave - 1) / kPlanWave;  // wave tiles
  uint32_t* tc = static_cast<uint32_t*>(temp);
  uint32_t* total = tc + tiles * size_t(world) + 1;
  if (n == 0 || world <= 0) {
    hipError_t e = hipMemsetAsync(starts, 0, (world + 1) * sizeof(int64_t), s);
    return e;
  }
  if (world > 64) return hipErrorInvalidValue;
  const unsigned g = unsigned((tiles + kBlock / 64 - 1) / (kBlock / 64));
  k_plan_count<<<g, kBlock, 0, s>>>(masks, n, world, tiles, tc);
  k_scan_blocks<<<1, 1024, 0, s>>>(tc, uint32_t(tiles * world), total);
  if (idx) k_plan_write<<<g, kBlock, 0, s>>>(masks, n, world, tiles, tc, idx);
  k_plan_bounds<<<1, 128, 0, s>>>(tc, uint32_t(tiles), world, total, starts);
  return hipGetLastError();
}

hipError_t launch_gather_rows(hipStream_t s, const void* src, size_t row_bytes,
                              const int64_t* idx, size_t n, void* dst) {
  if (n == 0) return hipSuccess;
  const uint32_t* a = static_cast<const uint32_t*>(src);
  uint32_t* b = static_cast<uint32_t*>(dst);
  switch (row_bytes) {
    case 4: k_gather_rows<1><<<grid_for(n), kBlock, 0, s>>>(a, idx, n, b); break;
    case 8: k_gather_rows<2><<<grid_for(n), kBlock, 0, s>>>(a, idx, n, b); break;
    case 16: k_gather_rows<4><<<grid_for(n), kBlock, 0, s>>>(a, idx, n, b); break;
    case 32: k_gather_rows<8><<<grid_for(n), kBlock, 0, s>>>(a, idx, n, b); break;
    case 48: k_gather_rows<12><<<grid_for(n), kBlock, 0, s>>>(a, idx, n, b); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_eye_rays_ooc(hipStream_t s, const float* cam14, int image_w,
                               int spp, int tx, int ty, int tw, int th,
                               spray_rt_ray* rays, int32_t* pixid,
                               int32_t* samid) {
  const size_t n = size_t(tw) * th * spp;
  if (n == 0) return hipSuccess;
  Cam c;
  for (int k = 0; k < 14; ++k) c.p[k] = cam14[k];
  k_eye_rays_ooc<<<grid_for(n), kBlock, 0, s>>>(c, image_w, spp, tx, ty, tw, th,
                                                rays, pixid, samid);
  return hipGetLastError();
}

hipError_t launch_eye_rays_ooc_tiles(hipStream_t s, const float* cam14, int image_w, int spp,
                                    const int* tiles, int ntiles, spray_rt_ray* rays,
                                    int32_t* pixid, int32_t* samid) {
  Cam c;
  for (int k = 0; k < 14; ++k) c.p[k] = cam14[k];
  size_t base = 0;
  for (int k0 = 0; k0 < ntiles; k0 += kEyeTiles) {
    EyeTiles T{};
    T.n = ntiles - k0 < kEyeTiles ? ntiles - k0 : kEyeTiles;
    uint32_t off = 0;
    for (int k = 0; k < T.n; ++k) {
      for (int q = 0; q < 4; ++q) T.t[k][q] = tiles[4 * (k0 + k) + q];
      T.off[k] = off;
      off += uint32_t(size_t(T.t[k][2]) * T.t[k][3] * spp);
    }
    T.off[T.n] = off;
    if (off) {
      k_eye_rays_ooc_tiles<<<(off + kBlock - 1) / kBlock, kBlock, 0, s>>>(
          c, image_w, spp, T, rays + base, pixid ? pixid + base : nullptr,
          samid ? samid + base : nullptr);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    base += off;
  }
  return hipSuccess;
}

hipError_t launch_eye_rays_ooc_table(hipStream_t s, const float* cam14, int image_w, int spp,
                                    const CamTable& T, spray_rt_ray* rays, int32_t* pixid,
                                    int32_t* samid) {
  const size_t n = size_t(T.npix) * size_t(spp);
  if (n == 0) return hipSuccess;
  Cam c;
  for (int k = 0; k < 14; ++k) c.p[k] = cam14[k];
  k_eye_rays_ooc_table<<<grid_for(n), kBlock, 0, s>>>(c, image_w, spp, T, rays, pixid, samid);
  return hipGetLastError();
}

hipError_t launch_spawn_pt(hipStream_t s, const spray_rt_ray* rays,
                           const spray_rt_hit* hits, size_t M,
                           const float* shade10, spray_rt_ray* out_rays,
                           int32_t* out_src, uint32_t* d_count,
                           void* scratch) {
  ShadePt sh;
  for (int k = 0; k < 3; ++k) {
    sh.lp[k] = shade10[k];
    sh.lr[k] = shade10[3 + k];
    sh.ks[k] = shade10[6 + k];
  }
  sh.shininess = shade10[9];
  if (M == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
  const unsigned g = unsigned((M + size_t(kBlock) * kSpawnPer - 1) / (size_t(kBlock) * kSpawnPer));
  unsigned long long* state = static_cast<unsigned long long*>(scratch);
  hipError_t e = hipMemsetAsync(state, 0, (size_t(g) + 1) * sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  k_spawn_pt_onepass<<<g, kBlock, 0, s>>>(rays, hits, M, sh, state, g, out_rays, out_src,
                                          d_count);
  return hipGetLastError();
}

hipError_t launch_spawn_ao(hipStream_t s, const spray_rt_ray* rays, const spray_rt_hit* hits,
                           const int32_t* pixid, size_t M, int nsamples,
                           spray_rt_ray* out_rays, int32_t* out_src, uint32_t* d_count,
                           void* scratch, uint32_t* order, bool traced) {
  if (M == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
  const uint32_t npairs = uint32_t(M * size_t(nsamples));
  if (nsamples <= 32) {
    const uint32_t g = uint32_t((M + kBlock - 1) / kBlock);
    uint2* meta = static_cast<uint2*>(scratch);
    uint32_t* tiles = reinterpret_cast<uint32_t*>(meta + M);
    k_spawn_ao_hitmask<<<g, kBlock, 0, s>>>(rays, hits, pixid, uint32_t(M),
                                            uint32_t(nsamples), meta, tiles, nullptr,
                                            0xFFFFFFFFu);
    k_scan_blocks<<<1, 1024, 0, s>>>(tiles, g, d_count);
    k_spawn_ao_write_hits<<<g, kBlock, 0, s>>>(rays, hits, pixid, uint32_t(M),
                                               uint32_t(nsamples), meta, tiles, out_rays,
                                               out_src, order, traced ? 1 : 0);
    return hipGetLastError();
  }
  const uint32_t g = (npairs + kAoTile - 1) / kAoTile;
  uint32_t* tiles = static_cast<uint32_t*>(scratch);
  k_spawn_ao_count<<<g, kBlock, 0, s>>>(rays, hits, pixid, npairs, uint32_t(nsamples), tiles);
  k_scan_blocks<<<1, 1024, 0, s>>>(tiles, g, d_count);
  k_spawn_ao_write<<<g, kBlock, 0, s>>>(rays, hits, pixid, npairs, uint32_t(nsamples), tiles,
                                        out_rays, out_src);
  // more samples than a mask holds: the trace order is the output order
  if (order) k_iota<<<(npairs + kBlock - 1) / kBlock, kBlock, 0, s>>>(order, npairs);
  return hipGetLastError();
}

hipError_t launch_spawn_ao_pairs(hipStream_t s, const spray_rt_ray* rays,
                                 const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                 int nsamples, size_t npix, uint32_t* out_pairs, float* lv,
                                 float* rec, uint32_t* d_count, void* scratch) {
  if (M == 0) return hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
  if (nsamples > 32) return hipErrorInvalidValue;
  const uint32_t g = uint32_t((M + kBlock - 1) / kBlock);
  uint2* meta = static_cast<uint2*>(scratch);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(meta + M);
  k_spawn_ao_hitmask<<<g, kBlock, 0, s>>>(rays, hits, pixid, uint32_t(M), uint32_t(nsamples),
                                          meta, tiles, reinterpret_cast<float4*>(rec),
                                          uint32_t(npix < 0xFFFFFFFFull ? npix : 0xFFFFFFFFull));
  k_scan_blocks<<<1, 1024, 0, s>>>(tiles, g, d_count);
  k_spawn_ao_index<<<g, kBlock, 0, s>>>(uint32_t(M), uint32_t(nsamples), meta, tiles,
                                        out_pairs, pixid, reinterpret_cast<float4*>(lv));
  return hipGetLastError();
}

hipError_t launch_scene_rep_keyed(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                  size_t n, const uint32_t* idx, size_t nc,
                                  const float* shade10, spray_rt_hit* hits, uint64_t* keys,
                                  uint32_t* tkeys, float* sw, uint8_t* sv) {
  if (nc == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, nc);
  a.nrays = n;
  a.idx = idx;
  a.hits = hits;
  a.keys = keys;
  a.tkeys = tkeys;
  a.sw = reinterpret_cast<float4*>(sw);
  a.sh_valid = sv;
  a.shade = shade_from10(shade10);
  return launch_scene_w<false, kEpiKeysShade>(s, a, v);
}

hipError_t launch_scene_rep_shadows(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                    size_t n, const uint32_t* idx, size_t nc,
                                    const uint32_t* tmin, const float* shade10, uint8_t* occ) {
  if (nc == 0) return hipSuccess;
  SceneArgs a = scene_args(v, rays, nc);
  a.nrays = n;
  a.idx = idx;
  a.tmin = tmin;
  a.occ = occ;
  a.shade = shade_from10(shade10);
  return launch_scene_w<true, kEpiShadowGen>(s, a, v);
}

hipError_t launch_iota_u32(hipStream_t s, uint32_t* out, size_t n) {
  if (n == 0) return hipSuccess;
  k_iota<<<grid_for(n), kBlock, 0, s>>>(out, uint32_t(n));
  return hipGetLastError();
}

static SceneArgs cam_args(const SceneView& v, const CamFrame& F, const CamTable& T) {
  SceneArgs a = scene_args(v, nullptr, size_t(T.npix) * size_t(F.spp));
  a.cam_tab = T;
  for (int k = 0; k < 14; ++k) a.cam.p[k] = F.cam[k];
  a.cam_w = F.image_w;
  a.cam_spp = F.spp;
  return a;
}

hipError_t launch_scene_cam_keyed(hipStream_t s, const SceneView& v, const CamFrame& F,
                                  const CamTable& T, const float* shade10, spray_rt_hit* hits,
                                  uint64_t* keys, uint32_t* tkeys, float* sw, uint8_t* sv,
                                  bool defer_lp, uint32_t* heads) {
  if (T.npix == 0) return hipSuccess;
  SceneArgs a = cam_args(v, F, T);
  if (heads) {
    a.heads = heads;
    a.heads_ready = 1;
  }
  a.direct_res = defer_lp ? 1 : 0;
  a.hits = hits;
  a.keys = keys;
  a.tkeys = tkeys;
  a.sw = reinterpret_cast<float4*>(sw);
  a.sh_valid = sv;
  a.shade = shade_from10(shade10);
  return launch_scene_w<false, kEpiKeysShade>(s, a, v);
}

hipError_t launch_scene_cam_shadows(hipStream_t s, const SceneView& v, const CamFrame& F,
                                    const CamTable& T, const uint32_t* tmin,
                                    const float* shade10, uint8_t* occ, bool direct) {
  if (T.npix == 0) return hipSuccess;
  SceneArgs a = cam_args(v, F, T);
  a.direct_res = direct ? 1 : 0;
  a.tmin = tmin;
  a.occ = occ;
  a.shade = shade_from10(shade10);
  return launch_scene_w<true, kEpiShadowGen>(s, a, v);
}

struct ClearList {
  ClearSeg seg[kClearSegs];
  int n;
};
// each segment: 16-B stores over its 16-B aligned body (the buffers are
// allocation-aligned), bytes for the rest
__global__ __launch_bounds__(kBlock) void k_clear(const ClearList L) {
  const size_t tid = size_t(blockIdx.x) * kBlock + threadIdx.x;
  const size_t nth = size_t(gridDim.x) * kBlock;
  for (int q = 0; q < L.n; ++q) {
    uint8_t* p = static_cast<uint8_t*>(L.seg[q].p);
    const size_t bytes = L.seg[q].bytes;
    const uint32_t b = uint32_t(L.seg[q].value) & 0xFFu;
    const uint32_t w = b * 0x01010101u;
    const uint4 v = make_uint4(w, w, w, w);
    const size_t nv = bytes / 16;
    for (size_t i = tid; i < nv; i += nth) reinterpret_cast<uint4*>(p)[i] = v;
    for (size_t i = 16 * nv + tid; i < bytes; i += nth) p[i] = uint8_t(b);
  }
}

hipError_t launch_clear(hipStream_t s, const ClearSeg* segs, int n) {
  if (n < 0 || n > kClearSegs) return hipErrorInvalidValue;
  ClearList L{};
  size_t total = 0;
  for (int q = 0; q < n; ++q) {
    if (segs[q].bytes && (!segs[q].p || (segs[q].bytes >= 16 &&
                                         (reinterpret_cast<uintptr_t>(segs[q].p) & 15u))))
      return hipErrorInvalidValue;
    L.seg[L.n++] = segs[q];
    total += segs[q].bytes;
  }
  if (total == 0) return hipSuccess;
  const unsigned g = unsigned(std::min<size_t>((total / 16 + kBlock) / kBlock, 4096));
  k_clear<<<g, kBlock, 0, s>>>(L);
  return hipGetLastError();
}

hipError_t launch_occluded_ao_pairs(hipStream_t s, const SceneView& v, size_t max_n,
                                    const uint32_t* pairs, const float* rec, const float* lv,
                                    int nsamples, const uint32_t* d_count, uint8_t* occ,
                                    unsigned long long* counters, const uint32_t* idx,
                                    uint32_t* fields, int fb) {
  if (max_n == 0) return hipSuccess;
  if (fields && fb != 2 && fb != 4 && fb != 8) return hipErrorInvalidValue;
  SceneArgs a = scene_args(v, nullptr, max_n);
  a.d_count = d_count;
  a.idx = idx;
  a.occ = occ;
  a.counters = counters;
  a.ao_pairs = pairs;
  a.ao_rec = reinterpret_cast<const float4*>(rec);
  a.ao_lv = reinterpret_cast<const float4*>(lv);
  a.ao_ns = nsamples;
  a.ao_fields = fields;
  a.ao_fb = fb;
  return fields ? launch_scene_w<true, kEpiAoGenF>(s, a, v) : launch_scene_w<true, kEpiAoGen>(s, a, v);
}

// Replicated AO frames: flag[k] = AO pair k (k < min(*d_count, M)) enters
// a resident domain's box (ao_own).  The flagged pairs are compacted and
// traced alone: culling lanes inside the traced waves instead (measured)
// left every wave as long as its slowest lane, and a rank's launch as long
// as the whole frame's.
// mode 1 / 2 split the pairs between two rounds (trace_replicated_ao): 1 =
// the pairs that start in a resident domain (the winner's domain, the low
// bits of the source's key minimum kmin), 2 = the other pairs entering a
// resident box whose bit in bits_a (the first round's occlusion over the
// group) is clear; 0 = every pair entering a resident box.
template <int W>
__global__ __launch_bounds__(kBlock) void k_ao_own_flags(const SceneArgs A, uint8_t* flag,
                                                        const uint64_t* __restrict__ kmin,
                                                        const uint32_t* __restrict__ bits_a,
                                                        int mode) {
  __shared__ float sbox[6 * 64 * W];
  __shared__ uint32_t resm[2 * W];  // resident domains as a bit mask
  // padded as build_domain_tree pads internal boxes (kTopPad x the larger
  // of the box's own scale and the scene's largest finite coordinate, where
  // the AO rays start)
  __shared__ float spad[6 * 64 * W];
  __shared__ uint8_t sres[64 * W];
  __shared__ float sun[6];  // union of the resident padded boxes
  __shared__ int nres;
  __shared__ float gmax;
  __shared__ float wg[kBlock / 64];
  for (int k = threadIdx.x; k < 6 * A.ndom; k += kBlock) sbox[k] = A.boxes[k];
  {
    float g = 0.f;
    for (int k = threadIdx.x; k < 6 * A.ndom; k += kBlock)
      if (isfinite(A.boxes[k])) g = fmaxf(g, fabsf(A.boxes[k]));
    for (int o = 32; o > 0; o >>= 1) g = fmaxf(g, __shfl_xor(g, o));
    if ((threadIdx.x & 63) == 0) wg[threadIdx.x >> 6] = g;
    // the resident domains, one thread per domain (their bits in domain order)
    if (threadIdx.x < 2 * W) resm[threadIdx.x] = 0u;
    __syncthreads();
    for (int d = threadIdx.x; d < A.ndom; d += kBlock) {
      const float4 t = ld4(A.domtrav, d);
      if (__float_as_uint(t.x) | __float_as_uint(t.y)) atomicOr(&resm[d >> 5], 1u << (d & 31));
    }
    if (threadIdx.x == 0) {
      float m = 0.f;
      for (int w = 0; w < kBlock / 64; ++w) m = fmaxf(m, wg[w]);
      gmax = m;
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < 3 * A.ndom; k += kBlock) {
    const int d = k / 3, j = k - 3 * d;
    const float lo = A.boxes[6 * d + j], hi = A.boxes[6 * d + 3 + j];
    const float m = fmaxf(fmaxf(fmaxf(fabsf(lo), fabsf(hi)), hi - lo), gmax);
    const float p = m * kTopPad;
    const bool fin = isfinite(A.boxes[6 * d]) && isfinite(A.boxes[6 * d + 3]);
    spad[6 * d + j] = fin ? lo - p : lo;
    spad[6 * d + 3 + j] = fin ? hi + p : hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // the resident list in domain order, their union
    int q = 0;
    float u[6] = {kInf, kInf, kInf, -kInf, -kInf, -kInf};
    for (int w = 0; w < 2 * W; ++w) {
      uint32_t b = resm[w];
      while (b) {
        const int d = 32 * w + __ffs(b) - 1;
        b &= b - 1;
        sres[q++] = uint8_t(d);
        for (int j = 0; j < 3; ++j) {
          u[j] = fminf(u[j], spad[6 * d + j]);
          u[3 + j] = fmaxf(u[3 + j], spad[6 * d + 3 + j]);
        }
      }
    }
    for (int j = 0; j < 6; ++j) sun[j] = u[j];
    nres = q;
  }
  __syncthreads();
  const size_t n = A.d_count ? min(size_t(*A.d_count), A.M) : A.M;
  // the grid-stride loop is a chain of dependent loads per pair (pair ->
  // key minimum / record -> sample): the next pair is loaded one iteration
  // ahead, and a mode-2 pair's record and sample are loaded beside its key
  // minimum, before the flag says whether its ray is needed (16 pairs share
  // a record, 8 sources of a pixel its samples: mostly cache hits)
  const size_t stride = size_t(gridDim.x) * kBlock;
  size_t k = size_t(blockIdx.x) * kBlock + threadIdx.x;
  uint32_t pr_next = k < n ? A.ao_pairs[k] : 0u;
  for (; k < A.M; k += stride) {
    const uint32_t pr = pr_next;
    pr_next = k + stride < n ? A.ao_pairs[k + stride] : 0u;
    bool f = false;
    if (k < n) {
      if (mode == 0) {
        f = ao_own(ao_load(A, pr), sbox, spad, sun, sres, nres);
      } else {
        const uint64_t km = kmin[pr >> 5];
        const uint32_t bw = mode == 2 ? bits_a[k >> 5] : 0u;
        AoSrc o{};
        if (mode == 2) o = ao_load(A, pr);
        const uint32_t d = uint32_t(km & 0xFFFFu);
        const bool home = d < uint32_t(A.ndom) && ((resm[d >> 5] >> (d & 31)) & 1u);
        if (mode == 1)
          f = home;
        else
          f = !home && !((bw >> (k & 31)) & 1u) && ao_own(o, sbox, spad, sun, sres, nres);
      }
    }
    flag[k] = f ? 1 : 0;
  }
}

hipError_t launch_ao_own_flags(hipStream_t s, const SceneView& v, size_t max_n,
                               const uint32_t* pairs, const float* rec, const float* lv,
                               int nsamples, const uint32_t* d_count, uint8_t* flag,
                               const uint64_t* kmin, const uint32_t* bits_a, int mode) {
  if (mode != 0 && !kmin) return hipErrorInvalidValue;
  if (mode == 2 && !bits_a) return hipErrorInvalidValue;
  if (max_n == 0) return hipSuccess;
  SceneArgs a = scene_args(v, nullptr, max_n);
  a.d_count = d_count;
  a.ao_pairs = pairs;
  a.ao_rec = reinterpret_cast<const float4*>(rec);
  a.ao_lv = reinterpret_cast<const float4*>(lv);
  a.ao_ns = nsamples;
  // a few resident blocks per CU walk the pairs grid-stride: each block's
  // setup (boxes, padding, resident list) is paid once per ~10 K pairs
  const unsigned g = unsigned(std::min<size_t>((max_n + kBlock - 1) / kBlock, 2048));
  if (a.ndom <= 64)
    k_ao_own_flags<1><<<g, kBlock, 0, s>>>(a, flag, kmin, bits_a, mode);
  else
    k_ao_own_flags<4><<<g, kBlock, 0, s>>>(a, flag, kmin, bits_a, mode);
  return hipGetLastError();
}

size_t ao_scratch_bytes(size_t M, int nsamples) {
  if (nsamples <= 32) return M * sizeof(uint2) + ((M + kBlock - 1) / kBlock + 1) * sizeof(uint32_t);
  const size_t g = (M * size_t(nsamples) + kAoTile - 1) / kAoTile;
  return (g + 1) * sizeof(uint32_t);
}

}  // namespace spray_rt
