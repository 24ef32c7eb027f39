// rt_kernels.h -- host-side launchers of the gfx950 kernels (rt_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt_common.h"
#include "spray_rt.h"

namespace spray_rt {

constexpr int kBlock = 256;  // 4 waves of 64

// Per-slot streams over Embree record layouts (RTCRayIntersection / RTCRay)
// with a byte stride.  seg_off has nseg+1 entries, seg_slot nseg (device).
hipError_t launch_rtc_intersect(hipStream_t s, const SlotDesc* slots,
                                const int* seg_slot, const size_t* seg_off,
                                int nseg, char* rays, size_t stride, size_t M);
hipError_t launch_rtc_occluded(hipStream_t s, const SlotDesc* slots,
                               const int* seg_slot, const size_t* seg_off,
                               int nseg, char* rays, size_t stride, size_t M);
// TriMeshBuffer::updateIntersection alone: color and Ns of the hit records
hipError_t launch_rtc_update(hipStream_t s, const SlotDesc* slots, const int* seg_slot,
                             const size_t* seg_off, int nseg, char* rays, size_t stride,
                             size_t M);

hipError_t launch_domains(hipStream_t s, const float* boxes, int ndom,
                          const float* org, const float* dir, size_t M,
                          int* ids, float* ts, int* counts, int maxhits);

// Fused scene path: domain list + per-domain traversal + epilogue.
// The resident scene as the kernels see it (all device pointers).
struct SceneView {
  const SlotDesc* slots;
  const int* dom2slot;
  const DomTrav* domtrav;  // [ndom]
  const float* boxes;      // [ndom][6]
  int ndom;
  const BvhNode* tlas;  // top-level tree over the domain boxes
  int ntlas;
  uint32_t* heads;  // kQueues*32 uint32 work-queue heads, zeroed by every launch
  int max_depth;    // max tree depth over resident slots and the top-level tree
  int coherence;    // SPRAY_RT_RAYS_* of the any-hit launches
};

// counters (optional, device uint64[3]: nodes, tris, visits) select the
// counting variant used to verify the canonical traversal.
hipError_t launch_scene_intersect(hipStream_t s, const SceneView& v,
                                  const spray_rt_ray* rays, size_t M,
                                  spray_rt_hit* hits, unsigned long long* counters);
// d_count (optional, device): the launch covers min(*d_count, M) rays.
hipError_t launch_scene_occluded(hipStream_t s, const SceneView& v,
                                 const spray_rt_ray* rays, size_t M,
                                 const uint32_t* d_count, uint8_t* occluded,
                                 unsigned long long* counters);

// idx_out[0..*d_num) = ascending i with flags[i] != 0 (tile count, scan,
// ordered write; temp == nullptr: *temp_bytes <- required scratch size).
hipError_t launch_select_flagged(hipStream_t s, const uint8_t* flags, size_t M,
                                 uint32_t* idx_out, uint32_t* d_num, void* temp,
                                 size_t* temp_bytes);
// Any hit over the rays i < M with valid[i] != 0, in place (no compaction:
// a packet wave walks the union of its valid lanes' paths).
hipError_t launch_scene_occluded_masked(hipStream_t s, const SceneView& v,
                                       const spray_rt_ray* rays, size_t M,
                                       const uint8_t* valid, uint8_t* occluded);
// Any hit over rays idx[0..*d_num) (d_num <= max_n), occluded[idx[j]] written.
hipError_t launch_scene_occluded_indexed(hipStream_t s, const SceneView& v,
                                        const spray_rt_ray* rays, size_t max_n,
                                        const uint32_t* idx, const uint32_t* d_num,
                                        uint8_t* occluded,
                                        unsigned long long* counters);
// Closest hit with the PT shadow-ray spawn fused into the epilogue,
// positional: out_rays[i] / out_valid[i] for source ray i; *d_count (may be
// null) = number spawned, zeroed by the launcher.
hipError_t launch_scene_intersect_pt(hipStream_t s, const SceneView& v,
                                     const spray_rt_ray* rays, size_t M,
                                     spray_rt_hit* hits, const float* shade10,
                                     spray_rt_ray* out_rays, uint8_t* out_valid,
                                     uint32_t* d_count);

// Closest hit, the fused PT shadow spawn and the shadow rays' any hit in one
// launch: sh_valid[i] = source i spawned a shadow ray, occluded[i] (written
// where sh_valid[i]) = it is blocked; *d_count (may be null) = shadow rays.
hipError_t launch_scene_intersect_shadow_pt(hipStream_t s, const SceneView& v,
                                            const spray_rt_ray* rays, size_t M,
                                            spray_rt_hit* hits, const float* shade10,
                                            uint8_t* occluded, uint8_t* sh_valid,
                                            uint32_t* d_count);

// The same for a frame's camera rays (one point light, diffuse surfaces,
// bounces = 1): the spawn rule and light weight of the shading pass
// (k_shade), the weight to sw[i] (float4) for the film.
hipError_t launch_scene_frame_pt(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                 size_t M, spray_rt_hit* hits, const float* shade10,
                                 uint8_t* occluded, uint8_t* sh_valid, float* sw,
                                 uint32_t* d_count, uint32_t* heads = nullptr);
// (heads: kHeadsBytes of queue heads the caller zeroed, with *d_count, in
// one launch -- no memsets before the launch)
// stats[live], stats[shadows] of the frame counters += M, *d_count
hipError_t launch_frame_stats_add(hipStream_t s, unsigned long long* stats, int stripes,
                                  size_t M, const uint32_t* d_count);

// Closest hit + composite key per ray for in-situ compositing:
// (t bits << 32) | (position in the ray's sorted domain list << 16) | domain,
// 0x7FFF...F on a miss (non-resident domains are skipped but counted).
hipError_t launch_scene_intersect_keyed(hipStream_t s, const SceneView& v,
                                        const spray_rt_ray* rays, size_t M,
                                        spray_rt_hit* hits, uint64_t* keys);
// The same over rays idx[0..*d_num) (d_num <= max_n; ray ids < max_n):
// hits[idx[j]] and keys[idx[j]] written.
hipError_t launch_scene_intersect_keyed_indexed(hipStream_t s, const SceneView& v,
                                                const spray_rt_ray* rays, size_t max_n,
                                                const uint32_t* idx, const uint32_t* d_num,
                                                spray_rt_hit* hits, uint64_t* keys);
// out[i] = OR over the ray's domain list of (1 << owner[domain]); owner < 0:
// unowned.  owner: device int[ndom], ranks < 64.  sel (optional): ray i is
// rays[sel[i]]; valid (optional): only slots with valid[i] hold a ray (mask
// 0 elsewhere), their number added to *nvalid (optional).
hipError_t launch_route(hipStream_t s, const SceneView& v, const int* owner,
                        const spray_rt_ray* rays, size_t M, uint64_t* out,
                        const uint32_t* sel = nullptr, const uint8_t* valid = nullptr,
                        unsigned long long* nvalid = nullptr);
hipError_t launch_eye_rays_insitu(hipStream_t s, const float* cam14, int image_w,
                                  int spp, int bx, int by, int bw, int tx, int ty,
                                  int tw, int th, spray_rt_ray* rays, int32_t* pixid,
                                  int32_t* samid);

// Exchange plan: idx = for d in 0..world-1 the ascending i with bit d of
// masks[i] (concatenated); starts[0..world] = list bounds (device int64).
// idx == nullptr: bounds only (size the list first).
// temp: plan_temp_bytes(n, world) bytes of device scratch.
size_t plan_temp_bytes(size_t n, int world);
hipError_t launch_plan(hipStream_t s, const uint64_t* masks, size_t n, int world,
                       int64_t* idx, int64_t* starts, void* temp);
// dst[j] = src[idx[j]], rows of 4, 8, 16, 32 or 48 bytes (16-B aligned
// buffers for the 16-B multiples).
hipError_t launch_gather_rows(hipStream_t s, const void* src, size_t row_bytes,
                              const int64_t* idx, size_t n, void* dst);

hipError_t launch_eye_rays_ooc(hipStream_t s, const float* cam14, int image_w,
                               int spp, int tx, int ty, int tw, int th,
                               spray_rt_ray* rays, int32_t* pixid,
                               int32_t* samid);

// The eye rays of ntiles tiles (x, y, w, h; host array) back to back, as
// one launch_eye_rays_ooc per tile at its offset would write them.
hipError_t launch_eye_rays_ooc_tiles(hipStream_t s, const float* cam14, int image_w, int spp,
                                    const int* tiles, int ntiles, spray_rt_ray* rays,
                                    int32_t* pixid, int32_t* samid);

// Deterministic (ascending source index) compaction of PT shadow rays, in
// one pass (decoupled look-back).  scratch: device memory of
// (ceil(M/kBlock) + 1) uint64.
hipError_t launch_spawn_pt(hipStream_t s, const spray_rt_ray* rays,
                           const spray_rt_hit* hits, size_t M,
                           const float* shade10, spray_rt_ray* out_rays,
                           int32_t* out_src, uint32_t* d_count,
                           void* scratch);

// Ambient-occlusion rays of ooc::ShaderAo, nsamples per hit, compacted in
// (source ray, sample) order; scratch: ao_scratch_bytes(M, nsamples) of
// device memory (per-hit sample masks and tile totals).  order (optional,
// M * nsamples uint32): a trace order of the written rays, sample-major
// within aligned blocks of 8 source rays (the spp rays of a pixel).
// traced: the rays and sources are written in that trace order instead.
hipError_t launch_spawn_ao(hipStream_t s, const spray_rt_ray* rays, const spray_rt_hit* hits,
                           const int32_t* pixid, size_t M, int nsamples,
                           spray_rt_ray* out_rays, int32_t* out_src, uint32_t* d_count,
                           void* scratch, uint32_t* order = nullptr, bool traced = false);
// AO spawn as (source, sample) pairs i << 5 | l in the trace order of
// launch_spawn_ao (traced); nsamples <= 32, M < 2^27; scratch:
// ao_scratch_bytes(M, nsamples).
// lv: the local hemisphere sample of every (pixel, l) the pairs use, as
// float4 at pixel * nsamples + l; rec: per source ray that spawns, 4 float4
// (origin + pixel bits, normal, tangent frame).
hipError_t launch_spawn_ao_pairs(hipStream_t s, const spray_rt_ray* rays,
                                 const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                 int nsamples, size_t npix, uint32_t* out_pairs, float* lv,
                                 float* rec, uint32_t* d_count, void* scratch);
// Replicated in-situ frames: slot j traces eye ray idx[j] (< n), j < nc,
// results at j.  Keyed closest hit over the resident domains (keys: 64-bit
// composite, tkeys: t bits, 0xFFFFFFFF for none) with the point-light
// shading of the own hit (sw float4, sv); hits optional (null: none).
hipError_t launch_scene_rep_keyed(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                  size_t n, const uint32_t* idx, size_t nc,
                                  const float* shade10, spray_rt_hit* hits, uint64_t* keys,
                                  uint32_t* tkeys, float* sw, uint8_t* sv);
// ... and the any hit of the point-light shadow ray of the hit at t bits
// tmin[j] (none: 0xFFFFFFFF, occ[j] untouched) over the resident domains
hipError_t launch_scene_rep_shadows(hipStream_t s, const SceneView& v, const spray_rt_ray* rays,
                                    size_t n, const uint32_t* idx, size_t nc,
                                    const uint32_t* tmin, const float* shade10, uint8_t* occ);
// out[j] = j, j < n
hipError_t launch_iota_u32(hipStream_t s, uint32_t* out, size_t n);
// ---- replicated frames from the camera (insitu.cpp, trace_camera) ----
// A set of the frame's pixels as row runs: pixels x0 .. x0 + len - 1 of row
// y, len = the next run's pbase - pbase (pbase: pixels of the table before
// the run); ubase: the U-space index of pixel (x0, y) (U = the pixels whose
// eye rays may enter a domain box: the union of every box's screen
// footprint, the index space every rank's replicated arrays share).  Work
// item j of a table = sample j % spp of its pixel j / spp; its slot in U =
// (ubase + x - x0) * spp + s.  first[g] = the run holding pixel 8 g of the
// table (one load and a short forward scan per lane instead of a search).
struct CamRun {
  int32_t y, x0;
  uint32_t pbase, ubase;
};
struct CamTable {
  const CamRun* runs;  // [nruns + 1]: a sentinel run with pbase = npix
  const uint32_t* first;
  uint32_t nruns, npix;
};
// render_tiles' footprint-culled eye rays: table T's pixels (each run's
// ubase = the tile-local pixel id of its first pixel), the tile launch's
// rays, pixel and tile-local sample ids at compact indices
hipError_t launch_eye_rays_ooc_table(hipStream_t s, const float* cam14, int image_w, int spp,
                                    const CamTable& T, spray_rt_ray* rays, int32_t* pixid,
                                    int32_t* samid);
// resident domains up to which the camera launches test a lane's boxes
// directly instead of walking the top-level tree
constexpr int kDirectRes = 32;
struct CamFrame {
  float cam[14];  // camera_init's record (eye, image-plane corner, u / v axes, w, h)
  int image_w, spp;
};
// keyed closest hit + point-light shading of the eye rays of table T's
// pixels, generated in the lanes (k_eye_rays_insitu's operations), culled by
// the resident boxes; results at their U slots (slots of dropped lanes
// untouched).  defer_lp (split keys, at most kDirectRes resident domains):
// a lane tests the resident boxes instead of walking the top-level tree,
// and the keys' list-position byte stays 0 for launch_cam_lp
// heads (optional): kHeadsBytes of queue heads the caller has zeroed (its
// frame's launch_clear), used instead of the context's heads and their memset
hipError_t launch_scene_cam_keyed(hipStream_t s, const SceneView& v, const CamFrame& F,
                                  const CamTable& T, const float* shade10, spray_rt_hit* hits,
                                  uint64_t* keys, uint32_t* tkeys, float* sw, uint8_t* sv,
                                  bool defer_lp, uint32_t* heads = nullptr);
// Several buffers set to a byte value in one launch (a frame's clears: one
// kernel instead of a memset -- often two fill kernels -- per buffer)
struct ClearSeg {
  void* p;
  size_t bytes;
  int value;
};
constexpr int kClearSegs = 8;
hipError_t launch_clear(hipStream_t s, const ClearSeg* segs, int n);
// any hit of the point-light shadow ray of every hit in T's pixels (t bits
// tmin[u]; none: 0xFFFFFFFF), the eye ray regenerated in the lane; direct:
// the resident boxes tested instead of the top-level walk (<= kDirectRes)
hipError_t launch_scene_cam_shadows(hipStream_t s, const SceneView& v, const CamFrame& F,
                                    const CamTable& T, const uint32_t* tmin,
                                    const float* shade10, uint8_t* occ, bool direct);
// any hit of those pairs' AO rays, each generated in its any-hit lane;
// idx (optional): only pairs idx[0..*d_count) (occ written at idx[j])
hipError_t launch_occluded_ao_pairs(hipStream_t s, const SceneView& v, size_t max_n,
                                    const uint32_t* pairs, const float* rec, const float* lv,
                                    int nsamples, const uint32_t* d_count, uint8_t* occ,
                                    unsigned long long* counters,
                                    const uint32_t* idx = nullptr, uint32_t* fields = nullptr,
                                    int fb = 0);
// flag[k] = AO pair k (k < min(*d_count, max_n)) enters a resident domain's
// box, 0 for the rest of [0, max_n): the replicated AO frame traces only
// the flagged pairs (idx of launch_occluded_ao_pairs, from
// launch_select_flagged).  mode 1: the pairs starting in a resident domain
// (the domain of the source's key minimum, kmin[pair >> 5] & 0xFFFF); mode
// 2: the other pairs entering a resident box with bit k of bits_a clear.
hipError_t launch_ao_own_flags(hipStream_t s, const SceneView& v, size_t max_n,
                               const uint32_t* pairs, const float* rec, const float* lv,
                               int nsamples, const uint32_t* d_count, uint8_t* flag,
                               const uint64_t* kmin = nullptr, const uint32_t* bits_a = nullptr,
                               int mode = 0);
size_t ao_scratch_bytes(size_t M, int nsamples);

// ---- out-of-core path (ooc_kernels.hip) ----
// One resident domain as its drain launch sees it.
struct OocDomain {
  const void* nodes;
  const void* tris;
  const uint32_t* prims;
  const uint32_t* faces;
  const uint32_t* colors;
  const float* normals;
  float box[6];  // world box (the reference's domain-list test)
  int domain;
};

// Device scratch of the queue build (sized by the caller).
struct OocScratch {
  uint64_t* masks;            // [M * W] per-ray domain list
  uint32_t* val;              // [pair_cap] the queues: ray ids grouped by domain
  uint32_t* first;            // [257] queue bounds
  uint32_t* bc;               // [block_cap] pairs per (ray block, domain), block-major
  uint32_t* sb;               // [block_cap] DomainStats weight per (ray block, domain)
  uint32_t* off;              // [block_cap] a block's offset in its queue, domain-major
  uint32_t* csum;             // [chunk_cap] pairs per (domain, chunk of ray blocks)
  uint32_t* cw;               // [chunk_cap] DomainStats weight per (domain, chunk)
  unsigned long long* score;  // [256] DomainStats score per domain
  uint32_t* live;             // [256] live pairs per queue (see k_ooc_ch_batch)
  uint32_t* dshard;           // [2][256 * kOocDeadShards] deaths since the last snapshot
  uint4* rec;                 // [M][rec_per][3] closest-hit records per batch position
  int rec_per;                // batch positions per ray (the drain's batch size)
  uint8_t* dpos;              // [256] a domain's batch position in the closest-hit pass
  size_t block_cap;           // >= ndom * ray blocks
  size_t chunk_cap;           // >= ndom * ceil(ray blocks / kOocChunk)
  size_t pair_cap;
  uint32_t npair;
};

// Host-visible liveness snapshot (pinned, device-mapped): the kernels that
// end a drain launch store snap[d] = gen << 32 | q.live[d] and then
// seq = gen << 32 | launch number + 1.
struct OocSnapshot {
  unsigned long long* snap;  // [256]
  unsigned long long* seq;   // [1]
  uint32_t gen;
  uint32_t launch;
};

// Builds the per-domain ray queues of a batch (rays with valid[i] == 0 are
// skipped; valid may be null) in one pass over the rays: domain lists,
// per-domain counts and DomainStats scores (ooc_domain_stats.cc:60-111: sum
// over queued pairs of SPRAY_RAY_DOMAIN_LIST_SIZE - list position), queue
// bounds, then a scatter of the ray ids (ascending within each block of
// rays).  key_init (closest hit: the per-ray keys, set to kOocMissKey) and
// occ_clear (any hit: the valid rays' flags, set to 0) may be null.
// Copies first[0..ndom] to h_first and the scores to h_score; q.live[d]
// starts at the queue lengths.  Returns hipErrorOutOfMemory (q.npair =
// needed) when pair_cap is too small.
hipError_t launch_ooc_queues(hipStream_t s, const BvhNode* tlas, int ntlas, int ndom,
                             const float* boxes, const spray_rt_ray* rays, const uint8_t* valid,
                             size_t M, OocScratch& q, uint64_t* key_init, uint8_t* occ_clear,
                             uint32_t* h_first, unsigned long long* h_score);
constexpr uint32_t kOocChunk = 4096;  // ray blocks per chunk of the queue-offset scan
constexpr uint32_t kOocDeadShards = 64;  // death counters per domain (by drain block)
// Per-ray closest-hit key of the ooc drains: t bits << 32 | position in the
// ray's sorted domain list << 16 | domain; a miss is kOocMissKey.
constexpr uint64_t kOocMissKey = ~0ull;
constexpr int kOocBatch = 8;  // resident domains drained by one launch
struct OocBatch {
  OocDomain d[kOocBatch];
  uint32_t begin[kOocBatch];  // queue of d[k]: idx[begin[k] .. begin[k] + n[k])
  uint32_t n[kOocBatch];
  uint32_t wave0[kOocBatch + 1];  // filled by the launcher
  int count;
  // the next batch's domain images, copied by extra blocks of this launch
  // from pinned host memory (device-mapped) into slots no launch of this
  // batch reads: the upload overlaps the drain without a second stream
  const uint4* pf_src[kOocBatch];
  uint4* pf_dst[kOocBatch];
  uint32_t pf_n16[kOocBatch];  // 16-B units
  int pf_count;
  uint32_t copy0;    // first copy block (filled by the launcher)
  uint32_t ncopy;    // copy blocks (filled by the launcher)
};
constexpr int kOocCopyBlocks = 8;  // copy blocks of a launch with prefetches (default; 8 vs 16: ooc 2.88 vs 2.94 ms, r3)
// Closest hit of a batch (traversal + key atomicMin, then the winners'
// records) over the queues of q; boxes the domain boxes.  Pairs whose ray
// gets a nearer hit are counted off q.live; the snapshot follows.
hipError_t launch_ooc_ch_batch(hipStream_t s, OocBatch B, int W, const spray_rt_ray* rays,
                               const OocScratch& q, const float* boxes, uint64_t* key,
                               spray_rt_hit* hits, OocSnapshot snap);
// Miss records of the rays no batch hit (after the last closest-hit batch).
hipError_t launch_ooc_finish(hipStream_t s, const uint64_t* key, const OocScratch& q,
                             spray_rt_hit* hits, size_t M);
// Any hit of a batch; the pairs of newly occluded rays are counted off
// q.live.  Launch k adds its deaths to shard set k & 1 of q.dshard (sets
// 64 * W * kOocDeadShards words apart); its block 0 publishes launch k - 1's
// set (complete at the kernel boundary) as snapshot k - 1.  The pass's last
// launch is not published; launch_ooc_queues clears both sets.
// coherence: SPRAY_RT_RAYS_* (the walk form, as the scene path's any hit)
hipError_t launch_ooc_ah_batch(hipStream_t s, OocBatch B, int W, const spray_rt_ray* rays,
                               const OocScratch& q, uint8_t* occ, OocSnapshot snap,
                               int coherence);
// frame layer (frame_kernels.hip)
hipError_t launch_shade(hipStream_t s, const spray_rt_shader& P, const spray_rt_bsdf* bsdfs,
                        int nbsdf, int bounce, int ns, spray_rt_ray* rays,
                        const spray_rt_hit* hits, float* w, uint8_t* valid,
                        const int32_t* pixid, const int32_t* samid, size_t M,
                        spray_rt_ray* shadows, float* sw, uint8_t* svalid,
                        unsigned long long* stats, int stripes = 1);
constexpr int kStatStripes = 64;  // render_tile's striped shading counters
hipError_t launch_path_init(hipStream_t s, float* w, uint8_t* valid, size_t M);
hipError_t launch_film(hipStream_t s, float* image, const int32_t* pixid, size_t M, int spp,
                       int ns, const float* sw, const uint8_t* svalid, const uint8_t* occ,
                       double scale);
// closest hit of the rays idx[0 .. *d_num) (selected on the device)
hipError_t launch_scene_intersect_indexed(hipStream_t s, const SceneView& v,
                                          const spray_rt_ray* rays, size_t max_n,
                                          const uint32_t* idx, const uint32_t* d_num,
                                          spray_rt_hit* hits);

}  // namespace spray_rt
