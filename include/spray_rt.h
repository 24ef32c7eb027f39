/*
 * spray_rt.h -- C ABI of the MI355X (gfx950) BVH traversal + ray/triangle
 * intersection engine that drops in behind SpRay's scene intersect/occluded
 * surface.
 *
 * Reference interface each entry point replaces (paths relative to the
 * hyungman/SpRay tree):
 *   spray_rt_domain_upload   TriMeshBuffer::load + mapEmbreeBuffer
 *                            (src/render/trimesh_buffer.cc:117-169, :189-225):
 *                            rtcNewTriangleMesh/rtcSetBuffer2/rtcCommit per
 *                            cache block, here a device BVH per slot.
 *   spray_rt_domain_bounds   WbvhEmbree::init/build
 *                            (src/render/wbvh_embree.cc:31-111).
 *   spray_rt_intersect1M     Scene::intersect (src/render/scene.h:157-173,
 *                            scene.inl:189-199): rtcIntersect + the
 *                            TriMeshBuffer::updateIntersection epilogue
 *                            (trimesh_buffer.cc:328-360), over a stream of
 *                            RTCRayIntersection records.
 *   spray_rt_occluded1M      Scene::occluded (scene.h:175-195,
 *                            scene.inl:201-209): rtcOccluded over RTCRay
 *                            records.
 *   spray_rt_domains1M       Scene::intersectDomains -> WbvhEmbree::intersect
 *                            (scene.h:197, wbvh_embree.cc:126-148) +
 *                            DomainList::sort (src/render/rays.h:71-79).
 *   spray_rt_*_segments      the per-domain queue drains of the schedulers
 *                            (src/ooc/ooc_tcontext.inl:28-100,
 *                            src/insitu/insitu_tcontext.inl:125-186) in one
 *                            launch.
 *   spray_rt_*_scene         the speculative resolution of a ray over every
 *                            domain of its list (ooc_isector.h:126-145 +
 *                            ooc_vbuf.cc:54-112): nearest hit over all
 *                            listed domains in one launch.
 *
 * Conventions
 *  - Every function returns SPRAY_RT_OK (0) or a negative status; nothing
 *    throws across the boundary.  spray_rt_last_error() gives the message.
 *  - Ray/hit buffers may be host or device pointers.  With host pointers the
 *    call is synchronous (results are in place on return), as Embree's is.
 *    With device pointers the work is enqueued on the context's stream
 *    (spray_rt_set_stream) and spray_rt_sync() waits for it.
 *  - Result semantics: tfar is written only on a hit;
 *    geomID becomes 0 on a hit / occlusion and is otherwise left as the
 *    caller set it (0xFFFFFFFF); instID is never touched; color (byte
 *    offset 60) and Ns (offset 84) are filled by the fused epilogue.
 *  - One context per GPU; a context is driven by one host thread at a time,
 *    except through lanes (spray_rt_lane_*): one lane per host thread, run
 *    concurrently.
 */
#ifndef SPRAY_RT_H_
#define SPRAY_RT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPRAY_RT_OK 0
#define SPRAY_RT_ERR_ARG (-1)
#define SPRAY_RT_ERR_HIP (-2)
#define SPRAY_RT_ERR_STATE (-3)
#define SPRAY_RT_ERR_NOMEM (-4)
#define SPRAY_RT_ERR_LIMIT (-5)
#define SPRAY_RT_ERR_UNSUPPORTED (-6) /* a case the reference aborts on */

#define SPRAY_RT_INVALID_ID 0xFFFFFFFFu
#define SPRAY_RT_MAX_SCENE_DOMAINS 256

typedef struct spray_rt_ctx* spray_rt_ctx_t;

/* Embree-2 record layouts the stream calls accept (src/render/rays.h:246-274
 * and embree2/rtcore_ray.h).  Only these byte offsets are read or written:
 * org 0, dir 16, tnear 32, tfar 36, Ng 48, color 60, u 64, v 68, geomID 72,
 * primID 76, Ns 84 (RTCRayIntersection; sizeof = 96). */
typedef struct spray_rt_ray_intersection {
  float org[3];
  float align0;
  float dir[3];
  float align1;
  float tnear;
  float tfar;
  float time;
  uint32_t mask;
  float Ng[3];
  uint32_t color;
  float u;
  float v;
  uint32_t geomID;
  uint32_t primID;
  uint32_t instID;
  float Ns[3];
} spray_rt_ray_intersection;

/* Compact ray of the fused scene path: 32 B, two 16-B loads per lane. */
typedef struct spray_rt_ray {
  float org[3];
  float tnear;
  float dir[3];
  float tfar;
} spray_rt_ray;

/* Scene-path hit record (48 B): t = +inf, prim = 0xFFFFFFFF, domain = -1 on
 * a miss; ng = Embree 2 unnormalised geometry normal (v0-v1)x(v2-v0);
 * color/ns = updateIntersection epilogue. */
typedef struct spray_rt_hit {
  float t, u, v;
  uint32_t prim;
  float ng[3];
  uint32_t color;
  float ns[3];
  int32_t domain;
} spray_rt_hit;

/* ---- context ---- */
int spray_rt_create(int hip_device, spray_rt_ctx_t* out);
int spray_rt_destroy(spray_rt_ctx_t ctx);
const char* spray_rt_last_error(spray_rt_ctx_t ctx);
/* Enqueue all further work on hip_stream (a hipStream_t; NULL = the null
 * stream).  A new context uses a private non-blocking stream. */
int spray_rt_set_stream(spray_rt_ctx_t ctx, void* hip_stream);
int spray_rt_sync(spray_rt_ctx_t ctx);

/* ---- domains / cache slots ---- */
/* Uploads one domain mesh (world-space vertices) into cache slot `slot`
 * (SceneInfo.cache_block): builds the BVH on the host and copies BVH,
 * triangles and the epilogue arrays (faces, colors 0xRRGGBB per vertex,
 * unnormalised vertex normals; either may be NULL) to the device.  async=0:
 * returns after the copy completed; async=1: copies are enqueued on the
 * context's upload stream and ordered before the next query. */
int spray_rt_domain_upload(spray_rt_ctx_t ctx, int slot, const float* verts_xyz,
                           size_t nverts, const uint32_t* faces, size_t nfaces,
                           const uint32_t* colors_rgb, const float* vnormals,
                           int async);
/* Releases a slot's device memory. */
int spray_rt_domain_release(spray_rt_ctx_t ctx, int slot);
/* Domain world bounds [n][6] = lo.xyz hi.xyz (Domain::world_aabb). */
int spray_rt_domain_bounds(spray_rt_ctx_t ctx, int ndomains,
                           const float* aabb_min_max);
/* Which slot holds domain `domain_id` for the scene path (-1 = none). */
int spray_rt_map_domain(spray_rt_ctx_t ctx, int domain_id, int slot);
/* BVH statistics of a slot: nodes, depth, triangles. */
int spray_rt_slot_info(spray_rt_ctx_t ctx, int slot, size_t* nnodes,
                       int* depth, size_t* ntris);

/* Host-only: the canonical BVH2 a slot upload would build (no GPU needed).
 * Call with NULL outputs for sizes.  nodes_out: 64-B nodes (padded boxes),
 * tris_out: [ntris][12] v0 e1 e2 Ng, prims_out: leaf order -> face index. */
int spray_rt_bvh_build_host(const float* verts_xyz, size_t nverts,
                            const uint32_t* faces, size_t nfaces,
                            size_t* nnodes, int* depth, void* nodes_out,
                            float* tris_out, uint32_t* prims_out);

/* Host-only: the 16-bit quantized copy of that BVH2 (32-B nodes: u16 l_lo xyz, l_hi xyz, r_lo xyz, r_hi xyz, int32
 * left, right; decoded bound = base + q * scale, grid_out = base xyz, scale
 * xyz).  SPRAY_RT_ERR_LIMIT if the coordinates exceed the grid's range. */
int spray_rt_qnodes_host(const float* verts_xyz, size_t nverts, const uint32_t* faces,
                         size_t nfaces, size_t* nnodes, float grid_out[6], void* qnodes_out);

/* Host-only: the 4-wide quantized collapse of that BVH2 the per-lane any-hit
 * walk reads (64-B nodes: u16 child boxes [4][lo xyz, hi xyz], int32 child
 * refs [4], >= 0 node index, < 0 leaf ~((first << 2) | (count - 1)), INT32_MIN
 * empty; same grid as above), and the walk's stack bound (entries).
 * SPRAY_RT_ERR_LIMIT if the coordinates exceed the grid's range. */
int spray_rt_qnodes4_host(const float* verts_xyz, size_t nverts, const uint32_t* faces,
                          size_t nfaces, size_t* nnodes, int* stack_bound, float grid_out[6],
                          void* qnodes_out);

/* ---- Embree-1M-style streams (drop-in) ---- */
int spray_rt_intersect1M(spray_rt_ctx_t ctx, int slot, void* rays, size_t M,
                         size_t stride);
int spray_rt_occluded1M(spray_rt_ctx_t ctx, int slot, void* rays, size_t M,
                        size_t stride);
/* TriMeshBuffer::updateIntersection (src/render/trimesh_buffer.cc:328-360;
 * Scene::updateIntersection, src/render/scene.h:203) over a stream: color
 * (offset 60) and Ns (offset 84) of every record whose geomID marks a hit,
 * from its primID, u and v and slot's mesh -- the epilogue intersect1M
 * fuses.  stride >= 96. */
int spray_rt_update_intersection1M(spray_rt_ctx_t ctx, int slot, void* rays, size_t M,
                                   size_t stride);
/* nseg segments: rays [offsets[i], offsets[i+1]) against slots[i];
 * offsets has nseg+1 entries (host memory). */
int spray_rt_intersect_segments(spray_rt_ctx_t ctx, const int* slots,
                                const size_t* offsets, int nseg, void* rays,
                                size_t stride);
int spray_rt_occluded_segments(spray_rt_ctx_t ctx, const int* slots,
                               const size_t* offsets, int nseg, void* rays,
                               size_t stride);
/* Sorted domain lists: org/dir are [M][3]; ids/ts are [M][maxhits],
 * counts[M] (truncated at maxhits). */
int spray_rt_domains1M(spray_rt_ctx_t ctx, const float* org, const float* dir,
                       size_t M, int* ids, float* ts, int* counts, int maxhits);

/* ---- lanes: concurrent per-thread submission (Scene's const queries) ---- */
/* The reference calls Scene::intersect / occluded / intersectDomains from
 * every OpenMP thread at once against the loaded domain
 * (src/ooc/ooc_pcontext.h:144-157, ooc_tcontext.inl:28-100).  A lane is one
 * host thread's private stream + staging: calls on different lanes of one
 * context may run concurrently; one lane is driven by one thread at a time.
 * They read the context's slot and domain tables, which must not change
 * while lanes run (the reference loads domains inside omp single between
 * barriers).  Host or device ray buffers; the call returns with the results
 * in place (host) or completed on the lane's stream (device). */
typedef struct spray_rt_lane* spray_rt_lane_t;
int spray_rt_lane_create(spray_rt_ctx_t ctx, spray_rt_lane_t* out);
/* The calling thread's last spray_rt_lane_create failure ("" after a
 * success): lane creation never writes the context's shared message, so
 * threads creating lanes concurrently do not race on it. */
const char* spray_rt_lane_create_error(void);
int spray_rt_lane_destroy(spray_rt_lane_t lane);
const char* spray_rt_lane_last_error(spray_rt_lane_t lane);
int spray_rt_lane_intersect1M(spray_rt_lane_t lane, int slot, void* rays, size_t M,
                              size_t stride);
int spray_rt_lane_occluded1M(spray_rt_lane_t lane, int slot, void* rays, size_t M,
                             size_t stride);
int spray_rt_lane_update_intersection1M(spray_rt_lane_t lane, int slot, void* rays, size_t M,
                                        size_t stride);
int spray_rt_lane_domains1M(spray_rt_lane_t lane, const float* org, const float* dir, size_t M,
                            int* ids, float* ts, int* counts, int maxhits);

/* ---- fused scene path (all listed domains in one launch) ---- */
int spray_rt_intersect_scene(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                             size_t M, spray_rt_hit* hits);
int spray_rt_occluded_scene(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                            size_t M, uint8_t* occluded);
/* Same, with per-launch traversal counters (device uint64[3]: node fetches,
 * triangle tests, (ray, domain) visits) accumulated atomically -- the
 * counting build used to verify the canonical traversal against the oracle. */
int spray_rt_intersect_scene_counted(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                     size_t M, spray_rt_hit* hits,
                                     unsigned long long* d_counters);
int spray_rt_occluded_scene_counted(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                    size_t M, uint8_t* occluded,
                                    unsigned long long* d_counters);
/* Closest hit with the point-light shadow spawn of ooc::ShaderPt fused into
 * the epilogue (shade as for spray_rt_spawn_shadows_pt), written
 * positionally: out_valid[i] = 1 and out_rays[i] = the shadow ray when
 * source ray i spawns one, out_valid[i] = 0 otherwise.  *d_count (device
 * uint32, may be NULL) receives the number spawned.  Deterministic.  Device
 * buffers only. */
int spray_rt_intersect_scene_spawn_pt(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                      size_t M, spray_rt_hit* hits,
                                      const float shade[10], spray_rt_ray* out_rays,
                                      uint8_t* out_valid, uint32_t* d_count);
/* Closest hit, PT shadow spawn and the shadow rays' any hit in ONE launch:
 * hits[i] as spray_rt_intersect_scene; sh_valid[i] = 1 when ray i spawned a
 * point-light shadow ray (as spray_rt_intersect_scene_spawn_pt's out_valid),
 * occluded[i] = its any-hit result (written where sh_valid[i]), *d_count
 * (optional, device) = number of shadow rays.  The shadow rays never leave
 * the chip: each wave queues its spawned rays in LDS and traces them as
 * 64-ray packets.  Results equal spawn_pt + occluded_scene_masked.  Device
 * buffers only. */
int spray_rt_intersect_scene_shadow_pt(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                       size_t M, spray_rt_hit* hits, const float shade[10],
                                       uint8_t* occluded, uint8_t* sh_valid,
                                       uint32_t* d_count);
/* Any hit over the rays i < M with valid[i] != 0 (e.g. the positional spawn
 * output): occluded[i] is written for those rays only.  The valid rays are
 * first compacted into an ascending index list (device select), so the
 * traversal runs on full wavefronts in source order.  Device buffers only. */
int spray_rt_occluded_scene_masked(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                   size_t M, const uint8_t* valid,
                                   uint8_t* occluded);
/* Occlusion of the first *d_count (device uint32, e.g. written by
 * spray_rt_spawn_shadows_pt) of at most max_rays device-resident rays, with
 * no host round trip.  d_counters may be NULL. */
int spray_rt_occluded_scene_devcount(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                     size_t max_rays, const uint32_t* d_count,
                                     uint8_t* occluded,
                                     unsigned long long* d_counters);
/* Any hit of the rays order[j], j < *d_count (device count, <= max_rays),
 * lanes taking them in that order; occluded[order[j]] is written (order =
 * NULL: the identity, rays 0 .. *d_count - 1).  The
 * results equal the positional launch's -- only the grouping of rays into
 * wavefronts changes (e.g. spray_rt_spawn_shadows_ao_ordered's order).
 * Device buffers only. */
int spray_rt_occluded_scene_order(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                  size_t max_rays, const uint32_t* order,
                                  const uint32_t* d_count, uint8_t* occluded);

/* ---- traversal form of the any-hit scene launches ---- */
/* Closest-hit scene launches walk each domain tree as a wave-wide packet
 * (one scalar fetch per node per wave).  Any-hit launches follow this
 * setting: COHERENT = packets (camera / point-light shadow rays), INCOHERENT
 * = one walk per lane (hemisphere-sampled AO rays), ADAPTIVE (default) =
 * per wave, packets when every direction is within ~8 degrees of the
 * wave's first.  Results are identical in every mode. */
#define SPRAY_RT_RAYS_ADAPTIVE 0
#define SPRAY_RT_RAYS_COHERENT 1
#define SPRAY_RT_RAYS_INCOHERENT 2
int spray_rt_set_coherence(spray_rt_ctx_t ctx, int mode);

/* ---- in-situ (domain-sharded, one rank per GPU) ---- */
/* Domain -> rank map of the partition (InsituPartition::rank,
 * src/render/data_partition.h:48-56): owner[ndomains] host array, ranks in
 * [0, 64), -1 = nobody.  Reset by spray_rt_domain_bounds. */
int spray_rt_set_owners(spray_rt_ctx_t ctx, const int* owner);
/* Routing of a ray batch (insitu::Isector::intersect,
 * src/insitu/insitu_isector.h:164-224, speculative: every domain on the
 * list): rank_mask[i] = OR of (1 << owner[d]) over the domains d whose box
 * the ray enters.  Device buffers only. */
int spray_rt_route(spray_rt_ctx_t ctx, const spray_rt_ray* rays, size_t M,
                   uint64_t* rank_mask);
/* Exchange plan of a routed batch (the per-destination queues of
 * insitu_comm.inl, built at once): idx = for d = 0..world-1 the ascending
 * indices i with bit d of rank_mask[i], concatenated; starts[0..world] =
 * the list bounds (int64).  idx == NULL computes the bounds only (starts
 * [world] = the capacity idx needs).  Device buffers only. */
int spray_rt_exchange_plan(spray_rt_ctx_t ctx, const uint64_t* rank_mask, size_t n,
                           int world, int64_t* idx, int64_t* starts);
/* Exchange packing: dst[j] = src[idx[j]] for rows of 4, 8, 16, 32 (a ray)
 * or 48 (a hit record) bytes; idx int64.  Device buffers only. */
int spray_rt_gather_rows(spray_rt_ctx_t ctx, const void* src, size_t row_bytes,
                         const int64_t* idx, size_t n, void* dst);
/* Closest hit over the RESIDENT domains of each ray's list (mapped slots;
 * the others are skipped) plus the composite key that orders hits the way
 * the sequential walk of the whole list does:
 *   keys[i] = (bits(t) << 32) | (list position << 16) | domain,
 *   0x7FFFFFFFFFFFFFFF on a miss.
 * The minimum key over all ranks (VBuf tbuf compositing,
 * src/insitu/insitu_vbuf.h:74-152) identifies the hit of the full scene.
 * Device buffers only. */
int spray_rt_intersect_scene_keyed(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                   size_t M, spray_rt_hit* hits, uint64_t* keys);

/* ---- out-of-core (streamed domains, config 4) ---- */
/* An LRU cache of cache_slots domain images in HBM, fed from pinned host
 * memory (LruCache::load, src/render/lru_cache.cc:65-171; Scene::load,
 * src/render/scene.inl:161-187).  Uses the context's domain boxes
 * (spray_rt_domain_bounds first), stream and device. */
typedef struct spray_rt_ooc* spray_rt_ooc_t;
int spray_rt_ooc_create(spray_rt_ctx_t ctx, int cache_slots, spray_rt_ooc_t* out);
int spray_rt_ooc_destroy(spray_rt_ooc_t ooc);
/* TriMeshBuffer::load (trimesh_buffer.cc:117-169) once per domain: the BVH
 * image is built here and kept in pinned host memory. */
int spray_rt_ooc_set_domain(spray_rt_ooc_t ooc, int domain, const float* verts_xyz,
                            size_t nverts, const uint32_t* faces, size_t nfaces,
                            const uint32_t* colors_rgb, const float* vnormals);
/* Closest hit of a device ray batch over every domain of each ray's list,
 * the domains streamed through the cache in ascending id order (queues
 * built on the device, one drain launch per domain).  Same hit records as
 * spray_rt_intersect_scene.  Device buffers only. */
int spray_rt_ooc_intersect(spray_rt_ooc_t ooc, const spray_rt_ray* rays, size_t M,
                           spray_rt_hit* hits);
/* Any hit of the rays with valid[i] != 0 (valid may be NULL), domains in
 * descending order; occluded[i] written for those rays.  Device buffers. */
int spray_rt_ooc_occluded(spray_rt_ooc_t ooc, const spray_rt_ray* rays, size_t M,
                          const uint8_t* valid, uint8_t* occluded);
/* out[4] = cache loads (misses), cache hits, bytes uploaded, drain launches */
int spray_rt_ooc_stats(spray_rt_ooc_t ooc, unsigned long long out[4]);

/* ---- ray sources on the device (caller side of the hot path) ---- */
/* cam[14] = pos[3], lowerleft[3], wvec[3], hvec[3], image_w, image_h
 * (Camera::init, src/render/camera.h:128-166).  ooc::Tracer::genMultiEyes
 * (src/ooc/ooc_tracer.inl:124-172) over blocking tile (tx,ty,tw,th):
 * rays[n], n = tw*th*spp in bufid order; pixid/samid may be NULL.  All
 * device pointers. */
int spray_rt_eye_rays_ooc(spray_rt_ctx_t ctx, const float cam[14], int image_w,
                          int spp, int tx, int ty, int tw, int th,
                          spray_rt_ray* rays, int32_t* pixid, int32_t* samid);
/* insitu::genMultiSampleEyeRays / genSingleSampleEyeRays
 * (src/insitu/insitu_ray.h:103-182): the stripe (tx,ty,tw,th) of blocking
 * tile (bx,by,bw,bh), jitter seeded by (pixid, sample); samid = the
 * blocking-tile-local sample id.  All device pointers. */
int spray_rt_eye_rays_insitu(spray_rt_ctx_t ctx, const float cam[14], int image_w,
                             int spp, int bx, int by, int bw, int bh, int tx, int ty,
                             int tw, int th, spray_rt_ray* rays, int32_t* pixid,
                             int32_t* samid);
/* Point-light shadow rays of ooc::ShaderPt (src/ooc/ooc_shader_pt.h:93-171)
 * for every hit: compacted into out_rays/out_src (source ray index); the
 * number written goes to *d_count (device int, zeroed by the call).
 * shade[8] = light pos[3], light radiance[3]... see DESIGN.md:
 * shade = {lx, ly, lz, lr, lg, lb, ks_r, ks_g, ks_b, shininess}. */
int spray_rt_spawn_shadows_pt(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                              const spray_rt_hit* hits, size_t M,
                              const float shade[10], spray_rt_ray* out_rays,
                              int32_t* out_src, uint32_t* d_count);

/* Ambient-occlusion rays of ooc::ShaderAo (src/ooc/ooc_shader_ao.h:
 * 120-146): nsamples cosine-weighted hemisphere directions per hit, sample l
 * of pixel p seeded by p * (l + 1) (pixid[i] = the ray's pixel), compacted
 * into out_rays/out_src in (source ray, sample) order; *d_count = number
 * written.  out_rays must hold M * nsamples rays.  Device buffers only. */
int spray_rt_spawn_shadows_ao(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                              const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                              int nsamples, spray_rt_ray* out_rays, int32_t* out_src,
                              uint32_t* d_count);
/* The same rays, plus trace_order[0 .. *d_count) (device uint32, room for
 * M * nsamples): a permutation of the written rays for
 * spray_rt_occluded_scene_order.  The reference seeds sample l of every ray
 * of a pixel with pixid * (l + 1), so the spp rays of one pixel draw the same
 * hemisphere samples; within each aligned block of 8 source rays the order
 * is sample-major (l, then ray), which puts rays of nearly the same origin
 * and direction on neighbouring lanes.  (nsamples > 32: identity.) */
int spray_rt_spawn_shadows_ao_ordered(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                      const spray_rt_hit* hits, const int32_t* pixid,
                                      size_t M, int nsamples, spray_rt_ray* out_rays,
                                      int32_t* out_src, uint32_t* d_count,
                                      uint32_t* trace_order);
/* The same rays written directly in that trace order (out_rays[k] and
 * out_src[k] for k < *d_count: a permutation of spray_rt_spawn_shadows_ao's
 * output), for spray_rt_occluded_scene_order with order = NULL: the any-hit
 * lanes then read rays and write occlusion flags contiguously. */
int spray_rt_spawn_shadows_ao_traced(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                     const spray_rt_hit* hits, const int32_t* pixid,
                                     size_t M, int nsamples, spray_rt_ray* out_rays,
                                     int32_t* out_src, uint32_t* d_count);
/* The spawn of spray_rt_spawn_shadows_ao_traced without the rays: entry k
 * of the same trace order is out_pairs[k] = source ray << 5 | sample l,
 * k < *d_count (4 bytes per AO ray instead of 36); lv receives the local
 * hemisphere sample of every (pixel, l) those rays use (the sampler draw
 * and the double-precision sincos, once per pixel and sample), float4 at
 * pixid * nsamples + l, and rec the origin, normal and tangent frame of
 * every source ray that spawns (16 floats at 16 * i).  nsamples <= 32,
 * M < 2^27; out_pairs holds M * nsamples entries, lv npix * nsamples * 4
 * floats, rec M * 16 floats.  A ray whose pixid lies outside [0, npix)
 * spawns no AO ray (its table entries would lie outside lv). */
int spray_rt_spawn_shadows_ao_pairs(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                    const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                    int nsamples, size_t npix, uint32_t* out_pairs, float* lv,
                                    float* rec, uint32_t* d_count);
/* Scene::occluded of those AO rays (ooc_shader_ao.h:114-160 spawn +
 * scene.inl:201-209), each ray generated in its any-hit lane from
 * (rec[i], lv[pixel * nsamples + l]) with the spawn's operations --
 * the same bits as spawn_shadows_ao_traced + occluded_scene_order(order =
 * NULL), without writing and re-reading 32 B per ray.  occ[k], k <
 * *d_count <= max_n.  d_counters (optional, device u64[3]): the canonical
 * node / triangle / domain-visit counts (counting build). */
int spray_rt_occluded_ao_pairs(spray_rt_ctx_t ctx, size_t max_n, const uint32_t* pairs,
                               const float* rec, const float* lv, int nsamples,
                               const uint32_t* d_count, uint8_t* occ,
                               unsigned long long* d_counters);
/* Both, one call. */
int spray_rt_occluded_ao(spray_rt_ctx_t ctx, const spray_rt_ray* rays, const spray_rt_hit* hits,
                         const int32_t* pixid, size_t M, int nsamples, size_t npix,
                         uint32_t* out_pairs, float* lv, float* rec, uint32_t* d_count,
                         uint8_t* occ, unsigned long long* d_counters);

/* ---- frames: path shading, film, tiles (callers of the hot path) ---- */
/* The shading pass of ooc::ShaderPt (src/ooc/ooc_shader_pt.h:93-227) /
 * ooc::ShaderAo (src/ooc/ooc_shader_ao.h:92-197), the retire-to-image step
 * (ooc_tcontext.inl:123-135 + HdrImage::add, src/display/image.h:90-99), the
 * blocking-tile list (src/render/tile.cc:52-200) and the PPM writer
 * (image.h:167-204), so a whole ooc-mode frame runs on the device. */
#define SPRAY_RT_SHADER_PT 0
#define SPRAY_RT_SHADER_AO 1
#define SPRAY_RT_LIGHT_POINT 0      /* PointLight, src/render/light.h:38-62 */
#define SPRAY_RT_LIGHT_HEMISPHERE 1 /* DiffuseHemisphereLight, light.h:64-90 */
#define SPRAY_RT_BSDF_DIFFUSE 0     /* reflection.h:234-262 */
#define SPRAY_RT_BSDF_MIRROR 1      /* reflection.h:264-287 */
#define SPRAY_RT_BSDF_GLASS 2       /* p = eta_exterior, eta_interior; :292-330 */
#define SPRAY_RT_BSDF_TRANSMISSION 3 /* p = eta_exterior, eta_interior; :335-364 */
#define SPRAY_RT_MAX_LIGHTS 8

typedef struct spray_rt_light {
  int32_t type;
  float pos[3];      /* point lights */
  float radiance[3];
} spray_rt_light;

typedef struct spray_rt_bsdf {
  int32_t type;
  float p[3];
} spray_rt_bsdf;

/* Shader configuration (spray::Config: bounces, ao_samples, ks, shininess;
 * the scene's lights). */
typedef struct spray_rt_shader {
  int32_t shader;   /* SPRAY_RT_SHADER_* */
  int32_t bounces;  /* >= 1 */
  int32_t samples;  /* AO rays per hit / samples per area light */
  int32_t nlights;  /* <= SPRAY_RT_MAX_LIGHTS */
  float ks[3];
  float shininess;
  spray_rt_light lights[SPRAY_RT_MAX_LIGHTS];
} spray_rt_shader;

/* Per-domain BSDFs (Scene::getBsdf(domain), scene_loader.cc:88-130), host
 * array of n entries; domains without an entry are diffuse. */
int spray_rt_set_bsdfs(spray_rt_ctx_t ctx, int n, const spray_rt_bsdf* bsdfs);
/* Shadow rays one path slot can spawn per shading pass (the slot stride of
 * the shadow buffers). */
int spray_rt_shadow_slots(const spray_rt_shader* shader);
/* Closest hit of the rays with valid[i] != 0 (device buffers); hits of the
 * other rays are left as they were. */
int spray_rt_intersect_scene_masked(spray_rt_ctx_t ctx, const spray_rt_ray* rays,
                                    size_t M, const uint8_t* valid, spray_rt_hit* hits);
/* One shading pass over M positional path slots at bounce `bounce` (0 =
 * camera rays).  In: rays[i] (the ray that produced hits[i]), w[i] = path
 * weight (float4, xyz), valid[i].  Out: shadow k of slot i at
 * i*ns + k (ns = spray_rt_shadow_slots) in shadows / sw (float4) /
 * svalid; the next radiance ray in rays[i], w[i], valid[i].  d_stats
 * (device uint64[4], may be NULL) += {cases the reference aborts on (they
 * are skipped), shadow rays spawned, next radiance rays, live slots shaded}.
 * pixid seeds the AO sampler, samid the PT samplers.  Device buffers. */
int spray_rt_shade(spray_rt_ctx_t ctx, const spray_rt_shader* shader, int bounce,
                   spray_rt_ray* rays, const spray_rt_hit* hits, float* w,
                   uint8_t* valid, const int32_t* pixid, const int32_t* samid, size_t M,
                   spray_rt_ray* shadows, float* sw, uint8_t* svalid,
                   unsigned long long* d_stats);
/* image_rgba[pixid] += scale * sw for every unoccluded shadow of the M
 * slots (pixel groups of spp consecutive slots, ns shadows each); float +=
 * double product, in slot then shadow order.  Device buffers. */
int spray_rt_film(spray_rt_ctx_t ctx, float* image_rgba, const int32_t* pixid, size_t M,
                  int spp, int ns, const float* sw, const uint8_t* svalid,
                  const uint8_t* occluded, double scale);
/* One tile of an ooc-mode frame on the device, enqueued on the context's
 * stream (no host synchronisation): eye rays (genMultiEyes), then per
 * bounce closest hit -> shade -> any hit of the shadows -> film.
 * image_rgba: device float[image_w*image_h*4]. */
int spray_rt_render_tile(spray_rt_ctx_t ctx, const spray_rt_shader* shader,
                         const float cam[14], int image_w, int spp, int tx, int ty, int tw,
                         int th, float* image_rgba);
/* Several tiles (tiles[ntiles][4] = x, y, w, h) as one device batch: each
 * tile's eye rays keep their tile-local seeds and every later pass is per
 * sample slot or per pixel, so the image equals rendering the tiles one by
 * one -- with one launch per pass instead of one per tile (the reference's
 * 1M-samples-per-rank tile cap bounds host memory; 288 GB of HBM holds a
 * whole 1024x1024x8 frame's buffers, ~1 GB, many times over). */
int spray_rt_render_tiles(spray_rt_ctx_t ctx, const spray_rt_shader* shader,
                          const float cam[14], int image_w, int spp, const int* tiles,
                          int ntiles, float* image_rgba);
/* Totals of the tiles rendered since the last reset (synchronises the
 * stream): out[3] = radiance rays traced, shadow rays traced, shading cases
 * the reference aborts on (skipped here).  Returns SPRAY_RT_ERR_UNSUPPORTED
 * when out[2] > 0. */
int spray_rt_frame_stats(spray_rt_ctx_t ctx, unsigned long long out[3], int reset);
/* This rank's tiles of the image, tiles[cap][4] = x, y, w, h; *n = count
 * (tiles = NULL, cap = 0: count only).
 *  SPRAY_RT_TILES_IMAGE (ooc mode, ImageScheduleTileList::init, tile.cc:
 *    317-391): the rank's vertical stripe (makeVerticalStripe) cut into
 *    horizontal tiles of at most max_samples_per_rank samples;
 *  SPRAY_RT_TILES_BLOCKING (in-situ mode, TileList::init, tile.cc:52-182):
 *    square-ish blocking tiles of the image, each cut to the rank's
 *    horizontal stripe (makeHorizontalStripe; empty stripes w = h = 0). */
#define SPRAY_RT_TILES_IMAGE 0
#define SPRAY_RT_TILES_BLOCKING 1
int spray_rt_tile_list(int schedule, int image_w, int image_h, int spp, int nranks, int rank,
                       long long max_samples_per_rank, int* tiles, int cap, int* n);
/* HdrImage::writePpm (image.h:167-204): P3, max 1023, bottom row first. */
int spray_rt_write_ppm(const char* path, const float* rgba_host, int w, int h);

/* ---- in-situ frames: the domain-sharded tracer and its exchange ---- */
/* The reference's in-situ mode (src/insitu/): every domain is resident on
 * one rank, rays travel to the owners of the domains on their lists.  The
 * whole per-bounce protocol runs in the engine on the context's stream:
 *   route (Isector::intersect, insitu_isector.h:164-224) -> per-destination
 *   lists -> count exchange -> ray exchange (Comm::run, insitu_comm.inl:
 *   28-101; one grouped ncclSend/ncclRecv all-to-all-v instead of tagged
 *   Isend/Iprobe/Recv) -> keyed closest hit at the owners -> keys back, min
 *   at the ray's holder, the min forward (VBuf::compositeTbuf,
 *   insitu_vbuf.h:109-129, per ray copy) -> the one owner whose key wins
 *   shades (ShaderPt / ShaderAo, insitu_shader_*.h) -> its shadow rays are
 *   routed and exchanged the same way, their occlusion bytes OR-ed back at
 *   the spawner (compositeObuf) -> film (retireShadows) -> the spawned
 *   radiance rays are the spawner's batch of the next bounce.
 * Host round trips per bounce: three small count reads (no per-ray host
 * work).  Collectives go through RCCL (the product: one communicator per
 * in-situ context, spray_rt_insitu_unique_id on rank 0, broadcast by the
 * caller) or, for tests and CPU-side debugging, through host callbacks
 * (spray_rt_transport, buffers staged through host memory). */
typedef struct spray_rt_insitu* spray_rt_insitu_t;

/* Host-memory collectives of the rank group (every rank calls each one in
 * the same order).  Return 0 on success.
 * ABI: this is layout version 2 (SPRAY_RT_TRANSPORT_ABI), which put
 * struct_size in FRONT of `user` -- a breaking change against version 1
 * (round <= 4 callers, `user` at offset 0).  spray_rt_insitu_create reads
 * struct_size before any other field and rejects a value outside
 * [offsetof(allreduce_min_u64), SPRAY_RT_TRANSPORT_MAX_SIZE] with
 * SPRAY_RT_ERR_ARG: a version-1 caller's `user` pointer (or NULL) read as
 * struct_size fails that check instead of shifting every callback.  Within
 * version 2 the struct only grows at its end: a caller's struct_size below
 * sizeof(spray_rt_transport) leaves the later callbacks NULL. */
#define SPRAY_RT_TRANSPORT_ABI 2
#define SPRAY_RT_TRANSPORT_MAX_SIZE 4096
typedef struct spray_rt_transport {
  size_t struct_size;
  void* user;
  /* send_bytes[r] bytes to rank r (consecutive in send), recv_bytes[r] from
   * rank r (consecutive in recv) */
  int (*alltoallv)(void* user, const void* send, const size_t* send_bytes, void* recv,
                   const size_t* recv_bytes);
  int (*allreduce_u64)(void* user, unsigned long long* data, size_t n); /* SUM, in place */
  int (*reduce_f32)(void* user, float* data, size_t n, int root);       /* SUM to root */
  /* replicated-ray frames (spray_rt_insitu_trace_frame); may be NULL, the
   * frame then fails with SPRAY_RT_ERR_UNSUPPORTED */
  int (*allreduce_min_u64)(void* user, unsigned long long* data, size_t n); /* MIN, in place */
  int (*allreduce_sum_u8)(void* user, uint8_t* data, size_t n);            /* SUM, in place */
} spray_rt_transport;

/* Optional per-sample record of a trace (tests, VBuf dumps): for every copy
 * this rank shaded, its sample id, bounce, winning hit and the spawned /
 * occluded bits of its shadow slots (slot k = bit k; <= 64 slots).
 * Appended at *d_count (device, caller-zeroed) in no particular order; the
 * arrays hold cap entries (device memory). */
typedef struct spray_rt_insitu_rec {
  int32_t* samid;
  int32_t* bounce;
  spray_rt_hit* hits;
  unsigned long long* svalid;
  unsigned long long* occluded;
  size_t cap;
  uint32_t* d_count;
} spray_rt_insitu_rec;

/* ncclGetUniqueId for the group's communicator (bytes >= 128). */
int spray_rt_insitu_unique_id(void* id_out, size_t bytes);
/* One in-situ context per rank on ctx (whose domain boxes, owner map
 * (spray_rt_set_owners) and resident slots describe this rank's share).
 * nccl_id != NULL: collectives over RCCL (ncclCommInitRank, blocks until
 * every rank joined); else host != NULL: the given host collectives. */
int spray_rt_insitu_create(spray_rt_ctx_t ctx, int world, int rank, const void* nccl_id,
                           const spray_rt_transport* host, spray_rt_insitu_t* out);
int spray_rt_insitu_destroy(spray_rt_insitu_t ins);
/* InsituPartition::partition, GROUP_CLOSE_DOMAINS (src/render/
 * data_partition.h:59-137): Morton codes of the domain-box centres in the
 * scene bound, sorted by (code, id), dealt out in contiguous shares of
 * ndomains / nranks.  Host only. */
int spray_rt_insitu_partition(const float* boxes, int ndomains, const float scene_bound[6],
                              int nranks, int* owner_out);
/* The same with the partition mode of data_partition.h: GROUP_CLOSE (the
 * contiguous shares above, :118-137, the reference's compiled mode) or
 * ROUND_ROBIN (the sorted Morton order dealt out one domain per rank in
 * turn, "trying to scatter close domains", :139-155). */
#define SPRAY_RT_PARTITION_GROUP_CLOSE 0
#define SPRAY_RT_PARTITION_ROUND_ROBIN 1
int spray_rt_insitu_partition_mode(const float* boxes, int ndomains, const float scene_bound[6],
                                   int nranks, int mode, int* owner_out);
/* This rank's part of a frame: rays[n] / pixid / samid are its eye rays
 * (spray_rt_eye_rays_insitu of its stripe; samid = blocking-tile sample id),
 * traced for shader->bounces bounces across the group; the contributions
 * of the samples this rank shades are added to image_rgba (device float
 * [w*h*4], scaled 1/spp).  totals (host, optional): the group's radiance
 * rays, shadow rays and reference-abort cases (the same on every rank).
 * rec (optional): see spray_rt_insitu_rec.  Device buffers only. */
int spray_rt_insitu_trace(spray_rt_insitu_t ins, const spray_rt_shader* shader,
                          const spray_rt_ray* rays, const int32_t* pixid, const int32_t* samid,
                          size_t n, int spp, float* image_rgba, const spray_rt_insitu_rec* rec,
                          unsigned long long totals[3]);
/* The whole frame with replicated eye rays: rays[n] / pixid / samid are
 * EVERY eye ray of the frame (spray_rt_eye_rays_insitu over the whole
 * blocking tile; tnear SPRAY_RAY_EPSILON and tfar +inf, as every radiance
 * ray of the reference), the same on every rank.  Instead of moving rays to
 * their domains' owners, each rank
 *   1. selects C' = the rays that enter the scene's bounding box (a
 *      superset of the rays with a domain on their list, the same ascending
 *      list on every rank);
 *   2. traces C' over its own domains in one launch: keyed closest hit (t,
 *      list position, domain) and the point-light shading of its own hit;
 *   3. joins a MIN all-reduce of the t bits, then of the list positions at
 *      that t (a byte each, beside step 4) -- the sequential walk's winner
 *      of every ray on every rank (VBuf::compositeTbuf, insitu_vbuf.h:
 *      109-129, per ray instead of per tile);
 *   4. any-hits the point-light shadow ray of every hit, built in the lanes
 *      from (org, dir, minimum t) -- the winner's bits -- over its domains;
 *   5. joins one SUM all-reduce of the occlusion bytes over C', the frame
 *      totals riding behind them (compositeObuf + WorkStats::reduce);
 *   6. films the unoccluded shadows of the rays it won into per-run sums
 *      (a run = consecutive rays of C' with one pixel: the spp samples of a
 *      pixel), which one RCCL reduce (12 B per run instead of the 16-B-per-
 *      pixel image) brings to rank 0, where they are added to image_rgba.
 * The WHOLE frame lands in rank 0's image; the other ranks' images are not
 * touched (no spray_rt_insitu_composite needed).  No ray, hit or shadow
 * record crosses the wire and no count is exchanged: three all-reduces, one
 * reduce and one host read per frame.  Results per sample are the
 * protocol's (the same winner, shading and occlusion).
 * AO (ooc::ShaderAo, one bounce, <= 32 samples, diffuse surfaces): after 3.
 * the winners publish their hits' shading normal and colour (one SUM
 * all-reduce, 16 B per ray of C), every rank spawns the same AO rays of
 * every hit and any-hits them over its own domains, one SUM all-reduce of
 * per-sample occlusion count fields (2 / 4 / 8 bits for world <= 3 / 15 /
 * 64) ORs the group's results, and rank 0 films the WHOLE frame (the other
 * ranks' images are not touched: no composite needed).  Three all-reduces
 * and one host read per frame; totals without a collective.
 * Needs one of those two cases and, with host collectives,
 * allreduce_min_u64 / allreduce_sum_u8; SPRAY_RT_ERR_UNSUPPORTED otherwise
 * (trace with spray_rt_insitu_trace).  World 1: the all-local frame. */
int spray_rt_insitu_trace_frame(spray_rt_insitu_t ins, const spray_rt_shader* shader,
                                const spray_rt_ray* rays, const int32_t* pixid,
                                const int32_t* samid, size_t n, int spp, float* image_rgba,
                                const spray_rt_insitu_rec* rec, unsigned long long totals[3]);
/* The replicated-ray frame of a camera (the N > 1 in-situ frame of
 * bench.py): the frame of spray_rt_insitu_trace_frame for the eye rays of
 * the whole image_w x image_h x spp image as one blocking tile
 * (insitu::genMultiSampleEyeRays, insitu_ray.h:103-182; the rays, pixel and
 * sample ids spray_rt_eye_rays_insitu writes for tile = stripe = image),
 * generated in the lanes from cam (spray_camera_init's 14 floats, for
 * that image size) -- no ray buffer.  Each rank's work follows its own
 * domains instead of the frame: the pixels whose eye rays may enter one of
 * its resident domain boxes (the boxes' conservative screen footprints) are
 * the closest-hit launch, the pixels whose hit points' point-light shadow
 * rays may cross one of its boxes the any-hit launch; the ranks agree
 * through the same collectives over U (the pixels any domain box may be
 * seen through, the same on every rank), with no host read.  Same results
 * per sample as spray_rt_insitu_trace_frame on those rays.  AO: U's eye rays
 * generated in one pass, then the replicated AO frame over them.  World 1:
 * the eye rays, then the all-local frame. */
int spray_rt_insitu_trace_camera(spray_rt_insitu_t ins, const spray_rt_shader* shader,
                                 const float cam[14], int image_w, int image_h, int spp,
                                 float* image_rgba, const spray_rt_insitu_rec* rec,
                                 unsigned long long totals[3]);
/* The image-parallel frame of a camera (the reference's ooc
 * mode shards as replicas -- any rank may hold any domain -- and only the
 * image is composited): EVERY domain resident on every rank (ERR_STATE
 * otherwise), the image_h rows cut into world * bands horizontal bands of
 * equal height (bands > 1: image_h divisible by world * bands), rank r
 * owns bands r, r + world, ... (bands = 1: makeHorizontalStripe,
 * tile.cc:187-209).  Each rank generates its bands' eye rays
 * (insitu::genMultiSampleEyeRays seeds: (pixel, sample), so any split
 * gives every pixel the same bits), traces them with the all-local frame of
 * world 1 (any shading spray_rt_insitu_trace supports: the fused PT launch,
 * or bounces, area lights, AO, delta BSDFs through the frame passes), adds
 * its film to its own rows of image_rgba, and the rows go to rank 0 in one
 * gather (HdrImage::composite, image.h:167-181, an MPI_Reduce SUM of
 * disjoint pixels there; here each rank sends only its own rows, 1/world of
 * the image -- when only the eye rays of pixels some domain box's footprint
 * covers are traced, see SPRAY_IMAGE_CULL, only those pixels' RGB, 12 B
 * each): rank 0's image holds the whole frame, its other ranks' pixels
 * REPLACED by theirs (clear the images first, HdrImage::clear).  One
 * gather (the data all-to-all-v, every rank but 0 sending) and one totals
 * all-reduce per frame; totals = the group's. */
int spray_rt_insitu_trace_image(spray_rt_insitu_t ins, const spray_rt_shader* shader,
                                const float cam[14], int image_w, int image_h, int spp, int bands,
                                float* image_rgba, const spray_rt_insitu_rec* rec,
                                unsigned long long totals[3]);
/* A view-aligned partition of n domain boxes (float[n][6]) over nranks for
 * camera cam: the box centres projected to the image and dealt by recursive
 * median splits (image x, then y, alternating; ties by domain id) into
 * groups of n / nranks (+1) -- each rank the domains along neighbouring
 * lines of sight, so that a ray's domain list mostly stays on one rank.  An
 * addition to InsituPartition's modes (data_partition.h:59-155) for a fixed
 * camera; results do not depend on the partition. */
int spray_rt_insitu_partition_view(const float* boxes, int n, const float cam[14], int nranks,
                                   int* owner);
/* Footprint primitives of the camera frames (tests): per image row y the
 * inclusive pixel range [x0[y], x1[y]] holding every eye ray of cam that
 * may enter box (x0 > x1: none; returns 0 = no pixel, 1 = rows, 2 = the
 * whole image; -1 bad arguments); the k slice boxes (out float[k][6])
 * whose union holds every hit point inside scene whose shadow ray toward
 * the point light may cross box (returns their count, -1 = everywhere). */
int spray_rt_camera_box_rows(const float cam[14], int image_w, int image_h, const float box[6],
                             int* x0, int* x1);
int spray_rt_camera_shadow_boxes(const float box[6], const float scene[6], const float light[3],
                                 int k, float* out);
/* Measurement: one rank of an N-rank group rehearsed alone on one GPU.  A
 * replay context's collectives do not communicate: the camera frame's
 * t-bits and list-position MINs copy the group results given by
 * spray_rt_insitu_replay_set (device arrays over U, as
 * spray_rt_insitu_replay_capture reads them after a one-rank replicated
 * camera frame with every domain resident, SPRAY_INSITU_REPLICATED=1), the
 * SUMs and the reduce keep the rank's own values.  Its device work is the
 * rank's exact share of the N-rank frame (its launches, their sizes and the
 * rays they walk), back to back on its stream; the film and totals it
 * produces are not the frame's.  PT camera frames with split keys, and AO
 * camera frames (spray_rt_insitu_replay_set_ao). */
int spray_rt_insitu_create_replay(spray_rt_ctx_t ctx, int world, int rank,
                                  spray_rt_insitu_t* out);
int spray_rt_insitu_replay_set(spray_rt_insitu_t ins, const uint32_t* d_tmin,
                               const uint8_t* d_lpmin, size_t n);
/* *n = U slots of the last camera PT frame; with d_tmin / d_lpmin (device,
 * cap entries) copies its group t-bits minima and list-position minima. */
int spray_rt_insitu_replay_capture(spray_rt_insitu_t ins, uint32_t* d_tmin, uint8_t* d_lpmin,
                                   size_t cap, size_t* n);
/* The same for AO camera frames: the 64-bit key minima over U (d_kmin, n)
 * and the winners' published normals and colours (d_pub, 2 n uint64 --
 * the publish step's SUM); capture after a one-rank replicated AO camera
 * frame with every domain resident. */
int spray_rt_insitu_replay_set_ao(spray_rt_insitu_t ins, const uint64_t* d_kmin,
                                  const uint64_t* d_pub, size_t n);
int spray_rt_insitu_replay_capture_ao(spray_rt_insitu_t ins, uint64_t* d_kmin, uint64_t* d_pub,
                                      size_t cap, size_t* n);
/* The AO frame's first-round occlusion bits (a pair occluded by its home
 * rank, which depend on the partition): with d_out, copies the last frame's
 * own bits (*n bytes; rehearse every rank once, OR them); else sets d_bits
 * (nbytes, the group's OR) as the result of that SUM; *n = the byte count. */
int spray_rt_insitu_replay_bits_ao(spray_rt_insitu_t ins, const uint8_t* d_bits, uint8_t* d_out,
                                   size_t nbytes, size_t* n);
/* Per-phase device time of the traces since the last call (then reset),
 * HIP events on the context's stream, when phase timing is on
 * (spray_rt_insitu_set_timing).  out_ms[9]; *nphases = phases of the last
 * trace's form: replicated frame {lists, keyed closest hit, shadows, film,
 * totals}; protocol {route + plan, ray exchange, keyed closest hit, key
 * composite, shading, shadow route + exchange, shadow any hit + return,
 * film + totals}; all-local {frame}.  out_ms[8]: the time inside the
 * collectives (and the host reads of their counts), whatever the form. */
int spray_rt_insitu_set_timing(spray_rt_insitu_t ins, int on);
int spray_rt_insitu_phase_times(spray_rt_insitu_t ins, double out_ms[9], int* nphases);
/* HdrImage::composite (src/display/image.h:167-181): SUM of the ranks'
 * images at rank 0 (device float[nfloats], in place). */
int spray_rt_insitu_composite(spray_rt_insitu_t ins, float* image_rgba, size_t nfloats);
/* out[6] = bytes sent to other ranks, bytes received, exchanges, host
 * count reads, collectives issued, traces -- since creation. */
int spray_rt_insitu_stats(spray_rt_insitu_t ins, unsigned long long out[6]);
/* The issue log of the group's collectives since creation or the last
 * clear, in host call order -- what every rank must enqueue identically for
 * RCCL (per communicator, across its streams).  Entry = op << 56 | side << 51
 * | element count (48 bits); op: 1 count all-to-all (int64[world]), 2 data
 * all-to-all-v (bytes; count 0: per-peer counts differ by rank and match
 * pairwise), 3 all-reduce SUM u64, 4 reduce SUM f32 to rank 0, 5 all-reduce
 * MIN u64, 6 all-reduce SUM u8, 7 all-reduce MIN u32, 8 all-reduce MIN u8;
 * side = enqueued on the engine's second stream.  *n = entries logged (the
 * first min(cap, 65536) are copied to out); clear != 0 empties the log. */
int spray_rt_insitu_collective_log(spray_rt_insitu_t ins, uint64_t* out, size_t cap, size_t* n,
                                   int clear);

#ifdef __cplusplus
}
#endif
#endif
