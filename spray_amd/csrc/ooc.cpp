// ooc.cpp -- out-of-core scene: the domain images live in pinned host memory
// and stream into a small set of HBM cache slots while the rays queued to
// the resident domains are drained (include/spray_rt.h, spray_rt_ooc_*).
//
// Mirrors LruCache::load (src/render/lru_cache.cc:65-171) + Scene::load
// (src/render/scene.inl:161-187): a domain that is not resident evicts the
// least recently used slot.  The reference rebuilds the mesh and the Embree
// BVH on every miss (TriMeshBuffer::load, trimesh_buffer.cc:117-169,
// TIMER_LOAD); here the BVH image is built once per domain on the host and a
// miss costs one pinned H2D copy on the upload stream, overlapped with the
// drain of the previous domains on the compute stream (events order a slot's
// reuse after its last drain).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "rt_ctx.h"
#include "rt_kernels.h"
#include "spray_rt.h"

using namespace spray_rt;
using namespace spray_rt::detail;

namespace {

struct HostDomain {
  SlotImage img;           // layout only: the bytes live in `pinned`
  void* pinned = nullptr;  // the image, page-locked (DMA source)
  size_t nbytes = 0;
  bool set = false;
};

struct CacheSlot {
  void* dmem = nullptr;
  size_t bytes = 0;
  int domain = -1;
  uint64_t used = 0;                // LRU stamp
  hipEvent_t ready = nullptr;       // upload done (upload stream)
  hipEvent_t released = nullptr;    // last drain using it done (compute stream)
  bool pending_release = false;
};

}  // namespace

struct spray_rt_ooc {
  spray_rt_ctx* ctx = nullptr;
  std::vector<HostDomain> dom;
  std::vector<CacheSlot> slot;
  hipStream_t up = nullptr;
  uint64_t clock = 0;
  unsigned long long loads = 0, hits = 0, bytes = 0, drains = 0;
  // queue scratch
  OocScratch q{};
  size_t q_rays = 0;
  void* q_mem = nullptr;
  uint64_t* tie = nullptr;  // per-ray closest-hit key (kOocMissKey: none yet)
  size_t tie_cap = 0;
  std::vector<uint32_t> first;
};

namespace {

void free_scratch(spray_rt_ooc* o) {
  if (o->q_mem) (void)hipFree(o->q_mem);
  o->q_mem = nullptr;
  o->q = OocScratch{};
  o->q_rays = 0;
}

// (Re)allocates the queue scratch for M rays and `pairs` (domain, ray) pairs.
int size_scratch(spray_rt_ooc* o, size_t M, size_t pairs, int W) {
  spray_rt_ctx* c = o->ctx;
  if (o->q_rays >= M && o->q.pair_cap >= pairs) return SPRAY_RT_OK;
  M = std::max(M, o->q_rays);
  pairs = std::max(pairs, o->q.pair_cap);
  free_scratch(o);
  const size_t temp = ooc_temp_bytes(M, pairs);
  const size_t b_masks = align256(M * W * sizeof(uint64_t));
  const size_t b_cnt = align256((M + 1) * sizeof(uint32_t));
  const size_t b_k = align256(pairs * sizeof(uint16_t));
  const size_t b_v = align256(pairs * sizeof(uint32_t));
  const size_t b_first = align256(257 * sizeof(uint32_t));
  const size_t b_pk = align256(pairs * sizeof(uint64_t));
  const size_t total =
      b_masks + 2 * b_cnt + 2 * b_k + 3 * b_v + b_pk + b_first + align256(temp);
  HIPCHK(c, hipMalloc(&o->q_mem, total));
  char* p = static_cast<char*>(o->q_mem);
  auto take = [&](size_t n) {
    char* r = p;
    p += n;
    return r;
  };
  o->q.masks = reinterpret_cast<uint64_t*>(take(b_masks));
  o->q.npairs = reinterpret_cast<uint32_t*>(take(b_cnt));
  o->q.poff = reinterpret_cast<uint32_t*>(take(b_cnt));
  o->q.key_in = reinterpret_cast<uint16_t*>(take(b_k));
  o->q.key_out = reinterpret_cast<uint16_t*>(take(b_k));
  o->q.val_in = reinterpret_cast<uint32_t*>(take(b_v));
  o->q.val_out = reinterpret_cast<uint32_t*>(take(b_v));
  o->q.first = reinterpret_cast<uint32_t*>(take(b_first));
  o->q.pkey = reinterpret_cast<uint64_t*>(take(b_pk));
  o->q.pleaf = reinterpret_cast<uint32_t*>(take(b_v));
  o->q.temp = take(align256(temp));
  o->q.temp_bytes = temp;
  o->q.pair_cap = pairs;
  o->q_rays = M;
  return SPRAY_RT_OK;
}

// Queues of a ray batch: o->first[d] .. o->first[d+1] index q.val_out.
int build_queues(spray_rt_ooc* o, const spray_rt_ray* rays, const uint8_t* valid, size_t M) {
  spray_rt_ctx* c = o->ctx;
  const int W = c->ndom <= 64 ? 1 : 4;
  int r = size_scratch(o, M, std::max<size_t>(M * 2, 1 << 16), W);
  if (r) return r;
  o->first.assign(c->ndom + 1, 0);
  hipStream_t s = stream_of(c);
  hipError_t e = launch_ooc_queues(s, c->d_tlas, c->ntlas, c->ndom, rays, valid, M, o->q,
                                   o->first.data());
  if (e == hipErrorOutOfMemory) {  // more pairs than guessed: grow, redo
    (void)hipGetLastError();
    r = size_scratch(o, M, o->q.npair, W);
    if (r) return r;
    e = launch_ooc_queues(s, c->d_tlas, c->ntlas, c->ndom, rays, valid, M, o->q,
                          o->first.data());
  }
  HIPCHK(c, e);
  return SPRAY_RT_OK;
}

// Makes domain d resident (LruCache::load) and returns its slot; the compute
// stream is made to wait for the upload.
int acquire(spray_rt_ooc* o, int d, int* out) {
  spray_rt_ctx* c = o->ctx;
  hipStream_t s = stream_of(c);
  int best = -1;
  for (size_t k = 0; k < o->slot.size(); ++k)
    if (o->slot[k].domain == d) best = int(k);
  if (best >= 0) {
    ++o->hits;
  } else {
    // victim: an empty slot, else the least recently used
    for (size_t k = 0; k < o->slot.size() && best < 0; ++k)
      if (o->slot[k].domain < 0) best = int(k);
    if (best < 0) {
      best = 0;
      for (size_t k = 1; k < o->slot.size(); ++k)
        if (o->slot[k].used < o->slot[best].used) best = int(k);
    }
    CacheSlot& cs = o->slot[best];
    const HostDomain& hd = o->dom[d];
    const size_t n = hd.nbytes;
    if (cs.bytes < n) {  // grow: wait for the slot's readers, reallocate
      if (cs.pending_release) HIPCHK(c, hipEventSynchronize(cs.released));
      if (cs.dmem) HIPCHK(c, hipFree(cs.dmem));
      cs.dmem = nullptr;
      HIPCHK(c, hipMalloc(&cs.dmem, n));
      cs.bytes = n;
    }
    if (cs.pending_release) HIPCHK(c, hipStreamWaitEvent(o->up, cs.released, 0));
    HIPCHK(c, hipMemcpyAsync(cs.dmem, hd.pinned, n, hipMemcpyHostToDevice, o->up));
    HIPCHK(c, hipEventRecord(cs.ready, o->up));
    cs.domain = d;
    ++o->loads;
    o->bytes += n;
  }
  CacheSlot& cs = o->slot[best];
  cs.used = ++o->clock;
  HIPCHK(c, hipStreamWaitEvent(s, cs.ready, 0));
  *out = best;
  return SPRAY_RT_OK;
}

OocDomain domain_view(const spray_rt_ooc* o, int d, int k, const float* boxes) {
  const HostDomain& hd = o->dom[d];
  const SlotDesc sd = hd.img.desc_at(o->slot[k].dmem);
  OocDomain D;
  D.nodes = sd.nodes;
  D.tris = sd.tris;
  D.prims = sd.prims;
  D.faces = sd.faces;
  D.colors = sd.colors;
  D.normals = sd.normals;
  std::memcpy(D.box, boxes + 6 * d, sizeof(D.box));
  D.domain = d;
  return D;
}

// Drains every non-empty queue, ascending or descending domain order (a
// closest-hit pass followed by a reversed any-hit pass reuses the domains
// left resident by the first), max(1, slots / 2) resident domains per
// launch: while one batch drains, the LRU victims of the next are the
// previous batch's slots, so its uploads overlap the drain.
template <typename Launch>
int drain(spray_rt_ooc* o, bool reverse, const std::vector<float>& boxes, Launch launch) {
  spray_rt_ctx* c = o->ctx;
  hipStream_t s = stream_of(c);
  const int n = c->ndom;
  const int per = std::max(1, std::min<int>(kOocBatch, int(o->slot.size()) / 2));
  OocBatch B{};
  int bslot[kOocBatch];
  auto flush = [&]() -> int {
    if (B.count == 0) return SPRAY_RT_OK;
    HIPCHK(c, launch(s, B));
    for (int k = 0; k < B.count; ++k) {
      HIPCHK(c, hipEventRecord(o->slot[bslot[k]].released, s));
      o->slot[bslot[k]].pending_release = true;
    }
    o->drains += B.count;  // domain queues drained
    B.count = 0;
    return SPRAY_RT_OK;
  };
  for (int k = 0; k < n; ++k) {
    const int d = reverse ? n - 1 - k : k;
    const uint32_t b = o->first[d], e = o->first[d + 1];
    if (e <= b || !o->dom[d].set || !o->dom[d].img.nnodes) continue;
    int sl = -1;
    int r = acquire(o, d, &sl);
    if (r) return r;
    B.d[B.count] = domain_view(o, d, sl, boxes.data());
    B.begin[B.count] = b;
    B.n[B.count] = e - b;
    bslot[B.count] = sl;
    if (++B.count == per && (r = flush())) return r;
  }
  return flush();
}

int check_batch(spray_rt_ooc* o, const void* rays, size_t M, const void* out) {
  if (!o) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = o->ctx;
  if (c->ndom <= 0 || c->ntlas <= 0)
    return fail(c, SPRAY_RT_ERR_STATE, "no domain bounds set");
  if (c->ndom > SPRAY_RT_MAX_SCENE_DOMAINS)
    return fail(c, SPRAY_RT_ERR_LIMIT, "ooc path supports <= %d domains",
                SPRAY_RT_MAX_SCENE_DOMAINS);
  if (M > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "M > 2^32");
  if (M && (!is_device_ptr(rays) || !is_device_ptr(out)))
    return fail(c, SPRAY_RT_ERR_ARG, "ooc batches need device buffers");
  HIPCHK(c, hipSetDevice(c->device));
  return SPRAY_RT_OK;
}

}  // namespace

extern "C" {

int spray_rt_ooc_create(spray_rt_ctx_t c, int cache_slots, spray_rt_ooc_t* out) {
  if (!c || !out) return SPRAY_RT_ERR_ARG;
  *out = nullptr;
  if (cache_slots <= 0) return fail(c, SPRAY_RT_ERR_ARG, "cache_slots must be > 0");
  if (c->ndom <= 0) return fail(c, SPRAY_RT_ERR_STATE, "no domain bounds set");
  HIPCHK(c, hipSetDevice(c->device));
  spray_rt_ooc* o = new (std::nothrow) spray_rt_ooc;
  if (!o) return SPRAY_RT_ERR_NOMEM;
  o->ctx = c;
  o->dom.resize(c->ndom);
  o->slot.resize(cache_slots);
  hipError_t e = hipStreamCreateWithFlags(&o->up, hipStreamNonBlocking);
  for (CacheSlot& s : o->slot) {
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.released, hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    spray_rt_ooc_destroy(o);
    return fail(c, SPRAY_RT_ERR_HIP, "ooc setup: %s", hipGetErrorString(e));
  }
  *out = o;
  return SPRAY_RT_OK;
}

int spray_rt_ooc_destroy(spray_rt_ooc_t o) {
  if (!o) return SPRAY_RT_ERR_ARG;
  (void)hipSetDevice(o->ctx->device);
  (void)hipDeviceSynchronize();
  for (CacheSlot& s : o->slot) {
    if (s.dmem) (void)hipFree(s.dmem);
    if (s.ready) (void)hipEventDestroy(s.ready);
    if (s.released) (void)hipEventDestroy(s.released);
  }
  for (HostDomain& d : o->dom)
    if (d.pinned) (void)hipHostFree(d.pinned);
  free_scratch(o);
  if (o->tie) (void)hipFree(o->tie);
  if (o->up) (void)hipStreamDestroy(o->up);
  delete o;
  return SPRAY_RT_OK;
}

int spray_rt_ooc_set_domain(spray_rt_ooc_t o, int id, const float* verts, size_t nverts,
                            const uint32_t* faces, size_t nfaces, const uint32_t* colors,
                            const float* normals) {
  if (!o) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = o->ctx;
  if (id < 0 || id >= int(o->dom.size())) return fail(c, SPRAY_RT_ERR_ARG, "bad domain %d", id);
  if ((nverts && !verts) || (nfaces && !faces))
    return fail(c, SPRAY_RT_ERR_ARG, "null mesh arrays");
  HostDomain& hd = o->dom[id];
  SlotImage img;
  if (const char* why = build_slot_image(verts, nverts, faces, nfaces, colors, normals, &img,
                                         /*quantized=*/false))
    return fail(c, SPRAY_RT_ERR_ARG, "ooc domain %d: %s", id, why);
  if (img.depth > kStack) return fail(c, SPRAY_RT_ERR_LIMIT, "tree deeper than the stack");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());  // a resident copy may still be read
  for (CacheSlot& s : o->slot)
    if (s.domain == id) s.domain = -1;  // stale
  if (hd.pinned) HIPCHK(c, hipHostFree(hd.pinned));
  hd.pinned = nullptr;
  HIPCHK(c, hipHostMalloc(&hd.pinned, img.bytes.size(), hipHostMallocDefault));
  std::memcpy(hd.pinned, img.bytes.data(), img.bytes.size());
  hd.nbytes = img.bytes.size();
  hd.img = std::move(img);
  hd.img.bytes.clear();
  hd.img.bytes.shrink_to_fit();
  hd.set = true;
  return SPRAY_RT_OK;
}

int spray_rt_ooc_intersect(spray_rt_ooc_t o, const spray_rt_ray* rays, size_t M,
                           spray_rt_hit* hits) {
  int r = check_batch(o, rays, M, hits);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  spray_rt_ctx* c = o->ctx;
  if (o->tie_cap < M) {
    if (o->tie) HIPCHK(c, hipFree(o->tie));
    o->tie = nullptr;
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&o->tie), M * sizeof(uint64_t)));
    o->tie_cap = M;
  }
  const std::vector<float>& boxes = c->h_boxes;
  if ((r = build_queues(o, rays, nullptr, M))) return r;
  HIPCHK(c, launch_ooc_init(stream_of(c), hits, o->tie, M));
  uint64_t* key = o->tie;
  const int W = c->ndom <= 64 ? 1 : 4;
  return drain(o, false, boxes, [&](hipStream_t s, const OocBatch& B) {
    return launch_ooc_ch_batch(s, B, W, rays, o->q.val_out, o->q.masks, c->d_boxes, key,
                               o->q.pkey, o->q.pleaf, hits);
  });
}

int spray_rt_ooc_occluded(spray_rt_ooc_t o, const spray_rt_ray* rays, size_t M,
                          const uint8_t* valid, uint8_t* occluded) {
  int r = check_batch(o, rays, M, occluded);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  spray_rt_ctx* c = o->ctx;
  if (valid && !is_device_ptr(valid))
    return fail(c, SPRAY_RT_ERR_ARG, "valid must be device memory");
  const std::vector<float>& boxes = c->h_boxes;
  if ((r = build_queues(o, rays, valid, M))) return r;
  HIPCHK(c, launch_ooc_clear_occ(stream_of(c), valid, occluded, M));
  return drain(o, true, boxes, [&](hipStream_t s, const OocBatch& B) {
    return launch_ooc_ah_batch(s, B, rays, o->q.val_out, occluded);
  });
}

int spray_rt_ooc_stats(spray_rt_ooc_t o, unsigned long long out[4]) {
  if (!o || !out) return SPRAY_RT_ERR_ARG;
  out[0] = o->loads;
  out[1] = o->hits;
  out[2] = o->bytes;
  out[3] = o->drains;
  return SPRAY_RT_OK;
}

}  // extern "C"
