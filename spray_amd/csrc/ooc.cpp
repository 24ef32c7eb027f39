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
#include <cstdio>
#include <cstdlib>
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
  void* pinned = nullptr;  // the image, page-locked and device-mapped
  void* dpinned = nullptr; // its device-side address (read by the copy blocks)
  size_t nbytes = 0;       // padded to 16 B
  bool set = false;
};

struct CacheSlot {
  void* dmem = nullptr;
  size_t bytes = 0;
  int domain = -1;
  uint64_t used = 0;                // LRU stamp
};

}  // namespace

struct spray_rt_ooc {
  spray_rt_ctx* ctx = nullptr;
  std::vector<HostDomain> dom;
  std::vector<CacheSlot> slot;
  uint64_t clock = 0;
  unsigned long long loads = 0, hits = 0, bytes = 0, drains = 0;
  // queue scratch
  OocScratch q{};
  size_t q_rays = 0;
  void* q_mem = nullptr;
  uint64_t* tie = nullptr;  // per-ray closest-hit key (kOocMissKey: none yet)
  size_t tie_cap = 0;
  void* rec = nullptr;  // closest-hit records per (ray, batch position), OocScratch::rec
  size_t rec_cap = 0;
  std::vector<uint32_t> first;
  std::vector<unsigned long long> score;  // DomainStats scores of the last queue build
  // drain launches: one event per launch in a ring (slot reuse, error
  // checks), the live-count snapshot the kernels publish (OocSnapshot:
  // pinned, device-mapped, [0..255] counts, [256] sequence), the any-hit
  // last-block counter
  static constexpr int kRing = 16;
  hipEvent_t launch_ev[kRing] = {};
  unsigned long long launches = 0;
  unsigned long long* snap = nullptr;
  uint32_t gen = 0;
  uint32_t* done = nullptr;  // any-hit last-block counter
  unsigned long long skipped = 0;
};

namespace {

void free_scratch(spray_rt_ooc* o) {
  if (o->q_mem) (void)hipFree(o->q_mem);
  o->q_mem = nullptr;
  o->q = OocScratch{};
  o->q_rays = 0;
}

// Domains drained per launch: half the slots (the other half takes the next
// batch's images during the launch).  SPRAY_OOC_PER overrides (A/B, tests):
// up to slots - 1 measured the same (4.14-4.22 vs 4.15-4.25 ms per frame,
// batches of 3 / 1), every slot with the uploads as DMAs between the
// launches slower (4.37 ms).
int batch_per(const spray_rt_ooc* o) {
  const char* per_s = std::getenv("SPRAY_OOC_PER");  // read per pass (tests set it)
  const int per_env = per_s ? std::atoi(per_s) : 0;
  const int nslots = int(o->slot.size());
  return std::max(1, std::min<int>(kOocBatch, per_env > 0 ? std::min(per_env, nslots)
                                                           : nslots / 2));
}

// (Re)allocates the queue scratch for M rays and `pairs` (domain, ray) pairs.
int size_scratch(spray_rt_ooc* o, size_t M, size_t pairs, int W) {
  spray_rt_ctx* c = o->ctx;
  if (o->q_rays >= M && o->q.pair_cap >= pairs) return SPRAY_RT_OK;
  M = std::max(M, o->q_rays);
  pairs = std::max(pairs, o->q.pair_cap);
  free_scratch(o);
  const size_t rblk = (M + kBlock - 1) / kBlock;  // ray blocks
  const size_t nblk = rblk * size_t(64 * W);
  const size_t nchk = (rblk + kOocChunk - 1) / kOocChunk * size_t(64 * W);
  const size_t b_masks = align256(M * W * sizeof(uint64_t));
  const size_t b_v = align256(pairs * sizeof(uint32_t));
  const size_t b_blk = align256(nblk * sizeof(uint32_t));
  const size_t b_dom = align256(257 * sizeof(uint32_t));
  const size_t b_score = align256(256 * sizeof(unsigned long long));
  const size_t b_dpos = align256(256);
  const size_t b_ch = align256(nchk * sizeof(uint32_t));
  // two sets: an any-hit launch adds to one while it publishes the other
  const size_t b_dsh = align256(2 * 256 * kOocDeadShards * sizeof(uint32_t));
  const size_t total =
      b_masks + b_v + 3 * b_blk + 2 * b_dom + 2 * b_ch + b_score + b_dsh + b_dpos;
  HIPCHK(c, hipMalloc(&o->q_mem, total));
  char* p = static_cast<char*>(o->q_mem);
  auto take = [&](size_t n) {
    char* r = p;
    p += n;
    return r;
  };
  o->q.masks = reinterpret_cast<uint64_t*>(take(b_masks));
  o->q.val = reinterpret_cast<uint32_t*>(take(b_v));
  o->q.bc = reinterpret_cast<uint32_t*>(take(b_blk));
  o->q.sb = reinterpret_cast<uint32_t*>(take(b_blk));
  o->q.off = reinterpret_cast<uint32_t*>(take(b_blk));
  o->q.first = reinterpret_cast<uint32_t*>(take(b_dom));
  o->q.live = reinterpret_cast<uint32_t*>(take(b_dom));
  o->q.csum = reinterpret_cast<uint32_t*>(take(b_ch));
  o->q.cw = reinterpret_cast<uint32_t*>(take(b_ch));
  o->q.score = reinterpret_cast<unsigned long long*>(take(b_score));
  o->q.dshard = reinterpret_cast<uint32_t*>(take(b_dsh));
  o->q.dpos = reinterpret_cast<uint8_t*>(take(b_dpos));
  o->q.block_cap = nblk;
  o->q.chunk_cap = nchk;
  o->q.pair_cap = pairs;
  o->q_rays = M;
  return SPRAY_RT_OK;
}

// Queues of a ray batch: o->first[d] .. o->first[d+1] index q.val_out.
// key_init / occ_clear: the pass's per-ray results to reset (may be null).
int build_queues(spray_rt_ooc* o, const spray_rt_ray* rays, const uint8_t* valid, size_t M,
                 uint64_t* key_init, uint8_t* occ_clear) {
  spray_rt_ctx* c = o->ctx;
  const int W = c->ndom <= 64 ? 1 : 4;
  int r = size_scratch(o, M, std::max<size_t>(M * 2, 1 << 16), W);
  if (r) return r;
  o->first.assign(c->ndom + 1, 0);
  o->score.assign(c->ndom, 0);
  hipStream_t s = stream_of(c);
  hipError_t e = launch_ooc_queues(s, c->d_tlas, c->ntlas, c->ndom, c->d_boxes, rays, valid, M,
                                   o->q, key_init, occ_clear, o->first.data(), o->score.data());
  if (e == hipErrorOutOfMemory) {  // more pairs than guessed: grow, redo
    (void)hipGetLastError();
    r = size_scratch(o, M, o->q.npair, W);
    if (r) return r;
    e = launch_ooc_queues(s, c->d_tlas, c->ntlas, c->ndom, c->d_boxes, rays, valid, M, o->q,
                          key_init, occ_clear, o->first.data(), o->score.data());
  }
  HIPCHK(c, e);
  return SPRAY_RT_OK;
}

// Makes domain d resident (LruCache::load) and returns its slot.  A miss
// evicts the least recently used slot (an empty one first) and returns the
// upload in *up (the caller issues it: copy blocks of the launch before, or
// a DMA on the compute stream); slots in `busy` are never evicted.
struct Upload {
  int slot = -1, domain = -1;
};
int acquire(spray_rt_ooc* o, int d, const std::vector<char>& busy, int* out, Upload* up) {
  spray_rt_ctx* c = o->ctx;
  int best = -1;
  for (size_t k = 0; k < o->slot.size(); ++k)
    if (o->slot[k].domain == d) best = int(k);
  if (best >= 0) {
    ++o->hits;
  } else {
    for (size_t k = 0; k < o->slot.size() && best < 0; ++k)
      if (o->slot[k].domain < 0 && !busy[k]) best = int(k);
    if (best < 0)
      for (size_t k = 0; k < o->slot.size(); ++k)
        if (!busy[k] && (best < 0 || o->slot[k].used < o->slot[best].used)) best = int(k);
    if (best < 0) {  // every slot is held by the batch before: after its launch
      *out = -1;
      return SPRAY_RT_OK;
    }
    CacheSlot& cs = o->slot[best];
    const size_t n = o->dom[d].nbytes;
    if (cs.bytes < n) {  // grow: every queued reader of the slot first
      HIPCHK(c, hipStreamSynchronize(stream_of(c)));
      if (cs.dmem) HIPCHK(c, hipFree(cs.dmem));
      cs.dmem = nullptr;
      HIPCHK(c, hipMalloc(&cs.dmem, n));
      cs.bytes = n;
    }
    cs.domain = d;
    ++o->loads;
    o->bytes += n;
    up->slot = best;
    up->domain = d;
  }
  o->slot[best].used = ++o->clock;
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

// Drains the queues in the reference's DomainStats order
// (ooc_pcontext.h:128-132: rstats_.schedule(), highest score first;
// ooc_domain_stats.cc:60-111), the any-hit pass starting with the domains
// the closest-hit pass left resident.  slots / 2 resident domains per
// launch, and each launch also uploads the next batch's missing images
// into the other slots (copy blocks reading the pinned images; the slots of
// the launch itself are never evicted): the upload overlaps the drain on
// the one compute stream, with no cross-stream wait.  With fewer than two
// batches' worth of slots the upload is a DMA on the stream between the two
// launches instead.
//
// A queue with no live pair left (q.live, see k_ooc_ch_batch: every queued
// ray already has a hit nearer than the domain's entry t, or is occluded) is
// skipped, domain load included -- the reference filters the same rays out
// of the queue when it drains it (filterRqs / filterSqs,
// ooc_tcontext.inl:138-170) and the sweep visits domains near the camera
// first, so most far domains die this way.  Each launch publishes its
// counts to pinned host memory from the device (OocSnapshot); the batch
// after next is chosen once the previous launch's counts have landed, so
// the compute stream always holds the next launch.  Counts only fall, so a
// queue seen dead is dead for certain and results equal draining everything.
template <typename Launch>
int drain(spray_rt_ooc* o, bool any_hit, const std::vector<float>& boxes, Launch launch) {
  spray_rt_ctx* c = o->ctx;
  hipStream_t s = stream_of(c);
  const int n = c->ndom;
  const int per = batch_per(o);  // slots / 2 domains per launch
  std::vector<int> order;
  std::vector<uint32_t> live(n, 0);
  for (int d = 0; d < n; ++d) {
    live[d] = o->first[d + 1] - o->first[d];
    if (live[d] && o->dom[d].set && o->dom[d].img.nnodes) order.push_back(d);
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return o->score[a] > o->score[b];  // ties: ascending id
  });
  if (any_hit)  // reuse what the closest-hit pass left resident
    std::stable_partition(order.begin(), order.end(), [&](int d) {
      for (const CacheSlot& cs : o->slot)
        if (cs.domain == d) return true;
      return false;
    });
  OocSnapshot S{o->snap, o->snap + 256, ++o->gen, 0};
  volatile unsigned long long* snap = o->snap;
  const unsigned long long g = (unsigned long long)S.gen << 32;
  // waits for launch `k` of this pass (0-based) to publish (or complete),
  // then folds the newest counts in
  // launch k's counts are published by launch k + 1 (a block of the next
  // drain), so the wait watches the publisher's event
  auto absorb = [&](uint32_t k, int ring) -> int {
    for (unsigned spins = 0; snap[256] < g + k + 1; ++spins) {
      if ((spins & 1023) == 1023) {  // also watch the launch itself (errors)
        const hipError_t e = hipEventQuery(o->launch_ev[ring]);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) HIPCHK(c, e);
      }
    }
    for (int d = 0; d < n; ++d) {
      const unsigned long long v = snap[d];
      if ((v >> 32) == S.gen) live[d] = std::min(live[d], uint32_t(v));
    }
    return SPRAY_RT_OK;
  };
  std::vector<char> done(n, 0);
  int r = SPRAY_RT_OK;
  int rings[4] = {0, 0, 0, 0};
  // the counts of launch k - 1 (measured the same as k - 2 / k - 3)
  constexpr int lag = 1;
  static const bool trace = std::getenv("SPRAY_OOC_TRACE") != nullptr;  // schedule log
  if (trace)
    std::fprintf(stderr, "ooc pass %s: %zu queues, %u pairs\n", any_hit ? "any" : "closest",
                 order.size(), o->first[n]);
  // the next batch: the first `per` undone queues not known dead; `busy`
  // slots (the batch launched before it, and the slots this batch already
  // took) are not evicted
  std::vector<char> busy(o->slot.size(), 0);
  auto pick = [&](OocBatch& B, int* bslot, std::vector<Upload>& ups) -> int {
    B = OocBatch{};
    ups.clear();
    for (int d : order) {
      if (done[d]) continue;
      if (live[d] == 0) {
        done[d] = 1;
        ++o->skipped;
        continue;
      }
      int sl = -1;
      Upload up;
      if (int e = acquire(o, d, busy, &sl, &up)) return e;
      if (sl < 0) break;  // no free slot until the batch before has run
      busy[size_t(sl)] = 1;  // not evicted by a later domain of this batch
      if (up.slot >= 0) ups.push_back(up);
      B.d[B.count] = domain_view(o, d, sl, boxes.data());
      B.begin[B.count] = o->first[d];
      B.n[B.count] = o->first[d + 1] - o->first[d];
      bslot[B.count] = sl;
      done[d] = 1;
      if (++B.count == per) break;
    }
    return SPRAY_RT_OK;
  };
  auto dma = [&](const Upload& u) -> int {
    HIPCHK(c, hipMemcpyAsync(o->slot[u.slot].dmem, o->dom[u.domain].pinned,
                             o->dom[u.domain].nbytes, hipMemcpyHostToDevice, s));
    return SPRAY_RT_OK;
  };
  OocBatch cur, nxt;
  int cslot[kOocBatch], nslot[kOocBatch];
  std::vector<Upload> cups, nups;
  if ((r = pick(cur, cslot, cups))) return r;
  for (const Upload& u : cups)  // the pass's first batch: DMA before its launch
    if ((r = dma(u))) return r;
  while (cur.count) {
    std::fill(busy.begin(), busy.end(), 0);
    for (int k = 0; k < cur.count; ++k) busy[cslot[k]] = 1;
    if ((r = pick(nxt, nslot, nups))) return r;
    // the next batch's uploads ride on this launch (their slots are free)
    cur.pf_count = 0;
    for (const Upload& u : nups) {
      CacheSlot& cs = o->slot[u.slot];
      cur.pf_src[cur.pf_count] = static_cast<const uint4*>(o->dom[u.domain].dpinned);
      cur.pf_dst[cur.pf_count] = static_cast<uint4*>(cs.dmem);
      cur.pf_n16[cur.pf_count] = uint32_t(o->dom[u.domain].nbytes / 16);
      ++cur.pf_count;
    }
    const int ring = int(o->launches++ % spray_rt_ooc::kRing);
    if (trace) {
      std::fprintf(stderr, "  launch %u:", S.launch);
      for (int k = 0; k < cur.count; ++k)
        std::fprintf(stderr, " d%d q%u live%u score%llu", cur.d[k].domain, cur.n[k],
                     live[cur.d[k].domain], o->score[cur.d[k].domain]);
      std::fprintf(stderr, " (+%d prefetched)\n", cur.pf_count);
    }
    HIPCHK(c, launch(s, cur, S));
    HIPCHK(c, hipEventRecord(o->launch_ev[ring], s));
    if (nxt.count == 0) {  // slots all held by this batch (small caches): pick
      std::fill(busy.begin(), busy.end(), 0);  // again, upload after the launch
      if ((r = pick(nxt, nslot, nups))) return r;
      for (const Upload& u : nups)
        if ((r = dma(u))) return r;
    }
    o->drains += cur.count;
    rings[S.launch % 4] = ring;
    // launch k's counts are published by launch k + 1 (its block 0)
    if (S.launch >= uint32_t(lag) &&
        (r = absorb(S.launch - uint32_t(lag), rings[(S.launch - lag + 1) % 4])))
      return r;
    ++S.launch;
    cur = nxt;
    std::copy(nslot, nslot + kOocBatch, cslot);
  }
  return SPRAY_RT_OK;
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
  // fine-grained: device stores reach the host while kernels run
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&o->snap), 257 * sizeof(unsigned long long),
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) std::memset(o->snap, 0, 257 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&o->done), sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(o->done, 0, sizeof(uint32_t));
  for (int k = 0; k < spray_rt_ooc::kRing && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&o->launch_ev[k], hipEventDisableTiming);
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
  }
  for (HostDomain& d : o->dom)
    if (d.pinned) (void)hipHostFree(d.pinned);
  free_scratch(o);
  if (o->tie) (void)hipFree(o->tie);
  if (o->rec) (void)hipFree(o->rec);
  if (o->snap) (void)hipHostFree(o->snap);
  if (o->done) (void)hipFree(o->done);
  for (hipEvent_t ev : o->launch_ev)
    if (ev) (void)hipEventDestroy(ev);
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
  const size_t padded = (img.bytes.size() + 15) / 16 * 16;
  HIPCHK(c, hipHostMalloc(&hd.pinned, padded, hipHostMallocMapped));
  std::memcpy(hd.pinned, img.bytes.data(), img.bytes.size());
  std::memset(static_cast<char*>(hd.pinned) + img.bytes.size(), 0, padded - img.bytes.size());
  HIPCHK(c, hipHostGetDevicePointer(&hd.dpinned, hd.pinned, 0));
  hd.nbytes = padded;
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
  // the drains' hit records: one 48-B slot per (ray, batch position)
  const int per = batch_per(o);
  const size_t rec_bytes = M * size_t(per) * 48;
  if (o->rec_cap < rec_bytes) {
    if (o->rec) HIPCHK(c, hipFree(o->rec));
    o->rec = nullptr;
    o->rec_cap = 0;
    HIPCHK(c, hipMalloc(&o->rec, rec_bytes));
    o->rec_cap = rec_bytes;
  }
  uint64_t* key = o->tie;
  if ((r = build_queues(o, rays, nullptr, M, key, nullptr))) return r;
  o->q.rec = static_cast<uint4*>(o->rec);
  o->q.rec_per = per;
  const int W = c->ndom <= 64 ? 1 : 4;
  r = drain(o, false, boxes, [&](hipStream_t s, const OocBatch& B, const OocSnapshot& S) {
    return launch_ooc_ch_batch(s, B, W, rays, o->q, c->d_boxes, key, hits, S);
  });
  if (r) return r;
  HIPCHK(c, launch_ooc_finish(stream_of(c), key, o->q, hits, M));
  return SPRAY_RT_OK;
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
  if ((r = build_queues(o, rays, valid, M, nullptr, occluded))) return r;
  const int W = c->ndom <= 64 ? 1 : 4;
  return drain(o, true, boxes, [&](hipStream_t s, const OocBatch& B, const OocSnapshot& S) {
    return launch_ooc_ah_batch(s, B, W, rays, o->q, occluded, S, c->coherence);
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
