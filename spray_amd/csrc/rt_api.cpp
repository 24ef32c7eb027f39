// rt_api.cpp -- C ABI of the engine (include/spray_rt.h).
//
// Owns the per-slot device images (BVH, triangles, epilogue arrays), the
// slot descriptor table, the domain boxes / domain->slot map of the scene
// path, and staging for host-pointer streams.  No exception crosses the
// boundary: every entry point returns a status and records a message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "bvh_build.h"
#include "rt_common.h"
#include "rt_ctx.h"
#include "rt_kernels.h"
#include "spray_rt.h"

using namespace spray_rt;

using namespace spray_rt::detail;

// Masked any hit: 0 = traced in place under the mask, 1 = compacted first
// into an ascending index list (hipCUB select) -- diagnostic builds compare.
#ifndef SPRAY_MASKED_SELECT
#define SPRAY_MASKED_SELECT 1
#endif

namespace spray_rt {
namespace detail {

int fail(spray_rt_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

hipStream_t stream_of(spray_rt_ctx* c) {
  return c->user_stream_set ? c->user_stream : c->own_stream;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

int ensure(spray_rt_ctx* c, void** buf, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return SPRAY_RT_OK;
  if (*buf) HIPCHK(c, hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  size_t want = std::max(bytes, size_t(1) << 20);
  HIPCHK(c, hipMalloc(buf, want));
  *cap = want;
  return SPRAY_RT_OK;
}

const char* build_slot_image(const float* verts, size_t nverts, const uint32_t* faces,
                             size_t nfaces, const uint32_t* colors, const float* normals,
                             SlotImage* out, bool quantized) {
  if (nfaces >= (size_t(1) << 29)) return "mesh too large (>= 2^29 faces)";
  BvhImage img;
  if (!build_bvh(verts, nverts, faces, nfaces, &img)) return "face index out of range";
  for (size_t i = 0; i < img.prims.size(); ++i)  // v0, e1, e2 of every referenced face
    for (int k = 0; k < 9; ++k)
      if (!std::isfinite(img.tris[12 * i + k])) return "non-finite vertex coordinate";
  QGrid grid{};
  std::vector<QNode4> qn;
  int qstack = 0;  // <= kQ4Stack, which the any-hit launches provide
  if (quantized && !img.nodes.empty() && !quantize_nodes4(img.nodes, &grid, &qn, &qstack))
    return qstack > kQ4Stack ? "4-wide node collapse exceeds the any-hit walk's stack (kQ4Stack)"
                             : "vertex coordinates beyond the range of the quantized node grid";
  // QGrid at nodes - 32, QNode4 i at nodes - 64 - 64 (i + 1) (rt_common.h)
  const size_t b_q = qn.empty() ? 0 : align256(64 + qn.size() * sizeof(QNode4));
  const size_t b_nodes = align256(img.nodes.size() * sizeof(BvhNode));
  const size_t b_tris = align256(img.tris.size() * sizeof(float));
  const size_t b_prims = align256(img.prims.size() * sizeof(uint32_t));
  const size_t b_faces = align256(3 * nfaces * sizeof(uint32_t));
  const size_t b_colors = colors ? align256(nverts * sizeof(uint32_t)) : 0;
  const size_t b_normals = normals ? align256(3 * nverts * sizeof(float)) : 0;
  out->bytes.assign(
      std::max<size_t>(256, b_q + b_nodes + b_tris + b_prims + b_faces + b_colors + b_normals), 0);
  out->nbytes = out->bytes.size();
  char* host = out->bytes.data();
  size_t off = 0;
  auto put = [&](const void* src, size_t n, size_t padded) {
    if (n) std::memcpy(host + off, src, n);
    size_t o = off;
    off += padded;
    return o;
  };
  if (b_q) {
    std::memcpy(host + b_q - sizeof(QGrid), &grid, sizeof(QGrid));
    for (size_t i = 0; i < qn.size(); ++i)
      std::memcpy(host + b_q - 64 - (i + 1) * sizeof(QNode4), &qn[i], sizeof(QNode4));
    off = b_q;
  }
  out->o_nodes = put(img.nodes.data(), img.nodes.size() * sizeof(BvhNode), b_nodes);
  out->o_tris = put(img.tris.data(), img.tris.size() * sizeof(float), b_tris);
  out->o_prims = put(img.prims.data(), img.prims.size() * sizeof(uint32_t), b_prims);
  out->o_faces = put(faces, 3 * nfaces * sizeof(uint32_t), b_faces);
  out->o_colors = colors ? put(colors, nverts * sizeof(uint32_t), b_colors) : SIZE_MAX;
  out->o_normals = normals ? put(normals, 3 * nverts * sizeof(float), b_normals) : SIZE_MAX;
  out->nnodes = uint32_t(img.nodes.size());
  out->ntris = uint32_t(img.prims.size());
  out->nverts = uint32_t(nverts);
  out->depth = img.depth;
  return nullptr;
}

int upload_slot_image(spray_rt_ctx* c, int slot, const SlotImage& img, const void* pinned_src,
                      bool async) {
  if (slot < 0 || slot > 1 << 20) return fail(c, SPRAY_RT_ERR_ARG, "bad slot %d", slot);
  if (size_t(slot) >= c->slots.size()) c->slots.resize(slot + 1);
  SlotHost& sh = c->slots[slot];
  HIPCHK(c, hipSetDevice(c->device));
  // the previous image may still be read by queued work
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));
  if (sh.ready) HIPCHK(c, hipEventSynchronize(sh.ready));
  const size_t total = img.nbytes;
  if (!pinned_src && img.bytes.size() != total)
    return fail(c, SPRAY_RT_ERR_STATE, "slot image bytes released without a pinned copy");
  if (sh.bytes < total) {
    if (sh.dmem) HIPCHK(c, hipFree(sh.dmem));
    sh.dmem = nullptr;
    sh.bytes = 0;
    HIPCHK(c, hipMalloc(&sh.dmem, total));
    sh.bytes = total;
  }
  char* d = static_cast<char*>(sh.dmem);
  if (async || pinned_src) {  // from pinned memory, completion tracked by an event
    const void* src = pinned_src;
    if (!src) {  // staged through the slot's own pinned buffer
      if (sh.pinned_bytes < total) {
        if (sh.pinned) HIPCHK(c, hipHostFree(sh.pinned));
        sh.pinned = nullptr;
        HIPCHK(c, hipHostMalloc(&sh.pinned, total, hipHostMallocDefault));
        sh.pinned_bytes = total;
      }
      std::memcpy(sh.pinned, img.bytes.data(), total);
      src = sh.pinned;
    }
    if (!sh.ready) HIPCHK(c, hipEventCreateWithFlags(&sh.ready, hipEventDisableTiming));
    HIPCHK(c, hipMemcpyAsync(d, src, total, hipMemcpyHostToDevice, c->upload_stream));
    HIPCHK(c, hipEventRecord(sh.ready, c->upload_stream));
  } else {
    HIPCHK(c, hipMemcpy(d, img.bytes.data(), total, hipMemcpyHostToDevice));
  }
  sh.desc = img.desc_at(d);
  sh.depth = img.depth;
  c->slots_dirty = true;
  return SPRAY_RT_OK;
}

SlotDesc SlotImage::desc_at(const void* base) const {
  const char* d = static_cast<const char*>(base);
  SlotDesc s{};
  s.nodes = reinterpret_cast<const BvhNode*>(d + o_nodes);
  s.tris = reinterpret_cast<const float*>(d + o_tris);
  s.prims = reinterpret_cast<const uint32_t*>(d + o_prims);
  s.faces = reinterpret_cast<const uint32_t*>(d + o_faces);
  s.colors = o_colors == SIZE_MAX ? nullptr : reinterpret_cast<const uint32_t*>(d + o_colors);
  s.normals = o_normals == SIZE_MAX ? nullptr : reinterpret_cast<const float*>(d + o_normals);
  s.ntris = ntris;
  s.nverts = nverts;
  s.nnodes = nnodes;
  return s;
}

}  // namespace detail
}  // namespace spray_rt

namespace {

// Makes pending async uploads visible to the compute stream and pushes the
// slot table / domain map when they changed.
int prepare(spray_rt_ctx* c) {
  hipStream_t s = stream_of(c);
  for (SlotHost& sh : c->slots)
    if (sh.ready) HIPCHK(c, hipStreamWaitEvent(s, sh.ready, 0));
  const bool trav_dirty = c->slots_dirty || c->dom_dirty;
  if (c->slots_dirty) {
    size_t n = std::max<size_t>(c->slots.size(), 1);
    if (c->d_slots_cap < n) {
      if (c->d_slots) HIPCHK(c, hipFree(c->d_slots));
      HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_slots),
                          n * sizeof(SlotDesc)));
      c->d_slots_cap = n;
    }
    std::vector<SlotDesc> h(n);
    for (size_t i = 0; i < c->slots.size(); ++i) h[i] = c->slots[i].desc;
    HIPCHK(c, hipMemcpyAsync(c->d_slots, h.data(), n * sizeof(SlotDesc),
                             hipMemcpyHostToDevice, s));
    HIPCHK(c, hipStreamSynchronize(s));  // h goes out of scope
    c->slots_dirty = false;
  }
  if (c->dom_dirty && c->ndom > 0) {
    HIPCHK(c, hipMemcpyAsync(c->d_dom2slot, c->dom2slot.data(),
                             c->ndom * sizeof(int), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->dom_dirty = false;
  }
  if (trav_dirty && c->ndom > 0) {
    std::vector<DomTrav> t(c->ndom);
    for (int d = 0; d < c->ndom; ++d) {
      const int slot = c->dom2slot[d];
      t[d] = DomTrav{nullptr, 0, 0};
      if (slot < 0 || size_t(slot) >= c->slots.size()) continue;
      const SlotDesc& sd = c->slots[slot].desc;
      if (!sd.nnodes) continue;
      const char* base = reinterpret_cast<const char*>(sd.nodes);
      t[d].nodes = sd.nodes;
      t[d].tri_off = uint32_t(reinterpret_cast<const char*>(sd.tris) - base);
      t[d].prim_off = uint32_t(reinterpret_cast<const char*>(sd.prims) - base);
    }
    HIPCHK(c, hipMemcpyAsync(c->d_domtrav, t.data(), c->ndom * sizeof(DomTrav),
                             hipMemcpyHostToDevice, s));
    HIPCHK(c, hipStreamSynchronize(s));
  }
  return SPRAY_RT_OK;
}

int check_slot(spray_rt_ctx* c, int slot) {
  if (slot < 0 || size_t(slot) >= c->slots.size() || !c->slots[slot].dmem)
    return fail(c, SPRAY_RT_ERR_ARG, "slot %d is not loaded", slot);
  return SPRAY_RT_OK;
}

int upload_segments(spray_rt_ctx* c, const int* slots, const size_t* offsets,
                    int nseg) {
  if (size_t(nseg) > c->seg_cap) {
    if (c->d_seg_slot) HIPCHK(c, hipFree(c->d_seg_slot));
    if (c->d_seg_off) HIPCHK(c, hipFree(c->d_seg_off));
    size_t cap = std::max<size_t>(nseg, 64);
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_seg_slot), cap * sizeof(int)));
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_seg_off),
                        (cap + 1) * sizeof(size_t)));
    c->seg_cap = cap;
  }
  hipStream_t s = stream_of(c);
  HIPCHK(c, hipMemcpyAsync(c->d_seg_slot, slots, nseg * sizeof(int),
                           hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(c->d_seg_off, offsets, (nseg + 1) * sizeof(size_t),
                           hipMemcpyHostToDevice, s));
  HIPCHK(c, hipStreamSynchronize(s));  // caller's host arrays may go away
  return SPRAY_RT_OK;
}

// Runs a per-slot stream kernel over (possibly host-resident) AoS records.
template <typename Launch>
int run_rtc(spray_rt_ctx* c, const int* slots, const size_t* offsets, int nseg,
            void* rays, size_t stride, Launch launch) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (nseg <= 0 || !slots || !offsets)
    return fail(c, SPRAY_RT_ERR_ARG, "empty segment list");
  if (stride < 80 || (stride & 3))
    return fail(c, SPRAY_RT_ERR_ARG, "stride %zu too small or unaligned", stride);
  size_t M = offsets[nseg];
  if (offsets[0] != 0) return fail(c, SPRAY_RT_ERR_ARG, "offsets[0] must be 0");
  for (int i = 0; i < nseg; ++i) {
    if (offsets[i + 1] < offsets[i])
      return fail(c, SPRAY_RT_ERR_ARG, "offsets not ascending");
    if (offsets[i + 1] > offsets[i]) {
      int r = check_slot(c, slots[i]);
      if (r) return r;
    }
  }
  if (M == 0) return SPRAY_RT_OK;
  if (!rays) return fail(c, SPRAY_RT_ERR_ARG, "null ray buffer");
  int r = prepare(c);
  if (r) return r;
  r = upload_segments(c, slots, offsets, nseg);
  if (r) return r;
  hipStream_t s = stream_of(c);
  if (is_device_ptr(rays)) {
    HIPCHK(c, launch(s, c->d_slots, c->d_seg_slot, c->d_seg_off, nseg,
                     static_cast<char*>(rays), stride, M));
    return SPRAY_RT_OK;
  }
  size_t bytes = M * stride;
  r = ensure(c, &c->d_stage, &c->stage_cap, bytes);
  if (r) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_stage, rays, bytes, hipMemcpyHostToDevice, s));
  HIPCHK(c, launch(s, c->d_slots, c->d_seg_slot, c->d_seg_off, nseg,
                   static_cast<char*>(c->d_stage), stride, M));
  HIPCHK(c, hipMemcpyAsync(rays, c->d_stage, bytes, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

}  // namespace

int spray_rt::detail::scene_common(spray_rt_ctx* c, const void* rays, size_t M,
                                   const void* out) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (c->ndom <= 0) return fail(c, SPRAY_RT_ERR_STATE, "no domain bounds set");
  if (c->ndom > SPRAY_RT_MAX_SCENE_DOMAINS)
    return fail(c, SPRAY_RT_ERR_LIMIT, "scene path supports <= %d domains",
                SPRAY_RT_MAX_SCENE_DOMAINS);
  if (M && (!rays || !out)) return fail(c, SPRAY_RT_ERR_ARG, "null buffer");
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->d_heads)
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_heads), 2 * kHeadsBytes));
  return prepare(c);
}

// The kernels' view of the resident scene; max_depth picks the traversal
// stack size (the LDS footprint, hence the occupancy) of the launch.
SceneView spray_rt::detail::view(const spray_rt_ctx* c) {
  int depth = c->tlas_depth;
  for (const SlotHost& sh : c->slots)
    if (sh.dmem) depth = std::max(depth, sh.depth);
  return SceneView{c->d_slots, c->d_dom2slot, c->d_domtrav, c->d_boxes, c->ndom,
                   c->d_tlas,  c->ntlas,      c->d_heads,   depth,        c->coherence};
}

extern "C" {

int spray_rt_create(int hip_device, spray_rt_ctx_t* out) {
  if (!out) return SPRAY_RT_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    (void)hipGetLastError();
    return SPRAY_RT_ERR_HIP;
  }
  if (hip_device < 0 || hip_device >= n) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = new (std::nothrow) spray_rt_ctx;
  if (!c) return SPRAY_RT_ERR_NOMEM;
  c->device = hip_device;
  if (hipSetDevice(hip_device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->upload_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SPRAY_RT_ERR_HIP;
  }
  *out = c;
  return SPRAY_RT_OK;
}

int spray_rt_destroy(spray_rt_ctx_t c) {
  if (!c) return SPRAY_RT_ERR_ARG;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  for (SlotHost& s : c->slots) {
    if (s.dmem) (void)hipFree(s.dmem);
    if (s.ready) (void)hipEventDestroy(s.ready);
    if (s.pinned) (void)hipHostFree(s.pinned);
  }
  void* bufs[] = {c->d_slots, c->d_boxes, c->d_dom2slot, c->d_domtrav, c->d_owner, c->d_tlas, c->d_seg_slot,
                  c->d_seg_off, c->d_stage, c->d_stage2, c->d_stage3,
                  c->d_block_counts, c->d_heads, c->d_sel, c->d_bsdf, c->d_frame, c->d_fstats, c->d_ftab};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->upload_stream) (void)hipStreamDestroy(c->upload_stream);
  delete c;
  return SPRAY_RT_OK;
}

const char* spray_rt_last_error(spray_rt_ctx_t c) {
  return c ? c->err.c_str() : "null context";
}

int spray_rt_set_stream(spray_rt_ctx_t c, void* hip_stream) {
  if (!c) return SPRAY_RT_ERR_ARG;
  c->user_stream = static_cast<hipStream_t>(hip_stream);
  c->user_stream_set = true;
  return SPRAY_RT_OK;
}

int spray_rt_sync(spray_rt_ctx_t c) {
  if (!c) return SPRAY_RT_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));
  return SPRAY_RT_OK;
}

int spray_rt_domain_upload(spray_rt_ctx_t c, int slot, const float* verts,
                           size_t nverts, const uint32_t* faces, size_t nfaces,
                           const uint32_t* colors, const float* normals,
                           int async) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (slot < 0 || slot > 1 << 20)
    return fail(c, SPRAY_RT_ERR_ARG, "bad slot %d", slot);
  if ((nverts && !verts) || (nfaces && !faces))
    return fail(c, SPRAY_RT_ERR_ARG, "null mesh arrays");
  SlotImage img;
  if (const char* why = build_slot_image(verts, nverts, faces, nfaces, colors, normals, &img))
    return fail(c, SPRAY_RT_ERR_ARG, "domain upload (slot %d): %s", slot, why);
  return upload_slot_image(c, slot, img, nullptr, async != 0);
}

int spray_rt_bvh_build_host(const float* verts, size_t nverts,
                            const uint32_t* faces, size_t nfaces,
                            size_t* nnodes, int* depth, void* nodes_out,
                            float* tris_out, uint32_t* prims_out) {
  if ((nverts && !verts) || (nfaces && !faces)) return SPRAY_RT_ERR_ARG;
  BvhImage img;
  if (!build_bvh(verts, nverts, faces, nfaces, &img)) return SPRAY_RT_ERR_ARG;
  if (nnodes) *nnodes = img.nodes.size();
  if (depth) *depth = img.depth;
  if (nodes_out)
    std::memcpy(nodes_out, img.nodes.data(), img.nodes.size() * sizeof(BvhNode));
  if (tris_out) std::memcpy(tris_out, img.tris.data(), img.tris.size() * sizeof(float));
  if (prims_out)
    std::memcpy(prims_out, img.prims.data(), img.prims.size() * sizeof(uint32_t));
  return SPRAY_RT_OK;
}

int spray_rt_qnodes_host(const float* verts, size_t nverts, const uint32_t* faces,
                         size_t nfaces, size_t* nnodes, float grid_out[6], void* qnodes_out) {
  if ((nverts && !verts) || (nfaces && !faces)) return SPRAY_RT_ERR_ARG;
  BvhImage img;
  if (!build_bvh(verts, nverts, faces, nfaces, &img)) return SPRAY_RT_ERR_ARG;
  QGrid grid{};
  std::vector<QNode> qn;
  if (!img.nodes.empty() && !quantize_nodes(img.nodes, &grid, &qn)) return SPRAY_RT_ERR_LIMIT;
  if (nnodes) *nnodes = qn.size();
  if (grid_out) {
    std::memcpy(grid_out, grid.base, 12);
    std::memcpy(grid_out + 3, grid.scale, 12);
  }
  if (qnodes_out) std::memcpy(qnodes_out, qn.data(), qn.size() * sizeof(QNode));
  return SPRAY_RT_OK;
}

int spray_rt_qnodes4_host(const float* verts, size_t nverts, const uint32_t* faces,
                          size_t nfaces, size_t* nnodes, int* stack_bound, float grid_out[6],
                          void* qnodes_out) {
  if ((nverts && !verts) || (nfaces && !faces)) return SPRAY_RT_ERR_ARG;
  BvhImage img;
  if (!build_bvh(verts, nverts, faces, nfaces, &img)) return SPRAY_RT_ERR_ARG;
  QGrid grid{};
  std::vector<QNode4> qn;
  int bound = 0;
  if (!img.nodes.empty() && !quantize_nodes4(img.nodes, &grid, &qn, &bound))
    return SPRAY_RT_ERR_LIMIT;
  if (nnodes) *nnodes = qn.size();
  if (stack_bound) *stack_bound = bound;
  if (grid_out) {
    std::memcpy(grid_out, grid.base, 12);
    std::memcpy(grid_out + 3, grid.scale, 12);
  }
  if (qnodes_out) std::memcpy(qnodes_out, qn.data(), qn.size() * sizeof(QNode4));
  return SPRAY_RT_OK;
}

int spray_rt_domain_release(spray_rt_ctx_t c, int slot) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (slot < 0 || size_t(slot) >= c->slots.size())
    return fail(c, SPRAY_RT_ERR_ARG, "bad slot %d", slot);
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));
  SlotHost& sh = c->slots[slot];
  if (sh.ready) HIPCHK(c, hipEventSynchronize(sh.ready));
  if (sh.dmem) HIPCHK(c, hipFree(sh.dmem));
  sh.dmem = nullptr;
  sh.bytes = 0;
  sh.desc = SlotDesc{};
  c->slots_dirty = true;
  return SPRAY_RT_OK;
}

int spray_rt_slot_info(spray_rt_ctx_t c, int slot, size_t* nnodes, int* depth,
                       size_t* ntris) {
  if (!c) return SPRAY_RT_ERR_ARG;
  int r = check_slot(c, slot);
  if (r) return r;
  const SlotHost& sh = c->slots[slot];
  if (nnodes) *nnodes = sh.desc.nnodes;
  if (depth) *depth = sh.depth;
  if (ntris) *ntris = sh.desc.ntris;
  return SPRAY_RT_OK;
}

int spray_rt_domain_bounds(spray_rt_ctx_t c, int ndomains, const float* boxes) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (ndomains < 0 || (ndomains && !boxes))
    return fail(c, SPRAY_RT_ERR_ARG, "bad domain bounds");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));
  if (c->d_boxes) HIPCHK(c, hipFree(c->d_boxes));
  if (c->d_dom2slot) HIPCHK(c, hipFree(c->d_dom2slot));
  if (c->d_domtrav) HIPCHK(c, hipFree(c->d_domtrav));
  if (c->d_owner) HIPCHK(c, hipFree(c->d_owner));
  if (c->d_tlas) HIPCHK(c, hipFree(c->d_tlas));
  c->d_boxes = nullptr;
  c->d_dom2slot = nullptr;
  c->d_domtrav = nullptr;
  c->d_owner = nullptr;
  c->h_owner.clear();
  c->d_tlas = nullptr;
  c->ntlas = 0;
  c->tlas_depth = 0;
  c->ndom = ndomains;
  c->h_boxes.assign(boxes, boxes + 6 * size_t(ndomains));
  c->dom2slot.assign(ndomains, -1);
  c->dom_dirty = true;
  if (ndomains == 0) return SPRAY_RT_OK;
  HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_boxes), 6 * ndomains * sizeof(float)));
  HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_dom2slot), ndomains * sizeof(int)));
  HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_domtrav), ndomains * sizeof(DomTrav)));
  HIPCHK(c, hipMemcpy(c->d_boxes, boxes, 6 * ndomains * sizeof(float),
                      hipMemcpyHostToDevice));
  std::vector<BvhNode> tlas;
  int depth = 0;
  if (!build_domain_tree(boxes, size_t(ndomains), &tlas, &depth))
    return fail(c, SPRAY_RT_ERR_LIMIT, "too many domains");
  if (ndomains <= SPRAY_RT_MAX_SCENE_DOMAINS) {  // scene path stages it in LDS
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_tlas), tlas.size() * sizeof(BvhNode)));
    HIPCHK(c, hipMemcpy(c->d_tlas, tlas.data(), tlas.size() * sizeof(BvhNode),
                        hipMemcpyHostToDevice));
    c->ntlas = int(tlas.size());
    c->tlas_depth = depth;
  }
  return SPRAY_RT_OK;
}

int spray_rt_map_domain(spray_rt_ctx_t c, int domain_id, int slot) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (domain_id < 0 || domain_id >= c->ndom)
    return fail(c, SPRAY_RT_ERR_ARG, "domain %d out of range", domain_id);
  if (slot >= 0) {
    int r = check_slot(c, slot);
    if (r) return r;
  }
  c->dom2slot[domain_id] = slot < 0 ? -1 : slot;
  c->dom_dirty = true;
  return SPRAY_RT_OK;
}

int spray_rt_intersect1M(spray_rt_ctx_t c, int slot, void* rays, size_t M,
                         size_t stride) {
  size_t off[2] = {0, M};
  return run_rtc(c, &slot, off, 1, rays, stride, launch_rtc_intersect);
}

int spray_rt_occluded1M(spray_rt_ctx_t c, int slot, void* rays, size_t M,
                        size_t stride) {
  size_t off[2] = {0, M};
  return run_rtc(c, &slot, off, 1, rays, stride, launch_rtc_occluded);
}

int spray_rt_update_intersection1M(spray_rt_ctx_t c, int slot, void* rays, size_t M,
                                   size_t stride) {
  if (c && stride < sizeof(spray_rt_ray_intersection))
    return fail(c, SPRAY_RT_ERR_ARG, "stride %zu below the 96-B RTCRayIntersection", stride);
  size_t off[2] = {0, M};
  return run_rtc(c, &slot, off, 1, rays, stride, launch_rtc_update);
}

int spray_rt_intersect_segments(spray_rt_ctx_t c, const int* slots,
                                const size_t* offsets, int nseg, void* rays,
                                size_t stride) {
  return run_rtc(c, slots, offsets, nseg, rays, stride, launch_rtc_intersect);
}

int spray_rt_occluded_segments(spray_rt_ctx_t c, const int* slots,
                               const size_t* offsets, int nseg, void* rays,
                               size_t stride) {
  return run_rtc(c, slots, offsets, nseg, rays, stride, launch_rtc_occluded);
}

}  // extern "C"

// ---- lanes --------------------------------------------------------------
namespace {
int lane_fail(spray_rt_lane* L, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  L->err = buf;
  return code;
}
#define LCHK(L, expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return lane_fail(L, SPRAY_RT_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_e));   \
  } while (0)

int lane_buf(spray_rt_lane* L, size_t bytes) {
  if (L->cap >= bytes) return SPRAY_RT_OK;
  if (L->d_buf) LCHK(L, hipFree(L->d_buf));
  L->d_buf = nullptr;
  L->cap = 0;
  const size_t want = std::max<size_t>(bytes, size_t(1) << 16);
  LCHK(L, hipMalloc(&L->d_buf, want));
  L->cap = want;
  return SPRAY_RT_OK;
}

// the context's tables, rebuilt under its lock when a load made them stale
int lane_tables(spray_rt_lane* L) {
  spray_rt_ctx* c = L->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->slots_dirty && !c->dom_dirty) return SPRAY_RT_OK;
  const int r = prepare(c);
  if (r) return lane_fail(L, r, "%s", c->err.c_str());
  return SPRAY_RT_OK;
}

template <typename Launch>
int lane_rtc(spray_rt_lane* L, int slot, void* rays, size_t M, size_t stride, Launch launch) {
  if (!L) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = L->ctx;
  if (stride < 80 || (stride & 3)) return lane_fail(L, SPRAY_RT_ERR_ARG, "bad stride %zu", stride);
  if (M == 0) return SPRAY_RT_OK;
  if (!rays) return lane_fail(L, SPRAY_RT_ERR_ARG, "null ray buffer");
  {
    std::lock_guard<std::mutex> g(c->mu);
    if (slot < 0 || size_t(slot) >= c->slots.size() || !c->slots[slot].dmem)
      return lane_fail(L, SPRAY_RT_ERR_ARG, "slot %d is not loaded", slot);
  }
  LCHK(L, hipSetDevice(c->device));
  int r = lane_tables(L);
  if (r) return r;
  const size_t off[2] = {0, M};
  LCHK(L, hipMemcpyAsync(L->d_seg_slot, &slot, sizeof(int), hipMemcpyHostToDevice, L->stream));
  LCHK(L, hipMemcpyAsync(L->d_seg_off, off, sizeof(off), hipMemcpyHostToDevice, L->stream));
  if (is_device_ptr(rays)) {
    LCHK(L, launch(L->stream, c->d_slots, L->d_seg_slot, L->d_seg_off, 1, static_cast<char*>(rays),
                   stride, M));
    LCHK(L, hipStreamSynchronize(L->stream));
    return SPRAY_RT_OK;
  }
  const size_t bytes = M * stride;
  r = lane_buf(L, bytes);
  if (r) return r;
  LCHK(L, hipMemcpyAsync(L->d_buf, rays, bytes, hipMemcpyHostToDevice, L->stream));
  LCHK(L, launch(L->stream, c->d_slots, L->d_seg_slot, L->d_seg_off, 1,
                 static_cast<char*>(L->d_buf), stride, M));
  LCHK(L, hipMemcpyAsync(rays, L->d_buf, bytes, hipMemcpyDeviceToHost, L->stream));
  LCHK(L, hipStreamSynchronize(L->stream));
  return SPRAY_RT_OK;
}
}  // namespace

extern "C" {

// Lane creation runs on many host threads at once (one lane per thread,
// created on first use): its failures go to a thread-local message, never to
// the context's shared error string.
static thread_local std::string t_lane_create_err;

int spray_rt_lane_create(spray_rt_ctx_t c, spray_rt_lane_t* out) {
  if (!c || !out) {
    t_lane_create_err = "null context or output";
    return SPRAY_RT_ERR_ARG;
  }
  *out = nullptr;
  const hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) {
    t_lane_create_err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return SPRAY_RT_ERR_HIP;
  }
  spray_rt_lane* L = new (std::nothrow) spray_rt_lane;
  if (!L) {
    t_lane_create_err = "out of host memory";
    return SPRAY_RT_ERR_NOMEM;
  }
  L->ctx = c;
  if (hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&L->d_seg_slot), 256) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&L->d_seg_off), 256) != hipSuccess) {
    (void)hipGetLastError();
    spray_rt_lane_destroy(L);
    t_lane_create_err = "lane creation failed (stream or device buffers)";
    return SPRAY_RT_ERR_HIP;
  }
  t_lane_create_err.clear();
  *out = L;
  return SPRAY_RT_OK;
}

const char* spray_rt_lane_create_error(void) { return t_lane_create_err.c_str(); }

int spray_rt_lane_destroy(spray_rt_lane_t L) {
  if (!L) return SPRAY_RT_ERR_ARG;
  (void)hipSetDevice(L->ctx->device);
  if (L->stream) (void)hipStreamSynchronize(L->stream);
  if (L->d_buf) (void)hipFree(L->d_buf);
  if (L->d_seg_slot) (void)hipFree(L->d_seg_slot);
  if (L->d_seg_off) (void)hipFree(L->d_seg_off);
  if (L->stream) (void)hipStreamDestroy(L->stream);
  delete L;
  return SPRAY_RT_OK;
}

const char* spray_rt_lane_last_error(spray_rt_lane_t L) {
  return L ? L->err.c_str() : "null lane";
}

int spray_rt_lane_intersect1M(spray_rt_lane_t L, int slot, void* rays, size_t M, size_t stride) {
  return lane_rtc(L, slot, rays, M, stride, launch_rtc_intersect);
}

int spray_rt_lane_occluded1M(spray_rt_lane_t L, int slot, void* rays, size_t M, size_t stride) {
  return lane_rtc(L, slot, rays, M, stride, launch_rtc_occluded);
}

int spray_rt_lane_update_intersection1M(spray_rt_lane_t L, int slot, void* rays, size_t M,
                                        size_t stride) {
  if (L && stride < sizeof(spray_rt_ray_intersection))
    return lane_fail(L, SPRAY_RT_ERR_ARG, "stride %zu below the 96-B RTCRayIntersection", stride);
  return lane_rtc(L, slot, rays, M, stride, launch_rtc_update);
}

int spray_rt_lane_domains1M(spray_rt_lane_t L, const float* org, const float* dir, size_t M,
                            int* ids, float* ts, int* counts, int maxhits) {
  if (!L) return SPRAY_RT_ERR_ARG;
  spray_rt_ctx* c = L->ctx;
  if (maxhits <= 0) return lane_fail(L, SPRAY_RT_ERR_ARG, "maxhits must be > 0");
  if (c->ndom == 0) return lane_fail(L, SPRAY_RT_ERR_STATE, "no domain bounds set");
  if (M == 0) return SPRAY_RT_OK;
  if (!org || !dir || !ids || !ts || !counts) return lane_fail(L, SPRAY_RT_ERR_ARG, "null buffer");
  LCHK(L, hipSetDevice(c->device));
  int r = lane_tables(L);
  if (r) return r;
  if (is_device_ptr(org)) {
    LCHK(L, launch_domains(L->stream, c->d_boxes, c->ndom, org, dir, M, ids, ts, counts, maxhits));
    LCHK(L, hipStreamSynchronize(L->stream));
    return SPRAY_RT_OK;
  }
  const size_t b_in = align256(3 * M * sizeof(float));
  const size_t b_ids = align256(M * maxhits * sizeof(int));
  const size_t b_cnt = align256(M * sizeof(int));
  r = lane_buf(L, 2 * b_in + 2 * b_ids + b_cnt);
  if (r) return r;
  char* b = static_cast<char*>(L->d_buf);
  float* d_org = reinterpret_cast<float*>(b);
  float* d_dir = reinterpret_cast<float*>(b + b_in);
  int* d_ids = reinterpret_cast<int*>(b + 2 * b_in);
  float* d_ts = reinterpret_cast<float*>(b + 2 * b_in + b_ids);
  int* d_cnt = reinterpret_cast<int*>(b + 2 * b_in + 2 * b_ids);
  LCHK(L, hipMemcpyAsync(d_org, org, 3 * M * sizeof(float), hipMemcpyHostToDevice, L->stream));
  LCHK(L, hipMemcpyAsync(d_dir, dir, 3 * M * sizeof(float), hipMemcpyHostToDevice, L->stream));
  LCHK(L, launch_domains(L->stream, c->d_boxes, c->ndom, d_org, d_dir, M, d_ids, d_ts, d_cnt,
                         maxhits));
  LCHK(L, hipMemcpyAsync(ids, d_ids, M * maxhits * sizeof(int), hipMemcpyDeviceToHost, L->stream));
  LCHK(L, hipMemcpyAsync(ts, d_ts, M * maxhits * sizeof(float), hipMemcpyDeviceToHost, L->stream));
  LCHK(L, hipMemcpyAsync(counts, d_cnt, M * sizeof(int), hipMemcpyDeviceToHost, L->stream));
  LCHK(L, hipStreamSynchronize(L->stream));
  return SPRAY_RT_OK;
}

int spray_rt_domains1M(spray_rt_ctx_t c, const float* org, const float* dir,
                       size_t M, int* ids, float* ts, int* counts, int maxhits) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (maxhits <= 0) return fail(c, SPRAY_RT_ERR_ARG, "maxhits must be > 0");
  if (c->ndom == 0) return fail(c, SPRAY_RT_ERR_STATE, "no domain bounds set");
  if (M == 0) return SPRAY_RT_OK;
  if (!org || !dir || !ids || !ts || !counts)
    return fail(c, SPRAY_RT_ERR_ARG, "null buffer");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = stream_of(c);
  const bool dev = is_device_ptr(org);
  if (dev) {
    HIPCHK(c, launch_domains(s, c->d_boxes, c->ndom, org, dir, M, ids, ts,
                             counts, maxhits));
    return SPRAY_RT_OK;
  }
  const size_t b_in = 3 * M * sizeof(float);
  const size_t b_ids = M * maxhits * sizeof(int);
  const size_t b_cnt = M * sizeof(int);
  int r = ensure(c, &c->d_stage, &c->stage_cap, 2 * b_in);
  if (r) return r;
  r = ensure(c, &c->d_stage2, &c->stage2_cap, 2 * b_ids);
  if (r) return r;
  r = ensure(c, &c->d_stage3, &c->stage3_cap, b_cnt);
  if (r) return r;
  char* din = static_cast<char*>(c->d_stage);
  char* dout = static_cast<char*>(c->d_stage2);
  HIPCHK(c, hipMemcpyAsync(din, org, b_in, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(din + b_in, dir, b_in, hipMemcpyHostToDevice, s));
  HIPCHK(c, launch_domains(s, c->d_boxes, c->ndom, reinterpret_cast<float*>(din),
                           reinterpret_cast<float*>(din + b_in), M,
                           reinterpret_cast<int*>(dout),
                           reinterpret_cast<float*>(dout + b_ids),
                           static_cast<int*>(c->d_stage3), maxhits));
  HIPCHK(c, hipMemcpyAsync(ids, dout, b_ids, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(ts, dout + b_ids, b_ids, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipMemcpyAsync(counts, c->d_stage3, b_cnt, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

// counters: optional device uint64[3] (nodes, tris, visits); exported for the
// canonical-count tests and the bench's byte accounting cross-check.
extern "C" int spray_rt_intersect_scene_counted(spray_rt_ctx_t c,
                                                const spray_rt_ray* rays,
                                                size_t M, spray_rt_hit* hits,
                                                unsigned long long* d_counters) {
  int r = scene_common(c, rays, M, hits);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  hipStream_t s = stream_of(c);
  if (is_device_ptr(rays)) {
    HIPCHK(c, launch_scene_intersect(s, view(c), rays, M, hits, d_counters));
    return SPRAY_RT_OK;
  }
  r = ensure(c, &c->d_stage, &c->stage_cap, M * sizeof(spray_rt_ray));
  if (r) return r;
  r = ensure(c, &c->d_stage2, &c->stage2_cap, M * sizeof(spray_rt_hit));
  if (r) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_stage, rays, M * sizeof(spray_rt_ray),
                           hipMemcpyHostToDevice, s));
  HIPCHK(c, launch_scene_intersect(s, view(c), static_cast<spray_rt_ray*>(c->d_stage), M,
                                   static_cast<spray_rt_hit*>(c->d_stage2), d_counters));
  HIPCHK(c, hipMemcpyAsync(hits, c->d_stage2, M * sizeof(spray_rt_hit),
                           hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

extern "C" int spray_rt_occluded_scene_counted(spray_rt_ctx_t c,
                                               const spray_rt_ray* rays,
                                               size_t M, uint8_t* occ,
                                               unsigned long long* d_counters) {
  int r = scene_common(c, rays, M, occ);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  hipStream_t s = stream_of(c);
  if (is_device_ptr(rays)) {
    HIPCHK(c, launch_scene_occluded(s, view(c), rays, M, nullptr, occ, d_counters));
    return SPRAY_RT_OK;
  }
  r = ensure(c, &c->d_stage, &c->stage_cap, M * sizeof(spray_rt_ray));
  if (r) return r;
  r = ensure(c, &c->d_stage2, &c->stage2_cap, M);
  if (r) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_stage, rays, M * sizeof(spray_rt_ray),
                           hipMemcpyHostToDevice, s));
  HIPCHK(c, launch_scene_occluded(s, view(c), static_cast<spray_rt_ray*>(c->d_stage), M,
                                  nullptr, static_cast<uint8_t*>(c->d_stage2), d_counters));
  HIPCHK(c, hipMemcpyAsync(occ, c->d_stage2, M, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return SPRAY_RT_OK;
}

extern "C" int spray_rt_occluded_scene_devcount(spray_rt_ctx_t c,
                                                const spray_rt_ray* rays,
                                                size_t max_rays,
                                                const uint32_t* d_count,
                                                uint8_t* occ,
                                                unsigned long long* d_counters) {
  int r = scene_common(c, rays, max_rays, occ);
  if (r) return r;
  if (max_rays == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(rays) || !is_device_ptr(occ) || !is_device_ptr(d_count))
    return fail(c, SPRAY_RT_ERR_ARG, "devcount variant needs device buffers");
  HIPCHK(c, launch_scene_occluded(stream_of(c), view(c), rays, max_rays, d_count, occ,
                                  d_counters));
  return SPRAY_RT_OK;
}

extern "C" int spray_rt_occluded_scene_order(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                             size_t max_rays, const uint32_t* order,
                                             const uint32_t* d_count, uint8_t* occ) {
  int r = scene_common(c, rays, max_rays, occ);
  if (r) return r;
  if (max_rays == 0) return SPRAY_RT_OK;
  if (max_rays > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "max_rays > 2^32");
  if (!is_device_ptr(rays) || !is_device_ptr(occ) || (order && !is_device_ptr(order)) ||
      !is_device_ptr(d_count))
    return fail(c, SPRAY_RT_ERR_ARG, "ordered occlusion needs device buffers");
  HIPCHK(c, launch_scene_occluded_indexed(stream_of(c), view(c), rays, max_rays, order, d_count,
                                          occ, nullptr));
  return SPRAY_RT_OK;
}

int spray_rt_intersect_scene_spawn_pt(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                      size_t M, spray_rt_hit* hits,
                                      const float shade[10], spray_rt_ray* out_rays,
                                      uint8_t* out_valid, uint32_t* d_count) {
  int r = scene_common(c, rays, M, hits);
  if (r) return r;
  if (!shade) return fail(c, SPRAY_RT_ERR_ARG, "null shade parameters");
  if ((d_count && !is_device_ptr(d_count)) ||
      (M && (!is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(out_rays) ||
             !is_device_ptr(out_valid))))
    return fail(c, SPRAY_RT_ERR_ARG, "fused spawn needs device buffers");
  HIPCHK(c, launch_scene_intersect_pt(stream_of(c), view(c), rays, M, hits, shade,
                                      out_rays, out_valid, d_count));
  return SPRAY_RT_OK;
}

int spray_rt_intersect_scene_shadow_pt(spray_rt_ctx_t c, const spray_rt_ray* rays, size_t M,
                                       spray_rt_hit* hits, const float shade[10],
                                       uint8_t* occluded, uint8_t* sh_valid,
                                       uint32_t* d_count) {
  int r = scene_common(c, rays, M, hits);
  if (r) return r;
  if (!shade) return fail(c, SPRAY_RT_ERR_ARG, "null shade parameters");
  if (M > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "M > 2^32");
  if ((d_count && !is_device_ptr(d_count)) ||
      (M && (!is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(occluded) ||
             !is_device_ptr(sh_valid))))
    return fail(c, SPRAY_RT_ERR_ARG, "fused shadow tracing needs device buffers");
  HIPCHK(c, launch_scene_intersect_shadow_pt(stream_of(c), view(c), rays, M, hits, shade,
                                             occluded, sh_valid, d_count));
  return SPRAY_RT_OK;
}

int spray_rt_occluded_scene_masked(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                   size_t M, const uint8_t* valid, uint8_t* occ) {
  int r = scene_common(c, rays, M, occ);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  if (M > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "M > 2^32");
  if (!valid || !is_device_ptr(rays) || !is_device_ptr(occ) || !is_device_ptr(valid))
    return fail(c, SPRAY_RT_ERR_ARG, "masked occlusion needs device buffers");
  hipStream_t s = stream_of(c);
  if (!SPRAY_MASKED_SELECT) {
    HIPCHK(c, launch_scene_occluded_masked(s, view(c), rays, M, valid, occ));
    return SPRAY_RT_OK;
  }
  size_t temp = 0;
  HIPCHK(c, launch_select_flagged(s, valid, M, nullptr, nullptr, nullptr, &temp));
  const size_t b_idx = align256(M * sizeof(uint32_t));
  r = ensure(c, &c->d_sel, &c->sel_cap, b_idx + 256 + temp);
  if (r) return r;
  char* base = static_cast<char*>(c->d_sel);
  uint32_t* idx = reinterpret_cast<uint32_t*>(base);
  uint32_t* num = reinterpret_cast<uint32_t*>(base + b_idx);
  HIPCHK(c, launch_select_flagged(s, valid, M, idx, num, base + b_idx + 256, &temp));
  HIPCHK(c, launch_scene_occluded_indexed(s, view(c), rays, M, idx, num, occ, nullptr));
  return SPRAY_RT_OK;
}

int spray_rt_intersect_scene(spray_rt_ctx_t c, const spray_rt_ray* rays,
                             size_t M, spray_rt_hit* hits) {
  return spray_rt_intersect_scene_counted(c, rays, M, hits, nullptr);
}

int spray_rt_occluded_scene(spray_rt_ctx_t c, const spray_rt_ray* rays,
                            size_t M, uint8_t* occluded) {
  return spray_rt_occluded_scene_counted(c, rays, M, occluded, nullptr);
}

int spray_rt_set_coherence(spray_rt_ctx_t c, int mode) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (mode != SPRAY_RT_RAYS_ADAPTIVE && mode != SPRAY_RT_RAYS_COHERENT &&
      mode != SPRAY_RT_RAYS_INCOHERENT)
    return fail(c, SPRAY_RT_ERR_ARG, "bad coherence mode %d", mode);
  c->coherence = mode;
  return SPRAY_RT_OK;
}

int spray_rt_exchange_plan(spray_rt_ctx_t c, const uint64_t* rank_mask, size_t n,
                           int world, int64_t* idx, int64_t* starts) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (world <= 0 || world > 64) return fail(c, SPRAY_RT_ERR_ARG, "world must be in [1, 64]");
  if (n > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "n > 2^32");
  if (!is_device_ptr(starts) || (n && !is_device_ptr(rank_mask)) ||
      (idx && !is_device_ptr(idx)))
    return fail(c, SPRAY_RT_ERR_ARG, "exchange plan needs device buffers");
  HIPCHK(c, hipSetDevice(c->device));
  int r = ensure(c, &c->d_sel, &c->sel_cap, plan_temp_bytes(n, world));
  if (r) return r;
  HIPCHK(c, launch_plan(stream_of(c), rank_mask, n, world, idx, starts, c->d_sel));
  return SPRAY_RT_OK;
}

int spray_rt_gather_rows(spray_rt_ctx_t c, const void* src, size_t row_bytes,
                         const int64_t* idx, size_t n, void* dst) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (row_bytes != 4 && row_bytes != 8 && row_bytes != 16 && row_bytes != 32 &&
      row_bytes != 48)
    return fail(c, SPRAY_RT_ERR_ARG, "row size %zu not supported", row_bytes);
  if (n == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(src) || !is_device_ptr(idx) || !is_device_ptr(dst))
    return fail(c, SPRAY_RT_ERR_ARG, "gather needs device buffers");
  if (row_bytes % 16 == 0 &&
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
    return fail(c, SPRAY_RT_ERR_ARG, "16-B rows need 16-B aligned buffers");
  HIPCHK(c, launch_gather_rows(stream_of(c), src, row_bytes, idx, n, dst));
  return SPRAY_RT_OK;
}

int spray_rt_set_owners(spray_rt_ctx_t c, const int* owner) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (c->ndom <= 0) return fail(c, SPRAY_RT_ERR_STATE, "no domain bounds set");
  if (!owner) return fail(c, SPRAY_RT_ERR_ARG, "null owner map");
  for (int d = 0; d < c->ndom; ++d)
    if (owner[d] < -1 || owner[d] >= 64)
      return fail(c, SPRAY_RT_ERR_ARG, "owner[%d] = %d out of [-1, 64)", d, owner[d]);
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->d_owner)
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_owner), c->ndom * sizeof(int)));
  hipStream_t s = stream_of(c);
  HIPCHK(c, hipMemcpyAsync(c->d_owner, owner, c->ndom * sizeof(int), hipMemcpyHostToDevice, s));
  HIPCHK(c, hipStreamSynchronize(s));
  c->h_owner.assign(owner, owner + c->ndom);
  return SPRAY_RT_OK;
}

int spray_rt_route(spray_rt_ctx_t c, const spray_rt_ray* rays, size_t M,
                   uint64_t* rank_mask) {
  int r = scene_common(c, rays, M, rank_mask);
  if (r) return r;
  if (!c->d_owner) return fail(c, SPRAY_RT_ERR_STATE, "no owner map set");
  if (M == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(rays) || !is_device_ptr(rank_mask))
    return fail(c, SPRAY_RT_ERR_ARG, "route needs device buffers");
  HIPCHK(c, launch_route(stream_of(c), view(c), c->d_owner, rays, M, rank_mask));
  return SPRAY_RT_OK;
}

int spray_rt_intersect_scene_keyed(spray_rt_ctx_t c, const spray_rt_ray* rays, size_t M,
                                   spray_rt_hit* hits, uint64_t* keys) {
  int r = scene_common(c, rays, M, hits);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  if (!keys || !is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(keys))
    return fail(c, SPRAY_RT_ERR_ARG, "keyed intersect needs device buffers");
  HIPCHK(c, launch_scene_intersect_keyed(stream_of(c), view(c), rays, M, hits, keys));
  return SPRAY_RT_OK;
}

int spray_rt_eye_rays_insitu(spray_rt_ctx_t c, const float cam[14], int image_w, int spp,
                             int bx, int by, int bw, int bh, int tx, int ty, int tw, int th,
                             spray_rt_ray* rays, int32_t* pixid, int32_t* samid) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!cam || spp <= 0 || tw < 0 || th < 0 || bw <= 0 || bh <= 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad eye-ray arguments");
  if (tw && th && (tx < bx || ty < by || tx + tw > bx + bw || ty + th > by + bh))
    return fail(c, SPRAY_RT_ERR_ARG, "stripe outside its blocking tile");
  if (size_t(tw) * th * spp == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(rays) || (pixid && !is_device_ptr(pixid)) ||
      (samid && !is_device_ptr(samid)))
    return fail(c, SPRAY_RT_ERR_ARG, "eye-ray buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, launch_eye_rays_insitu(stream_of(c), cam, image_w, spp, bx, by, bw, tx, ty, tw,
                                   th, rays, pixid, samid));
  return SPRAY_RT_OK;
}

int spray_rt_eye_rays_ooc(spray_rt_ctx_t c, const float cam[14], int image_w,
                          int spp, int tx, int ty, int tw, int th,
                          spray_rt_ray* rays, int32_t* pixid, int32_t* samid) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!cam || spp <= 0 || tw < 0 || th < 0)
    return fail(c, SPRAY_RT_ERR_ARG, "bad eye-ray arguments");
  if (size_t(tw) * th * spp == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(rays) || (pixid && !is_device_ptr(pixid)) ||
      (samid && !is_device_ptr(samid)))
    return fail(c, SPRAY_RT_ERR_ARG, "eye-ray buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, launch_eye_rays_ooc(stream_of(c), cam, image_w, spp, tx, ty, tw, th,
                                rays, pixid, samid));
  return SPRAY_RT_OK;
}

int spray_rt_spawn_shadows_pt(spray_rt_ctx_t c, const spray_rt_ray* rays,
                              const spray_rt_hit* hits, size_t M,
                              const float shade[10], spray_rt_ray* out_rays,
                              int32_t* out_src, uint32_t* d_count) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!shade || !d_count) return fail(c, SPRAY_RT_ERR_ARG, "null argument");
  if (M && (!is_device_ptr(rays) || !is_device_ptr(hits) ||
            !is_device_ptr(out_rays) || !is_device_ptr(d_count)))
    return fail(c, SPRAY_RT_ERR_ARG, "spawn buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  size_t nb = (M + kBlock - 1) / kBlock + 1;
  void* bc = c->d_block_counts;
  int r = ensure(c, &bc, &c->block_cap, nb * sizeof(unsigned long long));
  if (r) return r;
  c->d_block_counts = static_cast<uint32_t*>(bc);
  HIPCHK(c, launch_spawn_pt(stream_of(c), rays, hits, M, shade, out_rays,
                            out_src, d_count, c->d_block_counts));
  return SPRAY_RT_OK;
}

namespace {
int spawn_ao(spray_rt_ctx_t c, const spray_rt_ray* rays, const spray_rt_hit* hits,
             const int32_t* pixid, size_t M, int nsamples, spray_rt_ray* out_rays,
             int32_t* out_src, uint32_t* d_count, uint32_t* trace_order, bool traced) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!d_count || nsamples <= 0 || nsamples > 1024)
    return fail(c, SPRAY_RT_ERR_ARG, "bad AO arguments");
  if (M * size_t(nsamples) > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "too many rays");
  if (M && (!is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(pixid) ||
            !is_device_ptr(out_rays) || !is_device_ptr(d_count) ||
            (trace_order && !is_device_ptr(trace_order))))
    return fail(c, SPRAY_RT_ERR_ARG, "spawn buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  void* bc = c->d_block_counts;
  int r = ensure(c, &bc, &c->block_cap, ao_scratch_bytes(M, nsamples));
  if (r) return r;
  c->d_block_counts = static_cast<uint32_t*>(bc);
  HIPCHK(c, launch_spawn_ao(stream_of(c), rays, hits, pixid, M, nsamples, out_rays, out_src,
                            d_count, c->d_block_counts, trace_order, traced));
  return SPRAY_RT_OK;
}
}  // namespace

int spray_rt_spawn_shadows_ao_ordered(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                      const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                      int nsamples, spray_rt_ray* out_rays, int32_t* out_src,
                                      uint32_t* d_count, uint32_t* trace_order) {
  return spawn_ao(c, rays, hits, pixid, M, nsamples, out_rays, out_src, d_count, trace_order,
                  false);
}

int spray_rt_spawn_shadows_ao(spray_rt_ctx_t c, const spray_rt_ray* rays,
                              const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                              int nsamples, spray_rt_ray* out_rays, int32_t* out_src,
                              uint32_t* d_count) {
  return spawn_ao(c, rays, hits, pixid, M, nsamples, out_rays, out_src, d_count, nullptr, false);
}

int spray_rt_spawn_shadows_ao_pairs(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                    const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                    int nsamples, size_t npix, uint32_t* out_pairs, float* lv,
                                    float* rec, uint32_t* d_count) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (npix == 0 || npix > (size_t(1) << 31))
    return fail(c, SPRAY_RT_ERR_ARG, "AO pairs need 0 < npix <= 2^31 (lv holds npix pixels)");
  if (!d_count || nsamples <= 0 || nsamples > 32)
    return fail(c, SPRAY_RT_ERR_ARG, "AO pairs need 1..32 samples and a device count");
  if (M >= (size_t(1) << 27) || M * size_t(nsamples) > 0xFFFFFFFFull)
    return fail(c, SPRAY_RT_ERR_LIMIT, "AO pairs need M < 2^27 source rays");
  if (!is_device_ptr(d_count) ||
      (M && (!is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(pixid) ||
             !is_device_ptr(out_pairs) || !is_device_ptr(lv) || !is_device_ptr(rec))))
    return fail(c, SPRAY_RT_ERR_ARG, "AO pairs need device buffers");
  HIPCHK(c, hipSetDevice(c->device));
  void* bc = c->d_block_counts;
  int r = ensure(c, &bc, &c->block_cap, ao_scratch_bytes(M, nsamples));
  if (r) return r;
  c->d_block_counts = static_cast<uint32_t*>(bc);
  HIPCHK(c, launch_spawn_ao_pairs(stream_of(c), rays, hits, pixid, M, nsamples, npix, out_pairs,
                                  lv, rec, d_count, c->d_block_counts));
  return SPRAY_RT_OK;
}

int spray_rt_occluded_ao_pairs(spray_rt_ctx_t c, size_t max_n, const uint32_t* pairs,
                               const float* rec, const float* lv, int nsamples,
                               const uint32_t* d_count, uint8_t* occ,
                               unsigned long long* d_counters) {
  int r = scene_common(c, pairs, max_n, occ);
  if (r) return r;
  if (nsamples <= 0 || nsamples > 32) return fail(c, SPRAY_RT_ERR_ARG, "1..32 AO samples");
  if (r) return r;
  if (max_n == 0) return SPRAY_RT_OK;
  if (max_n > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "max_n > 2^32");
  if (!d_count || !is_device_ptr(d_count) || (d_counters && !is_device_ptr(d_counters)) ||
      !is_device_ptr(pairs) || !is_device_ptr(rec) || !is_device_ptr(lv) || !is_device_ptr(occ))
    return fail(c, SPRAY_RT_ERR_ARG, "AO any hit needs device buffers and a device count");
  HIPCHK(c, launch_occluded_ao_pairs(stream_of(c), view(c), max_n, pairs, rec, lv, nsamples,
                                     d_count, occ, d_counters));
  return SPRAY_RT_OK;
}

int spray_rt_occluded_ao(spray_rt_ctx_t c, const spray_rt_ray* rays, const spray_rt_hit* hits,
                         const int32_t* pixid, size_t M, int nsamples, size_t npix,
                         uint32_t* out_pairs, float* lv, float* rec, uint32_t* d_count,
                         uint8_t* occ, unsigned long long* d_counters) {
  int r = spray_rt_spawn_shadows_ao_pairs(c, rays, hits, pixid, M, nsamples, npix, out_pairs, lv,
                                          rec, d_count);
  if (r) return r;
  return spray_rt_occluded_ao_pairs(c, M * size_t(nsamples), out_pairs, rec, lv, nsamples,
                                    d_count, occ, d_counters);
}

int spray_rt_spawn_shadows_ao_traced(spray_rt_ctx_t c, const spray_rt_ray* rays,
                                     const spray_rt_hit* hits, const int32_t* pixid, size_t M,
                                     int nsamples, spray_rt_ray* out_rays, int32_t* out_src,
                                     uint32_t* d_count) {
  return spawn_ao(c, rays, hits, pixid, M, nsamples, out_rays, out_src, d_count, nullptr, true);
}

}  // extern "C"
