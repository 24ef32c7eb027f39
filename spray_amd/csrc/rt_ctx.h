// rt_ctx.h -- the engine context behind spray_rt_ctx_t and the internal
// helpers shared by the C ABI translation units (rt_api.cpp, ooc.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "rt_common.h"
#include "rt_kernels.h"
#include "spray_rt.h"

namespace spray_rt {
namespace detail {

struct SlotHost {
  void* dmem = nullptr;  // one allocation: nodes|tris|prims|faces|colors|normals
  size_t bytes = 0;
  SlotDesc desc{};
  int depth = 0;
  hipEvent_t ready = nullptr;  // async upload completion
  void* pinned = nullptr;      // staging for async uploads
  size_t pinned_bytes = 0;
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace detail
}  // namespace spray_rt

struct spray_rt_ctx {
  using SlotHost = spray_rt::detail::SlotHost;
  using SlotDesc = spray_rt::SlotDesc;
  using DomTrav = spray_rt::DomTrav;
  using BvhNode = spray_rt::BvhNode;

  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t user_stream = nullptr;
  bool user_stream_set = false;
  hipStream_t upload_stream = nullptr;
  std::vector<SlotHost> slots;
  SlotDesc* d_slots = nullptr;
  size_t d_slots_cap = 0;
  bool slots_dirty = true;
  // scene path
  int ndom = 0;
  float* d_boxes = nullptr;
  std::vector<float> h_boxes;  // the same boxes on the host (ooc drain views)
  int* d_dom2slot = nullptr;
  DomTrav* d_domtrav = nullptr;  // per-domain traversal descriptors
  int* d_owner = nullptr;        // in-situ domain -> rank map
  std::vector<int> h_owner;      // the same map on the host
  BvhNode* d_tlas = nullptr;  // top-level tree over the domain boxes
  int ntlas = 0;
  int tlas_depth = 0;
  int coherence = SPRAY_RT_RAYS_ADAPTIVE;
  std::vector<int> dom2slot;
  bool dom_dirty = true;
  // segment tables
  int* d_seg_slot = nullptr;
  size_t* d_seg_off = nullptr;
  size_t seg_cap = 0;
  // host-pointer staging
  void* d_stage = nullptr;
  size_t stage_cap = 0;
  void* d_stage2 = nullptr;
  size_t stage2_cap = 0;
  void* d_stage3 = nullptr;
  size_t stage3_cap = 0;
  uint32_t* d_block_counts = nullptr;
  // work-queue heads of the persistent launches: [0, kHeadsBytes) zeroed by
  // each launch, [kHeadsBytes, 2 kHeadsBytes) zeroed by a frame's launch_clear
  uint32_t* d_heads = nullptr;
  void* d_sel = nullptr;        // selected indices + count + select scratch
  size_t sel_cap = 0;
  size_t block_cap = 0;
  // frame layer
  spray_rt_bsdf* d_bsdf = nullptr;  // per-domain BSDFs (Scene::getBsdf)
  int nbsdf = 0;
  bool bsdf_delta = false;  // some domain's BSDF is not diffuse
  void* d_frame = nullptr;  // render_tile path buffers
  size_t frame_cap = 0;
  unsigned long long* d_fstats = nullptr;  // render_tile totals (shade stats)
  // render_tiles' footprint-culled frame: the run table of the last
  // (camera, tiles, boxes) -- runs then first, frame.cpp -- and its key
  std::vector<float> ftab_key;
  void* d_ftab = nullptr;
  size_t ftab_cap = 0;
  uint32_t ftab_nruns = 0, ftab_npix = 0;
  size_t ftab_first_off = 0;  // bytes from d_ftab to the first[] array
  std::string err;
  std::mutex mu;  // lanes: the lazy table rebuild (prepare) runs under it
};

// A per-host-thread submission lane of a context (spray_rt_lane_*): its own
// stream, staging buffers and one-segment table, so concurrent threads never
// share mutable state; they only read the context's device tables.
struct spray_rt_lane {
  spray_rt_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  void* d_buf = nullptr;
  size_t cap = 0;
  int* d_seg_slot = nullptr;
  size_t* d_seg_off = nullptr;
  std::string err;
};

namespace spray_rt {
namespace detail {

// Device image of one domain, packed on the host: [quantized nodes + grid]
// | BVH2 nodes | triangle records | leaf->face map | faces | colors |
// normals, 256-B aligned (the HBM slot layout of rt_common.h).  The
// quantized copy (QNode, in front of the nodes) is built for scene slots
// only (quantized = true): the OOC drains do not read it, so its images
// stream without it.
struct SlotImage {
  std::vector<char> bytes;  // may be released once a pinned copy exists
  size_t nbytes = 0;        // the image's size (== bytes.size() while held)
  size_t o_nodes = 0, o_tris = 0, o_prims = 0, o_faces = 0;
  size_t o_colors = SIZE_MAX, o_normals = SIZE_MAX;  // SIZE_MAX: absent
  uint32_t nnodes = 0, ntris = 0, nverts = 0;
  int depth = 0;
  // descriptor of the image once copied to device address base
  SlotDesc desc_at(const void* base) const;
};
// Builds the canonical BVH2 (bvh_build.h) and packs the image.  Returns
// nullptr on success, else what is wrong with the mesh (face index out of
// range, too many faces, non-finite vertex, coordinates beyond the range of
// the quantized node grid).
const char* build_slot_image(const float* verts, size_t nverts, const uint32_t* faces,
                      size_t nfaces, const uint32_t* colors, const float* normals,
                      SlotImage* out, bool quantized = true);

// Copies a packed image into cache slot `slot` (allocating it), after the
// queued work that may read the slot's previous image.  From pinned_src
// (pinned host memory holding img.bytes, kept alive by the caller) or with
// async = true: an async copy on the upload stream, ordered before the next
// query by the slot's ready event; else a synchronous copy.
int upload_slot_image(spray_rt_ctx* c, int slot, const SlotImage& img, const void* pinned_src,
                      bool async);

// Records a message in the context; returns code.
int fail(spray_rt_ctx* c, int code, const char* fmt, ...);
hipStream_t stream_of(spray_rt_ctx* c);
bool is_device_ptr(const void* p);
// grows *buf to at least bytes (device memory)
int ensure(spray_rt_ctx* c, void** buf, size_t* cap, size_t bytes);
// scene-path entry checks + lazy rebuild of the device scene tables
int scene_common(spray_rt_ctx* c, const void* rays, size_t M, const void* out);
// the kernels' view of the resident scene (coherence = the context's)
SceneView view(const spray_rt_ctx* c);
// the whole shading of a bounce is the point-light term of camera rays (PT,
// one point light, diffuse surfaces, bounces = 1): it fuses into the
// closest-hit launch (launch_scene_frame_pt)
bool fused_pt_shading(const spray_rt_ctx* c, const spray_rt_shader* P);

}  // namespace detail
}  // namespace spray_rt

#define HIPCHK(ctx, expr)                                                   \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess)                                                   \
      return ::spray_rt::detail::fail(ctx, SPRAY_RT_ERR_HIP, "%s: %s", #expr, \
                                      hipGetErrorString(_e));               \
  } while (0)
