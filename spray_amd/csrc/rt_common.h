// rt_common.h -- layouts shared by the host runtime and the gfx950 kernels.
//
// HBM layout of one cache slot (one domain), all 16-B aligned:
//   nodes  : BvhNode[nnodes]        64 B  -- BVH2, both child boxes + refs
//   tris   : float4[3 * ntris]      48 B  -- v0 | e1 | e2 | Ng packed in
//                                            three float4 (leaf order)
//   prims  : uint32[ntris]          4 B   -- leaf order -> PLY face index
//   faces  : uint32[3 * nfaces]     epilogue gather (PLY order)
//   colors : uint32[nverts]         0xRRGGBB per vertex
//   normals: float[3 * nverts]      unnormalised vertex normals
// A device-side SlotDesc table points at these; the scene path adds a
// domain -> slot map and the domain AABBs.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace spray_rt {

constexpr int kLeafMax = 4;        // triangles per leaf (canonical BVH2)
constexpr int kBins = 32;          // SAH bins per axis
constexpr int kMaxDepth = 24;      // builder guarantees depth <= kMaxDepth
constexpr int kStack = 24;         // per-lane traversal stack (LDS), >= kMaxDepth
constexpr float kRayEpsilon = 0.001f;  // SPRAY_RAY_EPSILON, render/spray.h:46
constexpr unsigned kDomainListSize = 16;  // SPRAY_RAY_DOMAIN_LIST_SIZE, src/CMakeLists.txt:32-35
// Culling slack of the slab test (results never depend on culling as long as
// it is conservative; tests/ check BVH == brute force bit-exactly).
constexpr float kTfarSlack = 1.0000153f;  // 1 + 2^-16
constexpr float kBoxPad = 1e-6f;          // relative node-box padding
constexpr float kTopPad = 1e-5f;          // internal boxes of the domain tree
constexpr float kDirClamp = 1e-20f;       // |d| floor for the inverse dir

// 64-B BVH2 node: left box, right box, child refs.  ref >= 0: internal node
// index (slot-local); ref < 0: leaf ~((first << 2) | (count - 1)).
struct alignas(16) BvhNode {
  float l_lo[3];
  float l_hi[3];
  float r_lo[3];
  float r_hi[3];
  int32_t left;
  int32_t right;
  int32_t pad0;
  int32_t pad1;
};
static_assert(sizeof(BvhNode) == 64, "node must be 64 B");

// 32-B quantized copy of a BvhNode: both child boxes as 16-bit grid
// coordinates of the domain's grid (base + q * scale per axis), rounded
// outward by at least one extra grid step, so every decoded box contains the
// padded fp32 box and culling stays conservative; an empty (+inf) box
// becomes the grid's far corner.  The BVH2 form of the quantization (host
// export and tests); slots carry the 4-wide QNode4 below.  The quantized
// copy sits in front of the fp32 nodes of the same slot, so the scene
// descriptors (DomTrav) address it without another pointer.
struct alignas(16) QNode {
  uint16_t q[12];  // l_lo xyz, l_hi xyz, r_lo xyz, r_hi xyz
  int32_t left;
  int32_t right;
};
static_assert(sizeof(QNode) == 32, "quantized node must be 32 B");
// 64-B 4-wide quantized node (the BVH2 collapsed, bvh_build.h
// quantize_nodes4), the node layout of the per-lane any-hit walk of scene
// slots: four child boxes as 16-bit grid coordinates (child c: q[6c..6c+2]
// lo, q[6c+3..6c+5] hi) and four child refs (>= 0 QNode4 index, < 0 leaf
// as in BvhNode, kNoChild = empty).  In front of the fp32 nodes:
//   nodes - 32                : QGrid
//   nodes - 64 - 64 * (i + 1) : QNode4 i   (64-B aligned)
struct alignas(16) QNode4 {
  uint16_t q[24];
  int32_t child[4];
};
static_assert(sizeof(QNode4) == 64, "4-wide quantized node must be 64 B");
// stack entries of the 4-wide walk: the launch's LDS stack (STK) plus a
// private overflow of kQ4Stack - STK
constexpr int kQ4Stack = 40;
// the collapse's stack bound never exceeds the BVH2 height, which the builder
// caps at kMaxDepth (+1 for the root level): a tree the builder accepts always
// fits the 4-wide walk's stack, so quantize_nodes4 fails only on the grid
static_assert(kMaxDepth + 1 <= kQ4Stack, "4-wide walk stack below the BVH2 height bound");
struct alignas(16) QGrid {
  float base[3];
  float pad0;
  float scale[3];
  float pad1;
};
static_assert(sizeof(QGrid) == 32, "grid header must be 32 B");

struct alignas(16) SlotDesc {
  const BvhNode* nodes;
  const float* tris;        // 12 floats per triangle
  const uint32_t* prims;
  const uint32_t* faces;
  const uint32_t* colors;
  const float* normals;
  uint32_t ntris;
  uint32_t nverts;
  uint32_t nnodes;
  uint32_t pad;
};

// Per-domain traversal descriptor of the scene path (16 B, staged in LDS by
// the scene kernels): tris / prims live at byte offsets from the slot's
// nodes; nodes == nullptr marks a domain that is not resident (or empty).
struct alignas(16) DomTrav {
  const BvhNode* nodes;
  uint32_t tri_off;
  uint32_t prim_off;
};
static_assert(sizeof(DomTrav) == 16, "DomTrav must be 16 B");

// Persistent scene launches: kQueues work queues (kQueues / 8 per XCD), head
// counters 32 words apart.
constexpr int kQueues = 64;
constexpr size_t kHeadsBytes = size_t(kQueues) * 32 * 4;  // queue heads, 32 words apart

}  // namespace spray_rt
