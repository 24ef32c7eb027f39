// bvh_build.h -- host builder of the per-domain BVH2 uploaded to HBM.
//
// Replaces the Embree bvh4.triangle4v build that TriMeshBuffer::mapEmbreeBuffer
// triggers through rtcCommit (src/render/trimesh_buffer.cc:189-225).  The tree
// is the canonical BVH2 of SURVEY.md 8(d): binned SAH over 32 bins on each
// axis, leaves of <= 4 triangles, depth-first layout, so its node / triangle
// counts are exactly the ones the algorithmic-byte formula is defined on.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "rt_common.h"

namespace spray_rt {

struct BvhImage {
  std::vector<BvhNode> nodes;   // padded child boxes (device-ready)
  std::vector<float> tris;      // [ntris][12] v0 e1 e2 Ng, leaf order
  std::vector<uint32_t> prims;  // leaf order -> face index
  int depth = 0;
};

// verts: [nverts][3] world space; faces: [nfaces][3].  Throws nothing;
// returns false on invalid face indices.
bool build_bvh(const float* verts, size_t nverts, const uint32_t* faces,
               size_t nfaces, BvhImage* out);

// 16-bit quantized copy of a domain tree for the per-lane any-hit walk
// (QNode, rt_common.h).  Every decoded child box fmaf(q, scale, base)
// contains the padded fp32 box with one grid step to spare; false if a box
// cannot be represented (non-finite finite-box bounds).
bool quantize_nodes(const std::vector<BvhNode>& nodes, QGrid* grid,
                    std::vector<QNode>* out);

// 4-wide quantized copy (QNode4, rt_common.h) of a domain tree, the layout
// the per-lane any hit walks: the BVH2 collapsed greedily (largest-area inner
// child expanded first) under a stack budget of kQ4Stack entries, child
// boxes quantized on the same grid as quantize_nodes.  stack_bound = the
// most entries the walk can hold pending (every entered child but the
// nearest pushed), <= kQ4Stack.  Node 0 is the root, children after parents.
bool quantize_nodes4(const std::vector<BvhNode>& nodes, QGrid* grid,
                     std::vector<QNode4>* out, int* stack_bound);

// Top-level tree over domain boxes [n][6] (lo, hi): same builder, one domain
// per leaf (ref ~(id << 2)), EXACT union boxes (no padding) so that the
// reference's intersectAabb evaluated on a parent accepts whenever it accepts
// a child (float sub/mul are monotone), i.e. the tree prunes nothing the
// brute-force domain test would keep.  An empty right child has ref
// kNoChild and an all-+inf box.
constexpr int32_t kNoChild = INT32_MIN;
bool build_domain_tree(const float* boxes, size_t n, std::vector<BvhNode>* out,
                       int* depth);

}  // namespace spray_rt
