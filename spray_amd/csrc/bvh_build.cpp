// bvh_build.cpp -- canonical BVH2 builder (binned SAH, 32 bins x 3 axes,
// <= 4 triangles per leaf, depth-first layout).  Compiled with
// -ffp-contract=off: box areas, bin indices and SAH costs are evaluated in a
// fixed order, so the tree is a deterministic function of the mesh (tests/
// compare it node for node with the oracle's canonical tree).
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

namespace spray_rt {
namespace {

constexpr float kInf = std::numeric_limits<float>::infinity();

struct Box {
  float lo[3], hi[3];
  void clear() {
    for (int j = 0; j < 3; ++j) {
      lo[j] = kInf;
      hi[j] = -kInf;
    }
  }
  void grow(const Box& o) {
    for (int j = 0; j < 3; ++j) {
      if (o.lo[j] < lo[j]) lo[j] = o.lo[j];
      if (o.hi[j] > hi[j]) hi[j] = o.hi[j];
    }
  }
  void grow_point(const float* p) {
    for (int j = 0; j < 3; ++j) {
      if (p[j] < lo[j]) lo[j] = p[j];
      if (p[j] > hi[j]) hi[j] = p[j];
    }
  }
  // half surface area, evaluated (dx*dy + dy*dz) + dz*dx
  float half_area() const {
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return (dx * dy + dy * dz) + dz * dx;
  }
};

int ceil_log2(size_t x) {
  int l = 0;
  while ((size_t(1) << l) < x) ++l;
  return l;
}

// Conservative padding of a finite child box (culling only): each bound
// moves out by rel x max(|lo|, |hi|, extent).
void pad_rel(float lo[3], float hi[3], float rel) {
  if (!(std::isfinite(lo[0]) && std::isfinite(hi[0]))) return;
  for (int j = 0; j < 3; ++j) {
    float e = hi[j] - lo[j];
    float m = std::fmax(std::fmax(std::fabs(lo[j]), std::fabs(hi[j])), e);
    float p = m * rel;
    lo[j] = lo[j] - p;
    hi[j] = hi[j] + p;
  }
}
void pad(float lo[3], float hi[3]) { pad_rel(lo, hi, kBoxPad); }

class Builder {
 public:
  // triangles
  Builder(const float* v, const uint32_t* f, size_t nf, BvhImage* out)
      : nf_(nf), out_(out) {
    init(nf);
    for (size_t i = 0; i < nf; ++i) {
      Box b;
      b.clear();
      for (int k = 0; k < 3; ++k) b.grow_point(v + 3 * size_t(f[3 * i + k]));
      set_prim(i, b);
    }
  }
  // boxes [n][6]
  Builder(const float* boxes, size_t n, int leaf_max, BvhImage* out)
      : nf_(n), out_(out), leaf_max_(leaf_max) {
    init(n);
    for (size_t i = 0; i < n; ++i) {
      Box b;
      for (int j = 0; j < 3; ++j) {
        b.lo[j] = boxes[6 * i + j];
        b.hi[j] = boxes[6 * i + 3 + j];
      }
      set_prim(i, b);
    }
  }

  void run() {
    out_->nodes.clear();
    out_->prims.clear();
    out_->depth = 0;
    if (nf_ == 0) return;
    if (nf_ <= size_t(leaf_max_)) {
      // root that is itself a leaf: left child = the leaf, right = empty box
      size_t self = alloc();
      Box lb;
      int32_t lref = recurse(0, nf_, 1, &lb);
      BvhNode& n = out_->nodes[self];
      std::memcpy(n.l_lo, lb.lo, 12);
      std::memcpy(n.l_hi, lb.hi, 12);
      for (int j = 0; j < 3; ++j) n.r_lo[j] = n.r_hi[j] = kInf;  // never hit
      n.left = lref;
      n.right = leaf_max_ == kLeafMax ? ~int32_t(0) : kNoChild;
    } else {
      Box rb;
      recurse(0, nf_, 0, &rb);
    }
  }

 private:
  void init(size_t n) {
    box_.resize(n);
    cent_.resize(3 * n);
    idx_.resize(n);
    tmp_.resize(n);
  }
  void set_prim(size_t i, const Box& b) {
    box_[i] = b;
    for (int j = 0; j < 3; ++j) cent_[3 * i + j] = (b.lo[j] + b.hi[j]) * 0.5f;
    idx_[i] = uint32_t(i);
  }

  size_t alloc() {
    out_->nodes.emplace_back();
    std::memset(&out_->nodes.back(), 0, sizeof(BvhNode));
    return out_->nodes.size() - 1;
  }

  int bin_of(uint32_t p, int axis, float lo, float scale) const {
    int k = int((cent_[3 * p + axis] - lo) * scale);
    return std::min(std::max(k, 0), kBins - 1);
  }

  int32_t recurse(size_t begin, size_t end, int depth, Box* bb_out) {
    const size_t n = end - begin;
    Box bb, cb;
    bb.clear();
    cb.clear();
    for (size_t i = begin; i < end; ++i) {
      uint32_t p = idx_[i];
      bb.grow(box_[p]);
      cb.grow_point(&cent_[3 * p]);
    }
    *bb_out = bb;
    out_->depth = std::max(out_->depth, depth);
    if (n <= size_t(leaf_max_)) {
      uint32_t first = uint32_t(out_->prims.size());
      for (size_t i = begin; i < end; ++i) out_->prims.push_back(idx_[i]);
      return ~int32_t((first << 2) | uint32_t(n - 1));
    }

    float ext[3] = {cb.hi[0] - cb.lo[0], cb.hi[1] - cb.lo[1], cb.hi[2] - cb.lo[2]};
    int best_axis = -1, best_split = -1;
    const bool median =
        depth + ceil_log2((n + leaf_max_ - 1) / leaf_max_) >= kMaxDepth;
    if (!median) {
      float best = kInf;
      for (int a = 0; a < 3; ++a) {
        if (!(ext[a] > 0.0f)) continue;
        const float scale = float(kBins) / ext[a];
        Box bins[kBins];
        uint32_t cnt[kBins];
        for (int k = 0; k < kBins; ++k) {
          bins[k].clear();
          cnt[k] = 0;
        }
        for (size_t i = begin; i < end; ++i) {
          uint32_t p = idx_[i];
          int k = bin_of(p, a, cb.lo[a], scale);
          bins[k].grow(box_[p]);
          ++cnt[k];
        }
        float right_area[kBins];
        uint32_t right_cnt[kBins];
        Box acc;
        acc.clear();
        uint32_t c = 0;
        for (int k = kBins - 1; k > 0; --k) {
          acc.grow(bins[k]);
          c += cnt[k];
          right_area[k] = c ? acc.half_area() : 0.0f;
          right_cnt[k] = c;
        }
        acc.clear();
        c = 0;
        for (int k = 0; k < kBins - 1; ++k) {
          acc.grow(bins[k]);
          c += cnt[k];
          if (c == 0 || right_cnt[k + 1] == 0) continue;
          float cost = float(c) * acc.half_area() +
                       float(right_cnt[k + 1]) * right_area[k + 1];
          if (cost < best) {
            best = cost;
            best_axis = a;
            best_split = k + 1;
          }
        }
      }
    }

    size_t mid;
    if (best_axis >= 0) {
      const float scale = float(kBins) / ext[best_axis];
      size_t l = begin, r = 0;
      for (size_t i = begin; i < end; ++i) {
        uint32_t p = idx_[i];
        if (bin_of(p, best_axis, cb.lo[best_axis], scale) < best_split)
          idx_[l++] = p;
        else
          tmp_[r++] = p;
      }
      std::copy(tmp_.begin(), tmp_.begin() + r, idx_.begin() + l);
      mid = l;
    } else {
      int a = 0;
      if (ext[1] > ext[a]) a = 1;
      if (ext[2] > ext[a]) a = 2;
      if (ext[a] > 0.0f) {
        const float* c = cent_.data();
        std::sort(idx_.begin() + begin, idx_.begin() + end,
                  [c, a](uint32_t x, uint32_t y) {
                    float cx = c[3 * x + a], cy = c[3 * y + a];
                    return cx < cy || (cx == cy && x < y);
                  });
      }
      mid = begin + n / 2;
    }

    size_t self = alloc();
    Box lb, rb;
    int32_t lref = recurse(begin, mid, depth + 1, &lb);
    int32_t rref = recurse(mid, end, depth + 1, &rb);
    BvhNode& nd = out_->nodes[self];
    std::memcpy(nd.l_lo, lb.lo, 12);
    std::memcpy(nd.l_hi, lb.hi, 12);
    std::memcpy(nd.r_lo, rb.lo, 12);
    std::memcpy(nd.r_hi, rb.hi, 12);
    nd.left = lref;
    nd.right = rref;
    return int32_t(self);
  }

  size_t nf_;
  BvhImage* out_;
  int leaf_max_ = kLeafMax;
  std::vector<Box> box_;
  std::vector<float> cent_;
  std::vector<uint32_t> idx_, tmp_;
};

}  // namespace

bool build_bvh(const float* verts, size_t nverts, const uint32_t* faces,
               size_t nfaces, BvhImage* out) {
  for (size_t i = 0; i < 3 * nfaces; ++i)
    if (faces[i] >= nverts) return false;
  if (nfaces >= (size_t(1) << 29)) return false;
  Builder b(verts, faces, nfaces, out);
  b.run();
  // padded child boxes for the device
  for (BvhNode& n : out->nodes) {
    pad(n.l_lo, n.l_hi);
    pad(n.r_lo, n.r_hi);
  }
  // triangle records in leaf order: v0, e1 = v0 - v1, e2 = v2 - v0,
  // Ng = e1 x e2 written with the kernels' explicit FMA form
  out->tris.resize(12 * out->prims.size());
  for (size_t i = 0; i < out->prims.size(); ++i) {
    const uint32_t* f = faces + 3 * size_t(out->prims[i]);
    const float* a = verts + 3 * size_t(f[0]);
    const float* b = verts + 3 * size_t(f[1]);
    const float* c = verts + 3 * size_t(f[2]);
    float* r = &out->tris[12 * i];
    r[0] = a[0];
    r[1] = a[1];
    r[2] = a[2];
    r[3] = a[0] - b[0];
    r[4] = a[1] - b[1];
    r[5] = a[2] - b[2];
    r[6] = c[0] - a[0];
    r[7] = c[1] - a[1];
    r[8] = c[2] - a[2];
    r[9] = std::fma(r[4], r[8], -(r[5] * r[7]));
    r[10] = std::fma(r[5], r[6], -(r[3] * r[8]));
    r[11] = std::fma(r[3], r[7], -(r[4] * r[6]));
  }
  return true;
}

bool build_domain_tree(const float* boxes, size_t n, std::vector<BvhNode>* out,
                       int* depth) {
  out->clear();
  *depth = 0;
  if (n == 0) return true;
  if (n >= (size_t(1) << 29)) return false;
  BvhImage img;
  Builder b(boxes, n, 1, &img);
  b.run();
  // leaves hold one box each: rewrite ~((first << 2) | 0) as ~(id << 2).
  // Internal children get a padded box: the packet walk tests them with the
  // fast (fma) slab, a superset of the exact test with this margin; leaf
  // boxes stay exact -- they decide the mask.
  for (BvhNode& nd : img.nodes) {
    for (int side = 0; side < 2; ++side) {
      int32_t* ref = side ? &nd.right : &nd.left;
      if (*ref >= 0) {
        pad_rel(side ? nd.r_lo : nd.l_lo, side ? nd.r_hi : nd.l_hi, kTopPad);
        continue;
      }
      if (*ref == kNoChild) continue;
      uint32_t first = ~uint32_t(*ref) >> 2;
      *ref = ~int32_t(img.prims[first] << 2);
    }
  }
  *out = std::move(img.nodes);
  *depth = img.depth;
  return true;
}

namespace {

bool empty_box(const float* lo) { return lo[0] == kInf; }  // builder's never-hit box

// grid over the union of the finite child boxes, ~700 steps of margin
bool make_qgrid(const std::vector<BvhNode>& nodes, QGrid* grid) {
  *grid = QGrid{};
  float lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
  for (const BvhNode& n : nodes)
    for (int side = 0; side < 2; ++side) {
      const float* bl = side ? n.r_lo : n.l_lo;
      const float* bh = side ? n.r_hi : n.l_hi;
      if (empty_box(bl)) continue;
      for (int j = 0; j < 3; ++j) {
        if (!std::isfinite(bl[j]) || !std::isfinite(bh[j])) return false;
        lo[j] = std::min(lo[j], bl[j]);
        hi[j] = std::max(hi[j], bh[j]);
      }
    }
  if (!(lo[0] <= hi[0])) {  // no finite box at all
    for (int j = 0; j < 3; ++j) lo[j] = hi[j] = 0.f;
  }
  for (int j = 0; j < 3; ++j) {
    double ext = double(hi[j]) - double(lo[j]);
    if (!(ext > 0)) ext = std::max(std::fabs(double(lo[j])), 1.0) * 1e-3;
    // The step never drops below 2^-19 of the axis' coordinate magnitude
    // (>= 16 ulps): a flat or tiny domain far from the origin (a ground quad
    // at y = -1, a wall at x = 5) then still has a base 700 steps below lo
    // that fp32 can represent, and every bound has a representable step of
    // margin.  Wider extents keep ext / 64000 (65535 steps cover ext + 1400).
    const double mag = std::max(std::fabs(double(lo[j])), std::fabs(double(hi[j])));
    grid->scale[j] = float(std::max(ext / 64000.0, std::ldexp(mag, -19)));
    grid->base[j] = float(double(lo[j]) - 700.0 * double(grid->scale[j]));
    if (!std::isfinite(grid->base[j]) || !(grid->scale[j] > 0.f)) return false;
  }
  return true;
}

// One child box as grid coordinates q[0..2] = lo, q[3..5] = hi, rounded
// outward with one extra step: the decoded bound (the value the kernel's
// folded slab evaluates up to rounding, which the extra step covers) lies a
// whole step outside the fp32 bound.  An empty box becomes the far corner.
bool quant_box(const QGrid& grid, const float* bl, const float* bh, uint16_t* q) {
  auto dec = [&](int j, long v) {
    return double(std::fma(float(v), grid.scale[j], grid.base[j]));
  };
  for (int j = 0; j < 3; ++j) {
    if (empty_box(bl)) {
      q[j] = q[3 + j] = 0xFFFF;
      continue;
    }
    const double s = grid.scale[j];
    long ql = long(std::floor((double(bl[j]) - grid.base[j]) / s)) - 2;
    while (ql > 0 && !(dec(j, ql) + s <= double(bl[j]))) --ql;
    long qh = long(std::ceil((double(bh[j]) - grid.base[j]) / s)) + 2;
    while (qh < 0xFFFF && !(dec(j, qh) - s >= double(bh[j]))) ++qh;
    if (ql < 0 || qh > 0xFFFF || !(dec(j, ql) + s <= double(bl[j])) ||
        !(dec(j, qh) - s >= double(bh[j])))
      return false;
    q[j] = uint16_t(ql);
    q[3 + j] = uint16_t(qh);
  }
  return true;
}

// Collapse of the BVH2 into QNode4s: a node's children start as the BVH2
// node's two children; the inner child with the largest box area is replaced
// by its own two children while fewer than four are held and the stack
// budget allows it (the per-lane walk pushes every entered child but the
// nearest: pend + k - 1 entries, and a child subtree of BVH2 height h can
// always be walked with h more).
struct Collapse {
  const std::vector<BvhNode>& n2;
  const QGrid& grid;
  std::vector<QNode4>* out;
  std::vector<int> height;  // BVH2 inner levels below (leaf 0)
  int budget;
  int bound = 0;
  bool ok = true;

  struct Cand {
    const float* lo;
    const float* hi;
    int32_t ref;
  };
  int h_of(int32_t ref) const { return ref >= 0 ? height[size_t(ref)] : 0; }
  static float area(const Cand& c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return (dx * dy + dy * dz) + dz * dx;
  }
  void children(int32_t node, std::vector<Cand>* cs) const {
    const BvhNode& n = n2[size_t(node)];
    if (n.left != kNoChild && !empty_box(n.l_lo)) cs->push_back({n.l_lo, n.l_hi, n.left});
    if (n.right != kNoChild && !empty_box(n.r_lo)) cs->push_back({n.r_lo, n.r_hi, n.right});
  }
  int32_t emit(int32_t node, int pend) {
    std::vector<Cand> cs;
    children(node, &cs);
    for (;;) {
      if (cs.size() >= 4) break;
      int pick = -1;
      float best = -1.f;
      for (size_t k = 0; k < cs.size(); ++k) {
        if (cs[k].ref < 0) continue;
        // the set after expanding k must keep pend + (size - 1) + max height <= budget
        std::vector<Cand> gc;
        children(cs[k].ref, &gc);
        int hmax = 0;
        for (size_t m = 0; m < cs.size(); ++m)
          if (m != k) hmax = std::max(hmax, h_of(cs[m].ref));
        for (const Cand& g : gc) hmax = std::max(hmax, h_of(g.ref));
        const int size = int(cs.size()) - 1 + int(gc.size());
        if (size > 4 || pend + size - 1 + hmax > budget) continue;
        const float a = area(cs[k]);
        if (a > best) {
          best = a;
          pick = int(k);
        }
      }
      if (pick < 0) break;
      std::vector<Cand> gc;
      children(cs[size_t(pick)].ref, &gc);
      cs.erase(cs.begin() + pick);
      cs.insert(cs.begin() + pick, gc.begin(), gc.end());
    }
    const int32_t id = int32_t(out->size());
    out->push_back(QNode4{});
    const int k = int(cs.size());
    const int p2 = pend + (k > 0 ? k - 1 : 0);
    bound = std::max(bound, p2);
    QNode4 q{};
    for (int c = 0; c < 4; ++c) {
      q.child[c] = kNoChild;
      for (int j = 0; j < 6; ++j) q.q[6 * c + j] = 0xFFFF;
    }
    for (int c = 0; c < k; ++c) {
      if (!quant_box(grid, cs[size_t(c)].lo, cs[size_t(c)].hi, q.q + 6 * c)) ok = false;
      q.child[c] = cs[size_t(c)].ref;
    }
    for (int c = 0; c < k && ok; ++c)
      if (cs[size_t(c)].ref >= 0) q.child[c] = emit(cs[size_t(c)].ref, p2);
    (*out)[size_t(id)] = q;
    return id;
  }
};

}  // namespace

bool quantize_nodes(const std::vector<BvhNode>& nodes, QGrid* grid,
                    std::vector<QNode>* out) {
  out->assign(nodes.size(), QNode{});
  if (!make_qgrid(nodes, grid)) return false;
  for (size_t i = 0; i < nodes.size(); ++i) {
    const BvhNode& n = nodes[i];
    QNode& o = (*out)[i];
    o.left = n.left;
    o.right = n.right;
    if (!quant_box(*grid, n.l_lo, n.l_hi, o.q) || !quant_box(*grid, n.r_lo, n.r_hi, o.q + 6))
      return false;
  }
  return true;
}

bool quantize_nodes4(const std::vector<BvhNode>& nodes, QGrid* grid,
                     std::vector<QNode4>* out, int* stack_bound) {
  out->clear();
  if (stack_bound) *stack_bound = 0;
  if (!make_qgrid(nodes, grid)) return false;
  if (nodes.empty()) return true;
  Collapse c{nodes, *grid, out, std::vector<int>(nodes.size(), 0), kQ4Stack};
  // depth-first layout: children follow their parent
  for (size_t i = nodes.size(); i-- > 0;)
    c.height[i] = 1 + std::max(c.h_of(nodes[i].left), c.h_of(nodes[i].right));
  if (c.height[0] > kQ4Stack) {  // reported as a stack overflow, not a grid failure
    if (stack_bound) *stack_bound = c.height[0];
    return false;
  }
  c.emit(0, 0);
  if (stack_bound) *stack_bound = c.bound;
  return c.ok && c.bound <= kQ4Stack;
}

}  // namespace spray_rt
