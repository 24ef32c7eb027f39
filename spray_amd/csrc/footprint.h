// footprint.h -- screen footprints of domain boxes under the in-situ camera
// (host): which eye rays may enter a box, which hit points' point-light
// shadow rays may cross one, as row runs of pixels; the run tables the
// replicated camera frame launches over (rt_kernels.h CamTable); the
// view-aligned domain partition.
//
// Conservative by construction: a box's pixel rectangle holds the
// perspective projection of its eight corners (the rays through a pixel
// enter the box only if the pixel meets that projection; the box is convex
// and in front of the eye) widened by kGuard pixels for the float rounding
// of the rays; a box that straddles the eye plane takes the whole image.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "rt_kernels.h"

namespace spray_rt {
namespace fp {

constexpr int kGuard = 2;  // pixels of margin around every projected rectangle

// camera_init's record: eye E, image-plane corner A, axes U, V, width, height;
// the eye ray of image point (x, y) points along A + U x / w + V y / h - E
struct Proj {
  double minv[9];  // inverse of [A - E | U | V]
  double e[3];
  double w, h;
};
bool make_proj(const float cam[14], Proj* p);
// pixel coordinates (x = u w, y = v h) of point X and its depth along the
// ray (> 0: in front of the eye)
void project(const Proj& p, const double X[3], double* x, double* y, double* depth);

// per image row: sorted, disjoint inclusive x intervals
using Rows = std::vector<std::vector<std::pair<int, int>>>;

// The pixels whose eye rays may enter box (lo[3], hi[3]): per row, the
// x-extent of the projected box (the convex hull of its eight projected
// corners) over the row's band, widened by kGuard pixels in x and y, added
// to rows (which has image_h rows).  Returns 0 = none, 1 = added, 2 = the
// whole image (a corner at or behind the eye plane; nothing added).
int box_rows(const Proj& p, const float box[6], int image_w, int image_h, Rows& rows);

// The hit points p inside scene box S whose shadow ray toward point light L
// may cross box B: {q + s (q - L) : q in B, 0 <= s <= s_max} within S
// (s_max: where the scaled copy (1 + s) B - s L leaves S along the first
// axis L lies outside B's slab in), as the union of k boxes: slice i is
// AABB(B(s_i) u B(s_i+1)) n S for s_i = s_max i / k -- the coordinates are
// affine in s, so each slice holds its interval's copies.  Returns the
// boxes written to out (<= k, float[k][6]), or -1 = every point (L inside
// S: an unbounded shadow ray may meet B beyond the light).
int shadow_boxes(const float box[6], const float scene[6], const float light[3], int k,
                 float* out);
constexpr int kShadowSlices = 16;
void merge_rows(Rows& rows);
// U: the union of n boxes' footprints (merged rows; a box straddling the eye
// plane: the whole image); *npix = its pixels
Rows union_rows(const Proj& p, const float* boxes, int n, int image_w, int image_h,
                uint64_t* npix);
Rows intersect_rows(const Rows& a, const Rows& b);

struct Table {
  std::vector<CamRun> runs;  // + a sentinel run with pbase = npix
  std::vector<uint32_t> first;
  uint32_t npix = 0;
  uint32_t ymax_pix = 0;  // the largest pixel id (W y + x) in the table
};
// the run table of `rows`; with U (rows inside U's), ubase = the U index of
// each run's first pixel, else ubase = pbase (the table is U)
Table make_table(const Rows& rows, int image_w, const Table* U);
// t.runs (pbase ascending) and t.npix set: the sentinel run and first[]
void finish_table(Table& t);

// View-aligned partition: the domains' box centres projected to the image,
// dealt into nranks groups of (nearly) equal count by recursive median
// splits (x, then y, alternating; ties by domain id) -- each group a set of
// domains along neighbouring lines of sight.
void partition_view(const float* boxes, int n, const Proj& p, int nranks, int* owner);

}  // namespace fp
}  // namespace spray_rt
