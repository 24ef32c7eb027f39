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

// rect = [x0, x1] x [y0, y1] (inclusive pixels) of the eye rays that may
// enter box (lo[3], hi[3]); returns 0 = none, 1 = rect, 2 = the whole image
int box_rect(const Proj& p, const float box[6], int image_w, int image_h, int rect[4]);

// The hit points p inside scene box S whose shadow ray toward point light L
// may cross box B: {q + s (q - L) : q in B, s >= 0} within S, bounded by the
// box AABB(B u B') n S with B' = (1 + s_max) B - s_max L (s_max: where the
// scaled copy leaves S along the first axis L lies outside B's slab in).
// Returns 0 and that box in out, or 1 = every point (L inside S: an
// unbounded shadow ray may meet B beyond the light).
int shadow_region(const float box[6], const float scene[6], const float light[3], float out[6]);

// per image row: sorted, disjoint inclusive x intervals
using Rows = std::vector<std::vector<std::pair<int, int>>>;
void add_rect(Rows& rows, const int rect[4]);
void merge_rows(Rows& rows);
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

// View-aligned partition: the domains' box centres projected to the image,
// dealt into nranks groups of (nearly) equal count by recursive median
// splits (x, then y, alternating; ties by domain id) -- each group a set of
// domains along neighbouring lines of sight.
void partition_view(const float* boxes, int n, const Proj& p, int nranks, int* owner);

}  // namespace fp
}  // namespace spray_rt
