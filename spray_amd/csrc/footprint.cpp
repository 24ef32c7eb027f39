// footprint.cpp -- see footprint.h.
#include "footprint.h"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <stdexcept>

namespace spray_rt {
namespace fp {

bool make_proj(const float cam[14], Proj* p) {
  double m[9];  // columns A - E, U, V (row-major m[3 r + c])
  for (int r = 0; r < 3; ++r) {
    m[3 * r + 0] = double(cam[3 + r]) - double(cam[r]);
    m[3 * r + 1] = double(cam[6 + r]);
    m[3 * r + 2] = double(cam[9 + r]);
  }
  const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8],
               c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  if (!(std::fabs(det) > 1e-300) || !std::isfinite(det)) return false;
  const double id = 1.0 / det;
  p->minv[0] = c00 * id;
  p->minv[1] = (m[2] * m[7] - m[1] * m[8]) * id;
  p->minv[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  p->minv[3] = c01 * id;
  p->minv[4] = (m[0] * m[8] - m[2] * m[6]) * id;
  p->minv[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  p->minv[6] = c02 * id;
  p->minv[7] = (m[1] * m[6] - m[0] * m[7]) * id;
  p->minv[8] = (m[0] * m[4] - m[1] * m[3]) * id;
  for (int k = 0; k < 3; ++k) p->e[k] = cam[k];
  p->w = cam[12];
  p->h = cam[13];
  return p->w > 0 && p->h > 0;
}

void project(const Proj& p, const double X[3], double* x, double* y, double* depth) {
  const double v[3] = {X[0] - p.e[0], X[1] - p.e[1], X[2] - p.e[2]};
  const double a = p.minv[0] * v[0] + p.minv[1] * v[1] + p.minv[2] * v[2];
  const double b = p.minv[3] * v[0] + p.minv[4] * v[1] + p.minv[5] * v[2];
  const double c = p.minv[6] * v[0] + p.minv[7] * v[1] + p.minv[8] * v[2];
  *depth = a;
  *x = b / a * p.w;
  *y = c / a * p.h;
}

int box_rect(const Proj& p, const float box[6], int image_w, int image_h, int rect[4]) {
  double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
  int front = 0, behind = 0;
  for (int k = 0; k < 8; ++k) {
    const double X[3] = {box[(k & 1) ? 3 : 0], box[(k & 2) ? 4 : 1], box[(k & 4) ? 5 : 2]};
    double x, y, d;
    project(p, X, &x, &y, &d);
    // a corner at or behind the eye plane (depth = the ray parameter of the
    // point in units of the image-plane distance): its projection is unbounded
    if (!(d > 1e-9) || !std::isfinite(x) || !std::isfinite(y)) {
      ++behind;
      continue;
    }
    ++front;
    xmin = std::min(xmin, x);
    xmax = std::max(xmax, x);
    ymin = std::min(ymin, y);
    ymax = std::max(ymax, y);
  }
  if (!front) return 0;  // wholly behind the eye: no eye ray enters it
  if (behind) {
    rect[0] = 0;
    rect[1] = image_w - 1;
    rect[2] = 0;
    rect[3] = image_h - 1;
    return 2;
  }
  const auto clampi = [](double v, int lo, int hi) {
    if (!(v > lo)) return lo;
    if (!(v < hi)) return hi;
    return int(v);
  };
  const int x0 = clampi(std::floor(xmin) - kGuard, 0, image_w - 1);
  const int x1 = clampi(std::floor(xmax) + kGuard, 0, image_w - 1);
  const int y0 = clampi(std::floor(ymin) - kGuard, 0, image_h - 1);
  const int y1 = clampi(std::floor(ymax) + kGuard, 0, image_h - 1);
  // wholly off one side of the image
  if (std::floor(xmax) + kGuard < 0 || std::floor(xmin) - kGuard > image_w - 1 ||
      std::floor(ymax) + kGuard < 0 || std::floor(ymin) - kGuard > image_h - 1)
    return 0;
  rect[0] = x0;
  rect[1] = x1;
  rect[2] = y0;
  rect[3] = y1;
  return 1;
}

int shadow_region(const float box[6], const float scene[6], const float light[3], float out[6]) {
  double ext = 0.0;
  for (int a = 0; a < 3; ++a) ext = std::max(ext, double(scene[3 + a]) - double(scene[a]));
  const double pad = 1e-3 * std::max(ext, 1.0);
  bool inside = true;
  for (int a = 0; a < 3; ++a)
    inside = inside && light[a] >= scene[a] - pad && light[a] <= scene[3 + a] + pad;
  if (inside) return 1;
  double smax = INFINITY;
  for (int a = 0; a < 3; ++a) {
    const double lo = box[a], hi = box[3 + a], L = light[a];
    if (L < lo) smax = std::min(smax, (double(scene[3 + a]) - lo) / (lo - L));
    if (L > hi) smax = std::min(smax, (hi - double(scene[a])) / (L - hi));
  }
  if (!std::isfinite(smax)) return 1;
  smax = std::max(smax, 0.0);
  for (int a = 0; a < 3; ++a) {
    const double lo = box[a], hi = box[3 + a], L = light[a];
    const double lo2 = (1.0 + smax) * lo - smax * L, hi2 = (1.0 + smax) * hi - smax * L;
    const double rlo = std::max(std::min(lo, lo2) - pad, double(scene[a]) - pad);
    const double rhi = std::min(std::max(hi, hi2) + pad, double(scene[3 + a]) + pad);
    out[a] = float(rlo);
    out[3 + a] = float(rhi);
    // float rounding of the bounds: outward
    if (double(out[a]) > rlo) out[a] = std::nextafter(out[a], -INFINITY);
    if (double(out[3 + a]) < rhi) out[3 + a] = std::nextafter(out[3 + a], INFINITY);
  }
  return 0;
}

void add_rect(Rows& rows, const int rect[4]) {
  for (int y = rect[2]; y <= rect[3]; ++y)
    if (y >= 0 && y < int(rows.size())) rows[size_t(y)].push_back({rect[0], rect[1]});
}

void merge_rows(Rows& rows) {
  for (auto& r : rows) {
    if (r.empty()) continue;
    std::sort(r.begin(), r.end());
    std::vector<std::pair<int, int>> m;
    for (const auto& iv : r) {
      if (!m.empty() && iv.first <= m.back().second + 1)
        m.back().second = std::max(m.back().second, iv.second);
      else
        m.push_back(iv);
    }
    r.swap(m);
  }
}

Rows intersect_rows(const Rows& a, const Rows& b) {
  Rows out(std::min(a.size(), b.size()));
  for (size_t y = 0; y < out.size(); ++y) {
    size_t i = 0, j = 0;
    const auto& ra = a[y];
    const auto& rb = b[y];
    while (i < ra.size() && j < rb.size()) {
      const int lo = std::max(ra[i].first, rb[j].first);
      const int hi = std::min(ra[i].second, rb[j].second);
      if (lo <= hi) out[y].push_back({lo, hi});
      if (ra[i].second < rb[j].second)
        ++i;
      else
        ++j;
    }
  }
  return out;
}

Table make_table(const Rows& rows, int image_w, const Table* U) {
  Table t;
  uint32_t np = 0;
  size_t ur = 0;  // U runs are in the same (y, x) order: one forward scan
  for (size_t y = 0; y < rows.size(); ++y)
    for (const auto& iv : rows[y]) {
      CamRun r{int32_t(y), iv.first, np, np};
      const uint32_t len = uint32_t(iv.second - iv.first + 1);
      if (U) {
        while (ur < U->runs.size() - 1) {
          const CamRun& q = U->runs[ur];
          const uint32_t qlen = U->runs[ur + 1].pbase - q.pbase;
          if (q.y > int32_t(y) || (q.y == int32_t(y) && q.x0 + int32_t(qlen) > iv.first)) break;
          ++ur;
        }
        if (ur >= U->runs.size() - 1) throw std::logic_error("footprint run outside U");
        const CamRun& q = U->runs[ur];
        const uint32_t qlen = U->runs[ur + 1].pbase - q.pbase;
        if (q.y != int32_t(y) || iv.first < q.x0 || iv.second >= q.x0 + int32_t(qlen))
          throw std::logic_error("footprint run outside U");
        r.ubase = q.ubase + uint32_t(iv.first - q.x0);
      }
      t.runs.push_back(r);
      t.ymax_pix = std::max(t.ymax_pix, uint32_t(image_w) * uint32_t(y) + uint32_t(iv.second));
      np += len;
    }
  t.npix = np;
  t.runs.push_back(CamRun{0, 0, np, np});  // sentinel
  t.first.assign((np + 7) / 8 + 1, 0u);
  uint32_t r = 0;
  for (uint32_t g = 0; g < t.first.size(); ++g) {
    const uint32_t pix = 8 * g;
    while (r + 1 < t.runs.size() - 1 && t.runs[r + 1].pbase <= pix) ++r;
    t.first[g] = r;
  }
  return t;
}

void partition_view(const float* boxes, int n, const Proj& p, int nranks, int* owner) {
  std::vector<double> x(static_cast<size_t>(n)), y(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    const double c[3] = {(double(boxes[6 * i]) + boxes[6 * i + 3]) * 0.5,
                         (double(boxes[6 * i + 1]) + boxes[6 * i + 4]) * 0.5,
                         (double(boxes[6 * i + 2]) + boxes[6 * i + 5]) * 0.5};
    double d;
    project(p, c, &x[size_t(i)], &y[size_t(i)], &d);
    if (!std::isfinite(x[size_t(i)])) x[size_t(i)] = 0.0;
    if (!std::isfinite(y[size_t(i)])) y[size_t(i)] = 0.0;
  }
  std::vector<int> ids(static_cast<size_t>(n));
  std::iota(ids.begin(), ids.end(), 0);
  struct Split {
    static void run(std::vector<int> v, int r0, int r1, int axis, const std::vector<double>& x,
                    const std::vector<double>& y, int* owner) {
      if (r1 - r0 <= 1) {
        for (int i : v) owner[i] = r0;
        return;
      }
      const std::vector<double>& key = axis == 0 ? x : y;
      std::sort(v.begin(), v.end(), [&](int a, int b) {
        return key[size_t(a)] < key[size_t(b)] || (key[size_t(a)] == key[size_t(b)] && a < b);
      });
      const int h = (r1 - r0) / 2;
      const size_t cut = v.size() * size_t(h) / size_t(r1 - r0);
      run(std::vector<int>(v.begin(), v.begin() + long(cut)), r0, r0 + h, 1 - axis, x, y, owner);
      run(std::vector<int>(v.begin() + long(cut), v.end()), r0 + h, r1, 1 - axis, x, y, owner);
    }
  };
  Split::run(ids, 0, nranks, 0, x, y, owner);
}

}  // namespace fp
}  // namespace spray_rt
