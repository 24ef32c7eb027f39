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

namespace {

struct P2 {
  double x, y;
};

// Andrew's monotone chain; the hull counter-clockwise without repeats
std::vector<P2> hull(std::vector<P2> p) {
  std::sort(p.begin(), p.end(), [](const P2& a, const P2& b) {
    return a.x < b.x || (a.x == b.x && a.y < b.y);
  });
  if (p.size() < 3) return p;
  std::vector<P2> h(2 * p.size());
  size_t k = 0;
  const auto cross = [](const P2& o, const P2& a, const P2& b) {
    return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x);
  };
  for (size_t i = 0; i < p.size(); ++i) {
    while (k >= 2 && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
    h[k++] = p[i];
  }
  for (size_t i = p.size() - 1, t = k + 1; i > 0; --i) {
    while (k >= t && cross(h[k - 2], h[k - 1], p[i - 1]) <= 0) --k;
    h[k++] = p[i - 1];
  }
  h.resize(k - 1);
  return h;
}

// x-extent of convex polygon `poly` within the band ya <= y <= yb (false:
// empty): the polygon clipped by the two lines (Sutherland-Hodgman)
bool band_extent(const std::vector<P2>& poly, double ya, double yb, double* x0, double* x1) {
  std::vector<P2> a = poly, b;
  const auto clip = [](const std::vector<P2>& in, std::vector<P2>& out, double y, bool keep_above) {
    out.clear();
    const size_t n = in.size();
    for (size_t i = 0; i < n; ++i) {
      const P2& c = in[i];
      const P2& d = in[(i + 1) % n];
      const bool ci = keep_above ? c.y >= y : c.y <= y;
      const bool di = keep_above ? d.y >= y : d.y <= y;
      if (ci) out.push_back(c);
      if (ci != di) {
        const double t = (y - c.y) / (d.y - c.y);
        out.push_back(P2{c.x + t * (d.x - c.x), y});
      }
    }
  };
  if (a.size() < 3) {  // degenerate hull: its points in the band
    double lo = INFINITY, hi = -INFINITY;
    for (const P2& q : a)
      if (q.y >= ya && q.y <= yb) {
        lo = std::min(lo, q.x);
        hi = std::max(hi, q.x);
      }
    *x0 = lo;
    *x1 = hi;
    return lo <= hi;
  }
  clip(a, b, ya, true);
  if (b.empty()) return false;
  clip(b, a, yb, false);
  if (a.empty()) return false;
  double lo = INFINITY, hi = -INFINITY;
  for (const P2& q : a) {
    lo = std::min(lo, q.x);
    hi = std::max(hi, q.x);
  }
  *x0 = lo;
  *x1 = hi;
  return true;
}

}  // namespace

int box_rows(const Proj& p, const float box[6], int image_w, int image_h, Rows& rows) {
  std::vector<P2> pts;
  int behind = 0;
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
    pts.push_back(P2{x, y});
  }
  if (pts.empty()) return 0;  // wholly behind the eye: no eye ray enters it
  if (behind) return 2;
  double ymin = INFINITY, ymax = -INFINITY;
  for (const P2& q : pts) {
    ymin = std::min(ymin, q.y);
    ymax = std::max(ymax, q.y);
  }
  const double ylo = std::floor(ymin) - kGuard, yhi = std::floor(ymax) + kGuard;
  if (yhi < 0 || ylo > image_h - 1) return 0;
  const std::vector<P2> h = hull(pts);
  const int y0 = int(std::max(ylo, 0.0)), y1 = int(std::min(yhi, double(image_h - 1)));
  bool any = false;
  for (int y = y0; y <= y1; ++y) {
    // rays of row y have image y in [y, y + 1); kGuard rows of margin
    double xa, xb;
    if (!band_extent(h, double(y - kGuard), double(y + 1 + kGuard), &xa, &xb)) continue;
    const double lo = std::floor(xa) - kGuard, hi = std::floor(xb) + kGuard;
    if (hi < 0 || lo > image_w - 1) continue;
    rows[size_t(y)].push_back({int(std::max(lo, 0.0)), int(std::min(hi, double(image_w - 1)))});
    any = true;
  }
  return any ? 1 : 0;
}

int shadow_boxes(const float box[6], const float scene[6], const float light[3], int k,
                 float* out) {
  double ext = 0.0;
  for (int a = 0; a < 3; ++a) ext = std::max(ext, double(scene[3 + a]) - double(scene[a]));
  const double pad = 1e-3 * std::max(ext, 1.0);
  bool inside = true;
  for (int a = 0; a < 3; ++a)
    inside = inside && light[a] >= scene[a] - pad && light[a] <= scene[3 + a] + pad;
  if (inside) return -1;
  double smax = INFINITY;
  for (int a = 0; a < 3; ++a) {
    const double lo = box[a], hi = box[3 + a], L = light[a];
    if (L < lo) smax = std::min(smax, (double(scene[3 + a]) - lo) / (lo - L));
    if (L > hi) smax = std::min(smax, (hi - double(scene[a])) / (L - hi));
  }
  if (!std::isfinite(smax)) return -1;
  smax = std::max(smax, 0.0);
  int n = 0;
  for (int i = 0; i < k; ++i) {
    const double s0 = smax * i / k, s1 = smax * (i + 1) / k;
    float* o = out + 6 * n;
    bool empty = false;
    for (int a = 0; a < 3; ++a) {
      const double lo = box[a], hi = box[3 + a], L = light[a];
      const double l0 = lo + s0 * (lo - L), l1 = lo + s1 * (lo - L);
      const double h0 = hi + s0 * (hi - L), h1 = hi + s1 * (hi - L);
      const double rlo = std::max(std::min(l0, l1) - pad, double(scene[a]) - pad);
      const double rhi = std::min(std::max(h0, h1) + pad, double(scene[3 + a]) + pad);
      if (rlo > rhi) empty = true;
      o[a] = float(rlo);
      o[3 + a] = float(rhi);
      // float rounding of the bounds: outward
      if (double(o[a]) > rlo) o[a] = std::nextafter(o[a], -INFINITY);
      if (double(o[3 + a]) < rhi) o[3 + a] = std::nextafter(o[3 + a], INFINITY);
    }
    if (!empty) ++n;
  }
  return n;
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

Rows union_rows(const Proj& p, const float* boxes, int n, int image_w, int image_h,
                uint64_t* npix) {
  Rows U(static_cast<size_t>(image_h));
  bool all = false;
  for (int d = 0; d < n; ++d) all = box_rows(p, boxes + 6 * size_t(d), image_w, image_h, U) == 2 || all;
  if (all)
    for (auto& row : U) row.assign(1, {0, image_w - 1});
  merge_rows(U);
  uint64_t np = 0;
  for (const auto& row : U)
    for (const auto& iv : row) np += uint64_t(iv.second - iv.first + 1);
  if (npix) *npix = np;
  return U;
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
  finish_table(t);
  return t;
}

void finish_table(Table& t) {
  const uint32_t np = t.npix;
  t.runs.push_back(CamRun{0, 0, np, np});  // sentinel
  t.first.assign((np + 7) / 8 + 1, 0u);
  uint32_t r = 0;
  for (uint32_t g = 0; g < t.first.size(); ++g) {
    const uint32_t pix = 8 * g;
    while (r + 1 < t.runs.size() - 1 && t.runs[r + 1].pbase <= pix) ++r;
    t.first[g] = r;
  }
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
