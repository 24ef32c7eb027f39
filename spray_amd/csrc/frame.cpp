// frame.cpp -- C ABI of the frame layer: per-domain BSDFs, the shading pass,
// the film, whole-tile rendering on the device, the blocking-tile list and
// the PPM writer.  The per-tile driver is the device form of
// ooc::Tracer::trace (src/ooc/ooc_tracer.inl:184-234) with the exact
// (non-speculative) resolution of every ray: eye rays -> per bounce
// closest hit -> shade -> any hit of the shadows -> film.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <vector>

#include <cstdlib>
#include <cstring>

#include "footprint.h"
#include "rt_ctx.h"
#include "rt_kernels.h"
#include "spray_rt.h"

using namespace spray_rt;
using namespace spray_rt::detail;

// 1: frames of camera rays lit by one point light take the fused launch
// (fused_frame); 0: every frame takes the general bounce loop.
#ifndef SPRAY_FRAME_FUSED
#define SPRAY_FRAME_FUSED 1
#endif

namespace {

bool shader_ok(const spray_rt_shader* P) {
  if (!P || P->bounces < 1 || P->nlights < 0 || P->nlights > SPRAY_RT_MAX_LIGHTS) return false;
  if (P->shader == SPRAY_RT_SHADER_AO) return P->samples >= 1;
  if (P->shader != SPRAY_RT_SHADER_PT) return false;
  for (int l = 0; l < P->nlights; ++l) {
    const int t = P->lights[l].type;
    if (t != SPRAY_RT_LIGHT_POINT && t != SPRAY_RT_LIGHT_HEMISPHERE) return false;
    if (t == SPRAY_RT_LIGHT_HEMISPHERE && P->samples < 1) return false;
  }
  return true;
}

// carve consecutive 256-B aligned pieces out of one allocation
struct Carve {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t n) {
    T* p = reinterpret_cast<T*>(base + off);
    off += align256(n * sizeof(T));
    return p;
  }
};

// A frame whose whole shading is the point-light term of camera rays (one
// point light, diffuse surfaces, bounces = 1): its single bounce runs as one
// fused launch (closest hit + shading + the shadow rays' any hit) and the
// film.
bool fused_frame(const spray_rt_ctx* c, const spray_rt_shader* P) {
  return SPRAY_FRAME_FUSED && spray_rt::detail::fused_pt_shading(c, P);
}

// The fused frame's eye rays over U only: U = the pixels some domain box's
// screen footprint covers (footprint.h, conservative for any jitter inside
// the pixel); an eye ray outside U misses the whole domain list, so it is
// counted as a radiance ray and not launched.  The run table holds, per
// tile, the runs of U within it (ubase = the run's first pixel's tile-local
// id: the jitter seed and sample id of the tile launch), cached by
// (camera, tiles, boxes).  Returns false when it does not apply
// (SPRAY_FRAME_CULL=0, a degenerate camera).
bool frame_table(spray_rt_ctx* c, const float cam[14], int image_w, const int* tiles, int ntiles,
                 CamTable* T, int* err) {
  *err = SPRAY_RT_OK;
  const char* e = std::getenv("SPRAY_FRAME_CULL");
  if (e && e[0] == '0') return false;
  std::vector<float> key(cam, cam + 14);
  key.push_back(float(image_w));
  key.push_back(float(ntiles));
  for (int k = 0; k < 4 * ntiles; ++k) key.push_back(float(tiles[k]));
  key.insert(key.end(), c->h_boxes.begin(), c->h_boxes.end());
  if (key.size() != c->ftab_key.size() ||
      std::memcmp(key.data(), c->ftab_key.data(), key.size() * sizeof(float)) != 0) {
    fp::Proj pj;
    if (!fp::make_proj(cam, &pj)) return false;
    const int image_h = int(cam[13]);
    const fp::Rows U = fp::union_rows(pj, c->h_boxes.data(), c->ndom, image_w, image_h, nullptr);
    fp::Table t;
    uint32_t np = 0;
    for (int k = 0; k < ntiles; ++k) {
      const int tx = tiles[4 * k], ty = tiles[4 * k + 1], tw = tiles[4 * k + 2],
                th = tiles[4 * k + 3];
      for (int y = ty; y < ty + th; ++y)
        for (const auto& iv : U[size_t(y)]) {
          const int lo = std::max(iv.first, tx), hi = std::min(iv.second, tx + tw - 1);
          if (lo > hi) continue;
          t.runs.push_back(CamRun{y, lo, np, uint32_t((y - ty) * tw + (lo - tx))});
          np += uint32_t(hi - lo + 1);
        }
    }
    t.npix = np;
    fp::finish_table(t);
    // the previous frame's launches may still read the old table
    if (hipStreamSynchronize(stream_of(c)) != hipSuccess) {
      *err = fail(c, SPRAY_RT_ERR_HIP, "frame table: stream sync");
      return false;
    }
    const size_t rb = align256(t.runs.size() * sizeof(CamRun));
    const size_t bytes = rb + t.first.size() * sizeof(uint32_t);
    *err = ensure(c, &c->d_ftab, &c->ftab_cap, bytes);
    if (*err) return false;
    char* d = static_cast<char*>(c->d_ftab);
    if (hipMemcpy(d, t.runs.data(), t.runs.size() * sizeof(CamRun), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMemcpy(d + rb, t.first.data(), t.first.size() * sizeof(uint32_t),
                  hipMemcpyHostToDevice) != hipSuccess) {
      *err = fail(c, SPRAY_RT_ERR_HIP, "frame table upload");
      return false;
    }
    c->ftab_nruns = uint32_t(t.runs.size() - 1);
    c->ftab_npix = np;
    c->ftab_first_off = rb;
    c->ftab_key.swap(key);
  }
  T->runs = static_cast<const CamRun*>(c->d_ftab);
  T->first = reinterpret_cast<const uint32_t*>(static_cast<char*>(c->d_ftab) + c->ftab_first_off);
  T->nruns = c->ftab_nruns;
  T->npix = c->ftab_npix;
  return true;
}

}  // namespace

bool spray_rt::detail::fused_pt_shading(const spray_rt_ctx* c, const spray_rt_shader* P) {
  return P->shader == SPRAY_RT_SHADER_PT && P->bounces == 1 && P->nlights == 1 &&
         P->lights[0].type == SPRAY_RT_LIGHT_POINT && !c->bsdf_delta;
}

extern "C" {

int spray_rt_shadow_slots(const spray_rt_shader* P) {
  if (!shader_ok(P)) return SPRAY_RT_ERR_ARG;
  if (P->shader == SPRAY_RT_SHADER_AO) return P->samples;
  int k = 0;
  for (int l = 0; l < P->nlights; ++l)
    k += P->lights[l].type == SPRAY_RT_LIGHT_HEMISPHERE ? P->samples : 1;
  return k;
}

int spray_rt_set_bsdfs(spray_rt_ctx_t c, int n, const spray_rt_bsdf* bsdfs) {
  if (!c || n < 0 || (n && !bsdfs)) return c ? fail(c, SPRAY_RT_ERR_ARG, "bad bsdf table") : SPRAY_RT_ERR_ARG;
  for (int i = 0; i < n; ++i) {
    const int t = bsdfs[i].type;
    if (t < SPRAY_RT_BSDF_DIFFUSE || t > SPRAY_RT_BSDF_TRANSMISSION)
      return fail(c, SPRAY_RT_ERR_ARG, "bsdf %d: unknown type %d", i, t);
    if ((t == SPRAY_RT_BSDF_GLASS || t == SPRAY_RT_BSDF_TRANSMISSION) &&
        !(bsdfs[i].p[0] > 0.f && bsdfs[i].p[1] > 0.f))
      return fail(c, SPRAY_RT_ERR_ARG, "bsdf %d: refractive indices must be positive", i);
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(stream_of(c)));  // the table may be in use
  if (c->d_bsdf) HIPCHK(c, hipFree(c->d_bsdf));
  c->d_bsdf = nullptr;
  c->nbsdf = 0;
  c->bsdf_delta = false;
  for (int i = 0; i < n; ++i) c->bsdf_delta |= bsdfs[i].type != SPRAY_RT_BSDF_DIFFUSE;
  if (n == 0) return SPRAY_RT_OK;
  HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_bsdf), n * sizeof(spray_rt_bsdf)));
  HIPCHK(c, hipMemcpy(c->d_bsdf, bsdfs, n * sizeof(spray_rt_bsdf), hipMemcpyHostToDevice));
  c->nbsdf = n;
  return SPRAY_RT_OK;
}

int spray_rt_intersect_scene_masked(spray_rt_ctx_t c, const spray_rt_ray* rays, size_t M,
                                    const uint8_t* valid, spray_rt_hit* hits) {
  int r = scene_common(c, rays, M, hits);
  if (r) return r;
  if (M == 0) return SPRAY_RT_OK;
  if (M > 0xFFFFFFFFull) return fail(c, SPRAY_RT_ERR_LIMIT, "M > 2^32");
  if (!valid || !is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(valid))
    return fail(c, SPRAY_RT_ERR_ARG, "masked closest hit needs device buffers");
  hipStream_t s = stream_of(c);
  size_t temp = 0;
  HIPCHK(c, launch_select_flagged(s, valid, M, nullptr, nullptr, nullptr, &temp));
  const size_t b_idx = align256(M * sizeof(uint32_t));
  r = ensure(c, &c->d_sel, &c->sel_cap, b_idx + 256 + temp);
  if (r) return r;
  char* base = static_cast<char*>(c->d_sel);
  uint32_t* idx = reinterpret_cast<uint32_t*>(base);
  uint32_t* num = reinterpret_cast<uint32_t*>(base + b_idx);
  HIPCHK(c, launch_select_flagged(s, valid, M, idx, num, base + b_idx + 256, &temp));
  HIPCHK(c, launch_scene_intersect_indexed(s, view(c), rays, M, idx, num, hits));
  return SPRAY_RT_OK;
}

int spray_rt_shade(spray_rt_ctx_t c, const spray_rt_shader* P, int bounce, spray_rt_ray* rays,
                   const spray_rt_hit* hits, float* w, uint8_t* valid, const int32_t* pixid,
                   const int32_t* samid, size_t M, spray_rt_ray* shadows, float* sw,
                   uint8_t* svalid, unsigned long long* d_stats) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!shader_ok(P) || bounce < 0) return fail(c, SPRAY_RT_ERR_ARG, "bad shader configuration");
  if (M == 0) return SPRAY_RT_OK;
  const int ns = spray_rt_shadow_slots(P);
  const bool need_pix = P->shader == SPRAY_RT_SHADER_AO;
  if (!is_device_ptr(rays) || !is_device_ptr(hits) || !is_device_ptr(w) ||
      !is_device_ptr(valid) || (need_pix && !is_device_ptr(pixid)) ||
      (!need_pix && !is_device_ptr(samid)) || (ns && (!is_device_ptr(shadows) ||
                                                      !is_device_ptr(sw) ||
                                                      !is_device_ptr(svalid))) ||
      (d_stats && !is_device_ptr(d_stats)))
    return fail(c, SPRAY_RT_ERR_ARG, "shading buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, launch_shade(stream_of(c), *P, c->d_bsdf, c->nbsdf, bounce, ns, rays, hits, w, valid,
                         pixid, samid, M, shadows, sw, svalid, d_stats));
  return SPRAY_RT_OK;
}

int spray_rt_film(spray_rt_ctx_t c, float* image, const int32_t* pixid, size_t M, int spp,
                  int ns, const float* sw, const uint8_t* svalid, const uint8_t* occ,
                  double scale) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (spp <= 0 || ns < 0 || M % size_t(spp))
    return fail(c, SPRAY_RT_ERR_ARG, "film: M must be a multiple of spp");
  if (M == 0 || ns == 0) return SPRAY_RT_OK;
  if (!is_device_ptr(image) || !is_device_ptr(pixid) || !is_device_ptr(sw) ||
      !is_device_ptr(svalid) || !is_device_ptr(occ))
    return fail(c, SPRAY_RT_ERR_ARG, "film buffers must be device memory");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, launch_film(stream_of(c), image, pixid, M, spp, ns, sw, svalid, occ, scale));
  return SPRAY_RT_OK;
}

int spray_rt_render_tiles(spray_rt_ctx_t c, const spray_rt_shader* P, const float cam[14],
                          int image_w, int spp, const int* tiles, int ntiles, float* image) {
  if (!c) return SPRAY_RT_ERR_ARG;
  if (!shader_ok(P) || !cam || spp <= 0 || image_w <= 0 || ntiles < 0 || (ntiles && !tiles))
    return fail(c, SPRAY_RT_ERR_ARG, "bad render arguments");
  size_t M = 0;
  for (int k = 0; k < ntiles; ++k) {
    const int tx = tiles[4 * k], ty = tiles[4 * k + 1], tw = tiles[4 * k + 2],
              th = tiles[4 * k + 3];
    if (tw < 0 || th < 0 || tx < 0 || ty < 0 || tx + tw > image_w || ty + th > int(cam[13]))
      return fail(c, SPRAY_RT_ERR_ARG, "bad tile %d", k);
    M += size_t(tw) * th * spp;
  }
  if (M == 0) return SPRAY_RT_OK;
  const int ns = spray_rt_shadow_slots(P);
  const size_t MS = M * size_t(ns);
  if (M > 0xFFFFFFFFull || MS > 0xFFFFFFFFull)
    return fail(c, SPRAY_RT_ERR_LIMIT, "batch too large (samples x shadow slots > 2^32)");
  if (!is_device_ptr(image)) return fail(c, SPRAY_RT_ERR_ARG, "image must be device memory");
  int r = scene_common(c, image, M, image);
  if (r) return r;
  const size_t bytes = align256(M * sizeof(spray_rt_ray)) + align256(M * sizeof(spray_rt_hit)) +
                       align256(M * 16) + align256(M) + 2 * align256(M * 4) +
                       align256(MS * sizeof(spray_rt_ray)) + align256(MS * 16) +
                       2 * align256(MS) + align256(sizeof(uint32_t));
  r = ensure(c, &c->d_frame, &c->frame_cap, bytes);
  if (r) return r;
  hipStream_t s = stream_of(c);
  if (!c->d_fstats) {
    const size_t fb = 4 * kStatStripes * sizeof(unsigned long long);
    HIPCHK(c, hipMalloc(reinterpret_cast<void**>(&c->d_fstats), fb));
    HIPCHK(c, hipMemsetAsync(c->d_fstats, 0, fb, s));
  }
  Carve cv{static_cast<char*>(c->d_frame)};
  uint32_t* nshadow = cv.take<uint32_t>(1);
  spray_rt_ray* rays = cv.take<spray_rt_ray>(M);
  spray_rt_hit* hits = cv.take<spray_rt_hit>(M);
  float* w = cv.take<float>(4 * M);
  uint8_t* valid = cv.take<uint8_t>(M);
  int32_t* pixid = cv.take<int32_t>(M);
  int32_t* samid = cv.take<int32_t>(M);
  spray_rt_ray* sh = cv.take<spray_rt_ray>(MS);
  float* sw = cv.take<float>(4 * MS);
  uint8_t* sv = cv.take<uint8_t>(MS);
  uint8_t* occ = cv.take<uint8_t>(MS);
  // each tile's eye rays (tile-local sampler seeds) at its offset; from
  // here on every pass is per slot (or per pixel group of spp slots), so
  // the batch gives each tile exactly its own-launch result
  const double scale = 1.0 / double(spp);
  if (fused_frame(c, P)) {
    const spray_rt_light& lt = P->lights[0];
    const float shade10[10] = {lt.pos[0],      lt.pos[1],      lt.pos[2], lt.radiance[0],
                               lt.radiance[1], lt.radiance[2], P->ks[0],  P->ks[1],
                               P->ks[2],       P->shininess};
    // the eye rays of U's pixels (frame_table) or of the whole tiles
    CamTable T{};
    size_t Mt = M;  // rays launched
    if (frame_table(c, cam, image_w, tiles, ntiles, &T, &r)) {
      Mt = size_t(T.npix) * size_t(spp);
      HIPCHK(c, launch_eye_rays_ooc_table(s, cam, image_w, spp, T, rays, pixid, samid));
    } else {
      if (r) return r;
      HIPCHK(c,
             launch_eye_rays_ooc_tiles(s, cam, image_w, spp, tiles, ntiles, rays, pixid, samid));
    }
    // the film needs the shading and occlusion only: no hit records
    HIPCHK(c, launch_scene_frame_pt(s, view(c), rays, Mt, nullptr, shade10, occ, sv, sw, nshadow));
    HIPCHK(c, launch_frame_stats_add(s, c->d_fstats, kStatStripes, M, nshadow));
    HIPCHK(c, launch_film(s, image, pixid, Mt, spp, ns, sw, sv, occ, scale));
    return SPRAY_RT_OK;
  }
  HIPCHK(c, launch_eye_rays_ooc_tiles(s, cam, image_w, spp, tiles, ntiles, rays, pixid, samid));
  HIPCHK(c, launch_path_init(s, w, valid, M));
  const int user = c->coherence;
  for (int b = 0; b < P->bounces; ++b) {
    if (b == 0) {
      // camera rays: coherent packets
      c->coherence = SPRAY_RT_RAYS_COHERENT;
      hipError_t e = launch_scene_intersect(s, view(c), rays, M, hits, nullptr);
      c->coherence = user;
      HIPCHK(c, e);
    } else {
      r = spray_rt_intersect_scene_masked(c, rays, M, valid, hits);
      if (r) return r;
    }
    HIPCHK(c, launch_shade(s, *P, c->d_bsdf, c->nbsdf, b, ns, rays, hits, w, valid, pixid, samid,
                           M, sh, sw, sv, c->d_fstats, kStatStripes));
    if (ns) {
      r = spray_rt_occluded_scene_masked(c, sh, MS, sv, occ);
      if (r) return r;
      HIPCHK(c, launch_film(s, image, pixid, M, spp, ns, sw, sv, occ, scale));
    }
  }
  return SPRAY_RT_OK;
}

int spray_rt_render_tile(spray_rt_ctx_t c, const spray_rt_shader* P, const float cam[14],
                         int image_w, int spp, int tx, int ty, int tw, int th, float* image) {
  const int t[4] = {tx, ty, tw, th};
  return spray_rt_render_tiles(c, P, cam, image_w, spp, t, 1, image);
}

int spray_rt_frame_stats(spray_rt_ctx_t c, unsigned long long out[3], int reset) {
  if (!c || !out) return SPRAY_RT_ERR_ARG;
  out[0] = out[1] = out[2] = 0;
  if (!c->d_fstats) return SPRAY_RT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t s = stream_of(c);
  unsigned long long hs[4 * kStatStripes], h[4] = {0, 0, 0, 0};
  HIPCHK(c, hipMemcpyAsync(hs, c->d_fstats, sizeof(hs), hipMemcpyDeviceToHost, s));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_fstats, 0, sizeof(hs), s));
  HIPCHK(c, hipStreamSynchronize(s));
  for (int k = 0; k < 4; ++k)
    for (int x = 0; x < kStatStripes; ++x) h[k] += hs[k * kStatStripes + x];
  out[0] = h[3];
  out[1] = h[1];
  out[2] = h[0];
  if (h[0])
    return fail(c, SPRAY_RT_ERR_UNSUPPORTED, "%llu shading cases the reference aborts on", h[0]);
  return SPRAY_RT_OK;
}

// ImageScheduleTileList::init (tile.cc:317-391): this rank's vertical
// stripe of the image (makeVerticalStripe, :208-230) cut into horizontal
// tiles of at most max_samples_per_rank samples.
static int image_schedule_tiles(int image_w, int image_h, int spp, int nranks, int rank,
                                long long max_samples, int* tiles, int cap, int* n) {
  const int sw = std::max(image_w / nranks, 1);
  const int sx = rank * sw;
  *n = 0;
  if (sx >= image_w) return SPRAY_RT_OK;  // empty stripe: no tiles
  const int vw = (sx + sw > image_w || rank == nranks - 1) ? image_w - sx : sw;
  const long long samples = (long long)vw * image_h * spp;
  const long long est = (samples + max_samples - 1) / max_samples;
  if (est >= INT_MAX) return SPRAY_RT_ERR_LIMIT;
  const int th = image_h / int(est);
  if (th <= 0) return SPRAY_RT_ERR_LIMIT;  // the reference divides by zero here
  *n = (image_h + th - 1) / th;
  if (*n > cap) return tiles ? SPRAY_RT_ERR_LIMIT : SPRAY_RT_OK;
  int k = 0;
  for (int y = 0; y < image_h; y += th) {
    int* t = tiles + 4 * k++;
    t[0] = sx;
    t[1] = y;
    t[2] = vw;
    t[3] = std::min(th, image_h - y);
  }
  return SPRAY_RT_OK;
}

int spray_rt_tile_list(int schedule, int image_w, int image_h, int spp, int nranks, int rank,
                       long long max_samples_per_rank, int* tiles, int cap, int* n) {
  if (image_w <= 0 || image_h <= 0 || spp <= 0 || nranks <= 0 || rank < 0 || rank >= nranks ||
      max_samples_per_rank <= 0 || !n || cap < 0 || (cap && !tiles))
    return SPRAY_RT_ERR_ARG;
  if (schedule == SPRAY_RT_TILES_IMAGE)
    return image_schedule_tiles(image_w, image_h, spp, nranks, rank, max_samples_per_rank,
                                tiles, cap, n);
  if (schedule != SPRAY_RT_TILES_BLOCKING) return SPRAY_RT_ERR_ARG;
  // BlockingTileList::init (tile.cc:52-153)
  const long long total = (long long)image_w * image_h * spp;
  const long long per_cluster = max_samples_per_rank * nranks;
  const long long ntiles = (total + per_cluster - 1) / per_cluster;
  const long long n1 = (long long)std::ceil(std::sqrt(double(ntiles)));
  if (n1 <= 0 || n1 > image_w || n1 > image_h) return SPRAY_RT_ERR_LIMIT;
  const int tw = int(image_w / n1), thh = int(image_h / n1);
  const int nx = (image_w + tw - 1) / tw, ny = (image_h + thh - 1) / thh;
  *n = nx * ny;
  if (*n > cap) return tiles ? SPRAY_RT_ERR_LIMIT : SPRAY_RT_OK;
  int k = 0;
  for (int y = 0; y < image_h; y += thh) {
    for (int x = 0; x < image_w; x += tw) {
      const int w = std::min(tw, image_w - x), h = std::min(thh, image_h - y);
      if ((long long)w * h * spp > per_cluster) return SPRAY_RT_ERR_LIMIT;  // CHECK_LE, :128
      // makeHorizontalStripe (tile.cc:184-206)
      const int sh = std::max(h / nranks, 1);
      const int sy = y + rank * sh, yend = y + h;
      int* t = tiles + 4 * k++;
      if (sy >= yend) {
        t[0] = 0; t[1] = sy; t[2] = 0; t[3] = 0;
      } else {
        t[0] = x;
        t[1] = sy;
        t[2] = w;
        t[3] = (sy + sh > yend || rank == nranks - 1) ? yend - sy : sh;
      }
    }
  }
  return SPRAY_RT_OK;
}

int spray_rt_write_ppm(const char* path, const float* rgba, int w, int h) {
  if (!path || !rgba || w <= 0 || h <= 0) return SPRAY_RT_ERR_ARG;
  FILE* f = std::fopen(path, "w");
  if (!f) return SPRAY_RT_ERR_ARG;
  std::fprintf(f, "P3\n%d %d\n1023\n", w, h);
  for (int y = h - 1; y > -1; --y) {
    for (int x = 0; x < w; ++x) {
      const float* p = rgba + 4 * (size_t(y) * w + x);
      unsigned v[3];
      for (int k = 0; k < 3; ++k) {
        // glm::clamp(c * 1023.f, 0, 1023) then (unsigned) truncation
        const float t = p[k] * 1023.f;
        const float cl = std::min(std::max(t, 0.0f), 1023.0f);
        v[k] = unsigned(cl);
      }
      std::fprintf(f, "%u %u %u\n", v[0], v[1], v[2]);
    }
  }
  return std::fclose(f) == 0 ? SPRAY_RT_OK : SPRAY_RT_ERR_ARG;
}

}  // extern "C"
