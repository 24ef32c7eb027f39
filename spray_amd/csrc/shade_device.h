// shade_device.h -- device side of the shading callers around the hot path:
// the reference's RandomSampler (deps/embree/random_sampler.h:34-113),
// cosine-hemisphere sampling (render/sampler.h:49-128, sampler.cc:54-60),
// Blinn-Phong and the delta BSDF rules (render/reflection.h:139-364) and the
// light samplers (render/light.h:30-96).
//
// Float operations follow glm's operand order, as oracle/oracle.c does; the
// transcendental calls are evaluated in double and rounded once
// (cos/sin/pow), so host and device agree bit for bit instead of to the few
// ulps two different libm's would give.
#pragma once

#include "rt_device.h"

namespace spray_rt {
namespace {

constexpr float kOneOverPi = 0.3183098861837907f;  // SPRAY_ONE_OVER_PI, spray.h:50
constexpr double kPi = 3.14159265358979323846;      // SPRAY_PI = M_PI, spray.h:48

// RandomSampler_init(id): murmur3 mix + finaliser; get1D: LCG step, top 31
// bits scaled to [0, 1).
__device__ __forceinline__ uint32_t mm_mix(uint32_t hash, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = (k << 15) | (k >> 17);
  k *= 0x1b873593u;
  hash ^= k;
  hash = ((hash << 13) | (hash >> 19)) * 5u + 0xe6546b64u;
  return hash;
}
__device__ __forceinline__ uint32_t mm_fin(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t sampler_init1(int id) {
  return mm_fin(mm_mix(0u, uint32_t(id)));
}
__device__ __forceinline__ float sampler_1d(uint32_t& s) {
  s = s * 1664525u + 1013904223u;
  return float(int32_t(s >> 1)) * 4.656612873077392578125e-10f;
}

__device__ __forceinline__ float gdot3(const float* a, const float* b) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
// glm::normalize: v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt
__device__ __forceinline__ void gnorm3(float* a) {
  const float inv = 1.0f / sqrtf(gdot3(a, a));
  a[0] *= inv;
  a[1] *= inv;
  a[2] *= inv;
}
__device__ __forceinline__ float gclamp01(float x) {
  return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x);
}
__device__ __forceinline__ float cos_r(float x) { return float(cos(double(x))); }
__device__ __forceinline__ float sin_r(float x) { return float(sin(double(x))); }
__device__ __forceinline__ float pow_r(float x, float y) {
  return float(pow(double(x), double(y)));
}

// util::unpack (utils/util.h): 0xRRGGBB -> channel * SPRAY_1_OVER_255 (double)
__device__ __forceinline__ void unpack_rgb(uint32_t c, float kd[3]) {
  kd[0] = float(double((c >> 16) & 0xffu) * 0.00392156862745098);
  kd[1] = float(double((c >> 8) & 0xffu) * 0.00392156862745098);
  kd[2] = float(double(c & 0xffu) * 0.00392156862745098);
}

// getCosineHemisphereSample(u1, u2, N, &wi, &pdf): ConcentricDiskSampling,
// v.z = sqrt(max(0, 1 - x^2 - y^2)), normalize, localToWorld (mat3(dx, dy,
// N) * v), normalize; pdf = v.z / pi.  theta *= SPRAY_PI / 4.f is a double
// product (M_PI is a double).
// Split in two: the sample in the local frame (a function of u1, u2 only) ...
__device__ __forceinline__ void hemisphere_local(float u1, float u2, float lv[3]) {
  const float sx = 2 * u1 - 1, sy = 2 * u2 - 1;
  float dx, dy;
  if (sx == 0.0f && sy == 0.0f) {
    dx = 0.0f;
    dy = 0.0f;
  } else {
    float rr, th;
    if (sx >= -sy) {
      if (sx > sy) {
        rr = sx;
        th = sy > 0.0f ? sy / rr : 8.0f + sy / rr;
      } else {
        rr = sy;
        th = 2.0f - sx / rr;
      }
    } else {
      if (sx <= sy) {
        rr = -sx;
        th = 4.0f - sy / rr;
      } else {
        rr = -sy;
        th = 6.0f + sx / rr;
      }
    }
    th = float(double(th) * (kPi / 4.0));
    // one shared argument reduction; the same values as cos() and sin()
    double sd, cd;
    sincos(double(th), &sd, &cd);
    dx = rr * float(cd);
    dy = rr * float(sd);
  }
  lv[0] = dx;
  lv[1] = dy;
  lv[2] = sqrtf(fmaxf(0.f, (1.f - dx * dx) - dy * dy));
  gnorm3(lv);
}

// ... rotated into the frame of N (localToWorld), and its pdf.  The frame
// (ax, ay) depends on N only: callers with many samples per normal build it
// once.
__device__ __forceinline__ void hemisphere_frame(const float N[3], float ax[3], float ay[3]) {
  const float dx0[3] = {0.f, N[2], -N[1]}, dx1[3] = {-N[2], 0.f, N[0]};
  const float* pick = gdot3(dx0, dx0) > gdot3(dx1, dx1) ? dx0 : dx1;
  ax[0] = pick[0];
  ax[1] = pick[1];
  ax[2] = pick[2];
  gnorm3(ax);
  ay[0] = N[1] * ax[2] - ax[1] * N[2];
  ay[1] = N[2] * ax[0] - ax[2] * N[0];
  ay[2] = N[0] * ax[1] - ax[0] * N[1];
  gnorm3(ay);
}

__device__ __forceinline__ void hemisphere_apply(const float lv[3], const float N[3],
                                                 const float ax[3], const float ay[3],
                                                 float wi[3], float& pdf) {
  wi[0] = (ax[0] * lv[0] + ay[0] * lv[1]) + N[0] * lv[2];
  wi[1] = (ax[1] * lv[0] + ay[1] * lv[1]) + N[1] * lv[2];
  wi[2] = (ax[2] * lv[0] + ay[2] * lv[1]) + N[2] * lv[2];
  gnorm3(wi);
  pdf = lv[2] * kOneOverPi;
}

__device__ __forceinline__ void hemisphere_world(const float lv[3], const float N[3],
                                                 float wi[3], float& pdf) {
  float ax[3], ay[3];
  hemisphere_frame(N, ax, ay);
  hemisphere_apply(lv, N, ax, ay, wi, pdf);
}

__device__ __forceinline__ void cosine_hemisphere(float u1, float u2, const float N[3],
                                                  float wi[3], float& pdf) {
  float lv[3];
  hemisphere_local(u1, u2, lv);
  hemisphere_world(lv, N, wi, pdf);
}

// blinnPhong (reflection.h:202-214): li * (kd * costheta + ks * pow(n.h, s))
__device__ __forceinline__ void blinn_phong(float costheta, const float kd[3],
                                            const float ks[3], float shininess,
                                            const float li[3], const float wi[3],
                                            const float n[3], const float wo[3],
                                            float out[3]) {
  float hh[3] = {wi[0] + wo[0], wi[1] + wo[1], wi[2] + wo[2]};
  gnorm3(hh);
  const float ndh = gclamp01(gdot3(n, hh));
  const float pw = pow_r(ndh, shininess);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = li[k] * (kd[k] * costheta + ks[k] * pw);
}

__device__ __forceinline__ bool has_positive(const float v[3]) {
  return v[0] > 0.0f || v[1] > 0.0f || v[2] > 0.0f;
}

// ooc::ShaderPt's point-light term for a camera ray -- path weight (1,1,1),
// one point light, a diffuse surface: the operations of the shading pass
// (frame_kernels.hip, shade_slot) in the same order, so the weight and the
// spawn rule are k_shade's bit for bit.  pos / wi: the shadow ray.
__device__ __forceinline__ bool shade_pt_point(const float o[3], const float d[3],
                                               const spray_rt_hit& h, const ShadePt& sh,
                                               float pos[3], float wi[3], float L[3]) {
  pos[0] = d[0] * h.t + o[0];
  pos[1] = d[1] * h.t + o[1];
  pos[2] = d[2] * h.t + o[2];
  float kd[3];
  unpack_rgb(h.color, kd);
  const float wo[3] = {-d[0], -d[1], -d[2]};
  const float cos_i = gdot3(wo, h.ns);
  float nff[3] = {h.ns[0], h.ns[1], h.ns[2]};
  if (!(cos_i > 0.0f)) {
    nff[0] = -nff[0];
    nff[1] = -nff[1];
    nff[2] = -nff[2];
  }
  gnorm3(nff);
  wi[0] = sh.lp[0] - pos[0];
  wi[1] = sh.lp[1] - pos[1];
  wi[2] = sh.lp[2] - pos[2];
  gnorm3(wi);
  const float ct = gclamp01(gdot3(nff, wi));
  float bp[3];
  blinn_phong(ct, kd, sh.ks, sh.shininess, sh.lr, wi, nff, wo, bp);
  const float sc = 1.0f / 1.0f;  // 1 / pdf of a point light
#pragma unroll
  for (int k = 0; k < 3; ++k) L[k] = (1.0f * bp[k]) * sc;
  return has_positive(L);
}

// ooc::ShaderAo (src/ooc/ooc_shader_ao.h:120-146): nsamples cosine-weighted
// hemisphere directions per hit (DiffuseBsdf::sampleRandom, reflection.h:
// 245-249; getCosineHemisphereSample, sampler.cc:54-60; ConcentricDisk-
// Sampling, sampler.h:49-92; localToWorld, sampler.h:101-110), seeded by
// pixid * (l + 1).  Sample l of hit i is emitted when its radiance weight
// is positive.  Operation order as the oracle (glm), trig rounded once from
// double (shade_device.h), so directions equal the host's bit for bit.
struct AoOut {
  float o[3], w[3];
  bool ok;
};
__device__ __forceinline__ AoOut ao_sample(const spray_rt_ray& ray, const spray_rt_hit& h,
                                           int32_t pixid, int l, int nsamples) {
  AoOut r;
  r.ok = false;
  if (h.domain < 0) return r;
  const float* o = ray.org;
  const float* d = ray.dir;
  r.o[0] = d[0] * h.t + o[0];
  r.o[1] = d[1] * h.t + o[1];
  r.o[2] = d[2] * h.t + o[2];
  const float kd[3] = {float(double((h.color >> 16) & 0xffu) * 0.00392156862745098),
                       float(double((h.color >> 8) & 0xffu) * 0.00392156862745098),
                       float(double(h.color & 0xffu) * 0.00392156862745098)};
  const float wo[3] = {-d[0], -d[1], -d[2]};
  float N[3] = {h.ns[0], h.ns[1], h.ns[2]};
  if (!(gdot3(wo, N) > 0.0f)) {
    N[0] = -N[0];
    N[1] = -N[1];
    N[2] = -N[2];
  }
  gnorm3(N);
  const float ao_w = 1.0f / float(nsamples);
  uint32_t st = sampler_init1(pixid * (l + 1));
  const float u1 = sampler_1d(st), u2 = sampler_1d(st);
  float pdf;
  cosine_hemisphere(u1, u2, N, r.w, pdf);
  float ct = gdot3(N, r.w);
  ct = ct < 0.0f ? 0.0f : (ct > 1.0f ? 1.0f : ct);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (kd[k] * (0.3183098861837907f * ct * ao_w / pdf) > 0.0f) r.ok = true;
  return r;
}

// Whether sample l of a hit yields an AO ray -- ao_sample(...).ok, without
// the trigonometry in the common case.  The concentric-disk radius is
// rr = max(|sx|, |sy|); for rr < 0.999 the local direction has
// lv.z >= 0.0447, so ct = N . w and pdf = lv.z / pi are positive and finite
// and the weight kd * (ct / (pi * ns * pdf)) is positive exactly when a
// colour channel is (kd >= 1/255, the factor is ~1/ns: no underflow) --
// given a finite normalised N.  Otherwise the full sample decides.
__device__ __forceinline__ bool ao_ok(const spray_rt_ray* ray, const spray_rt_hit& h,
                                      int32_t pixid, int l, int nsamples) {
  if (h.domain < 0) return false;
  float N[3] = {h.ns[0], h.ns[1], h.ns[2]};
  gnorm3(N);
  const bool nfin = isfinite(N[0]) && isfinite(N[1]) && isfinite(N[2]);
  uint32_t st = sampler_init1(pixid * (l + 1));
  const float u1 = sampler_1d(st), u2 = sampler_1d(st);
  const float rr = fmaxf(fabsf(2 * u1 - 1), fabsf(2 * u2 - 1));
  if (nfin && rr < 0.999f) return (h.color & 0xFFFFFFu) != 0u;
  return ao_sample(*ray, h, pixid, l, nsamples).ok;  // the ray is read only here
}

}  // namespace
}  // namespace spray_rt
