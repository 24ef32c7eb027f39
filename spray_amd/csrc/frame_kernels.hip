// frame_kernels.hip -- gfx950 kernels of the frame layer around the hot
// path: the path-shading pass (ooc::ShaderPt / ooc::ShaderAo) and the film
// (TContext::retire + HdrImage::add).  Both are positional: path slot i keeps
// its index for the whole frame, shadow k of slot i sits at i*ns + k, so the
// film can sum a pixel's contributions in a fixed order without atomics.
//
// Every operation restates oracle/oracle.c (or_shade, or_film) in the same
// order; -ffp-contract=off, trig/pow rounded once from double
// (shade_device.h): the image is bit-identical to the CPU oracle's.
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "shade_device.h"

namespace spray_rt {
namespace {

struct ShadeCount {
  uint32_t bad = 0, shadows = 0, next = 0, live = 0;
};
__device__ __forceinline__ void emit_shadow(spray_rt_ray* sh, float4* sw, uint8_t* sv,
                                            ShadeCount& cnt, size_t j, const float pos[3],
                                            const float wi[3], const float L[3]) {
  float4* op = reinterpret_cast<float4*>(sh + j);
  op[0] = make_float4(pos[0], pos[1], pos[2], kRayEpsilon);
  op[1] = make_float4(wi[0], wi[1], wi[2], kInf);
  sw[j] = make_float4(L[0], L[1], L[2], 0.f);
  sv[j] = 1;
  ++cnt.shadows;
}

// FrDielectric / Refract (src/render/reflection.h:134-172)
__device__ __forceinline__ float fr_dielectric(float cosI, float etaI, float etaT,
                                               const float wo[3], const float nff[3],
                                               float wt[3], bool& tir) {
  const float sin2I = fmaxf(0.0f, 1.0f - (cosI * cosI));
  const float eta = etaI / etaT;
  const float sin2T = eta * eta * sin2I;
  tir = sin2T >= 1.0f;
  if (tir) return 1.0f;
  const float cosT = sqrtf(1.0f - sin2T);
  const float rparl = ((etaT * cosI) - (etaI * cosT)) / ((etaT * cosI) + (etaI * cosT));
  const float rperp = ((etaI * cosI) - (etaT * cosT)) / ((etaI * cosI) + (etaT * cosT));
  const float a = eta * cosI - cosT;
#pragma unroll
  for (int k = 0; k < 3; ++k) wt[k] = (eta * -wo[k]) + (nff[k] * a);
  return (rparl * rparl + rperp * rperp) / 2.0f;
}

// One shading pass (src/ooc/ooc_shader_pt.h:93-227, ooc_shader_ao.h:92-197)
// at next_actual_depth = bounce + 1: the exact resolution needs no
// speculative history (ooc_vbuf.cc), so the reference's ray_depth +
// rayin.depth + 1 is the bounce count.
__device__ __forceinline__ void shade_slot(
    const spray_rt_shader& P, const spray_rt_bsdf* __restrict__ bsdfs, int nbsdf, int bounce,
    int ns, spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    float4* __restrict__ w, uint8_t* __restrict__ valid, const int32_t* __restrict__ pixid,
    const int32_t* __restrict__ samid, size_t i, spray_rt_ray* __restrict__ sh,
    float4* __restrict__ sw, uint8_t* __restrict__ sv, ShadeCount& cnt) {
  for (int k = 0; k < ns; ++k) sv[i * ns + k] = 0;
  if (!valid[i]) return;
  valid[i] = 0;
  ++cnt.live;
  const spray_rt_hit h = hits[i];
  if (h.domain < 0) return;
  const spray_rt_ray r = rays[i];
  const float* o = r.org;
  const float* d = r.dir;
  const float pos[3] = {d[0] * h.t + o[0], d[1] * h.t + o[1], d[2] * h.t + o[2]};
  float kd[3];
  unpack_rgb(h.color, kd);
  const float wo[3] = {-d[0], -d[1], -d[2]};
  const float4 w4 = w[i];
  const float Lin[3] = {w4.x, w4.y, w4.z};
  const float cos_i = gdot3(wo, h.ns);
  const bool entering = cos_i > 0.0f;
  float nff[3] = {h.ns[0], h.ns[1], h.ns[2]};
  if (!entering) {
    nff[0] = -nff[0];
    nff[1] = -nff[1];
    nff[2] = -nff[2];
  }
  gnorm3(nff);
  spray_rt_bsdf bs;
  bs.type = SPRAY_RT_BSDF_DIFFUSE;
  bs.p[0] = bs.p[1] = bs.p[2] = 0.f;
  if (bsdfs && h.domain < nbsdf) bs = bsdfs[h.domain];
  const bool delta = bs.type != SPRAY_RT_BSDF_DIFFUSE;
  const int nad = bounce + 1;
  float wi[3], pdf;
  if (P.shader == SPRAY_RT_SHADER_AO) {
    if (delta) {
      ++cnt.bad;
    } else {
      const float ao_w = 1.0f / float(P.samples);
      for (int l = 0; l < P.samples; ++l) {
        uint32_t st = sampler_init1(pixid[i] * (l + 1));
        const float u1 = sampler_1d(st), u2 = sampler_1d(st);
        cosine_hemisphere(u1, u2, nff, wi, pdf);
        const float ct = gclamp01(gdot3(nff, wi));
        const float s = 0.3183098861837907f * ct * ao_w / pdf;
        const float L[3] = {(Lin[0] * kd[0]) * s, (Lin[1] * kd[1]) * s, (Lin[2] * kd[2]) * s};
        if (has_positive(L)) emit_shadow(sh, sw, sv, cnt, i * ns + l, pos, wi, L);
      }
    }
  } else if (!delta) {
    uint32_t st = sampler_init1(samid[i] * nad);
    int k = 0;
    for (int l = 0; l < P.nlights; ++l) {
      const spray_rt_light& lt = P.lights[l];
      if (lt.type == SPRAY_RT_LIGHT_HEMISPHERE) {
        for (int s = 0; s < P.samples; ++s, ++k) {
          const float u1 = sampler_1d(st), u2 = sampler_1d(st);
          cosine_hemisphere(u1, u2, nff, wi, pdf);
          if (pdf > 0.0f) {
            const float ct = gclamp01(gdot3(nff, wi));
            float bp[3];
            blinn_phong(ct, kd, P.ks, P.shininess, lt.radiance, wi, nff, wo, bp);
            const float sc = 1.0f / (pdf * float(P.samples));
            const float L[3] = {(Lin[0] * bp[0]) * sc, (Lin[1] * bp[1]) * sc,
                                (Lin[2] * bp[2]) * sc};
            if (has_positive(L)) emit_shadow(sh, sw, sv, cnt, i * ns + k, pos, wi, L);
          }
        }
      } else {
        wi[0] = lt.pos[0] - pos[0];
        wi[1] = lt.pos[1] - pos[1];
        wi[2] = lt.pos[2] - pos[2];
        gnorm3(wi);
        pdf = 1.0f;
        const float ct = gclamp01(gdot3(nff, wi));
        float bp[3];
        blinn_phong(ct, kd, P.ks, P.shininess, lt.radiance, wi, nff, wo, bp);
        const float sc = 1.0f / pdf;
        const float L[3] = {(Lin[0] * bp[0]) * sc, (Lin[1] * bp[1]) * sc,
                            (Lin[2] * bp[2]) * sc};
        if (has_positive(L)) emit_shadow(sh, sw, sv, cnt, i * ns + k, pos, wi, L);
        ++k;
      }
    }
  }
  if (nad >= P.bounces) return;
  float won[3] = {wo[0], wo[1], wo[2]};
  gnorm3(won);
  float nw[3] = {0.f, 0.f, 0.f};
  bool emit = false;
  if (delta) {
    if (cos_i != 0.0f) {
      float c = cos_i < -1.0f ? -1.0f : (cos_i > 1.0f ? 1.0f : cos_i);
      const float ac = fabsf(c);
      if (!entering) c = ac;
      bool refl = false, trans = false;
      float fr = 0.0f;
      float wt[3] = {0.f, 0.f, 0.f};
      const float eI = entering ? bs.p[0] : bs.p[1], eT = entering ? bs.p[1] : bs.p[0];
      if (bs.type == SPRAY_RT_BSDF_MIRROR) {
        fr = 1.0f;
        refl = true;
      } else if (bs.type == SPRAY_RT_BSDF_GLASS) {
        bool tir;
        fr = fr_dielectric(c, eI, eT, won, nff, wt, tir);
        if (fr == 1.0f) {
          refl = true;
        } else if (fr == 0.0f) {
          trans = true;
        } else {
          refl = trans = true;
        }
      } else {
        bool tir;
        fr_dielectric(c, eI, eT, won, nff, wt, tir);
        if (tir) {
          refl = true;
          fr = 1.0f;
        } else {
          trans = true;
          fr = 0.0f;
        }
      }
      if (refl && trans) {
        ++cnt.bad;
      } else if (refl) {
        const float s2 = 2.0f * gdot3(won, nff);
        wi[0] = -won[0] + s2 * nff[0];
        wi[1] = -won[1] + s2 * nff[1];
        wi[2] = -won[2] + s2 * nff[2];
        gnorm3(wi);
        const float s = fr / ac;
        nw[0] = Lin[0] * s;
        nw[1] = Lin[1] * s;
        nw[2] = Lin[2] * s;
        emit = has_positive(nw);
      } else if (trans) {
        wi[0] = wt[0];
        wi[1] = wt[1];
        wi[2] = wt[2];
        gnorm3(wi);
        const float s = (1.0f - fr) / ac;
        nw[0] = Lin[0] * s;
        nw[1] = Lin[1] * s;
        nw[2] = Lin[2] * s;
        emit = has_positive(nw);
      }
    }
  } else {
    uint32_t st = sampler_init1(samid[i] * nad);
    const float u1 = sampler_1d(st), u2 = sampler_1d(st);
    cosine_hemisphere(u1, u2, nff, wi, pdf);
    const float ct = gclamp01(gdot3(nff, wi));
#pragma unroll
    for (int k = 0; k < 3; ++k) nw[k] = (((Lin[k] * kd[k]) * kOneOverPi) * ct) / pdf;
    emit = has_positive(nw);
  }
  if (emit) {
    float4* rp = reinterpret_cast<float4*>(rays + i);
    rp[0] = make_float4(pos[0], pos[1], pos[2], kRayEpsilon);
    rp[1] = make_float4(wi[0], wi[1], wi[2], kInf);
    w[i] = make_float4(nw[0], nw[1], nw[2], 0.f);
    valid[i] = 1;
    ++cnt.next;
  }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// stats[4] += {reference-abort cases, shadows spawned, next radiance rays,
// live slots shaded (= radiance rays traced this bounce)}
// stats: 4 counters, each striped over `stripes` words (counter k of block b
// at stats[k * stripes + b % stripes]: same-address atomics serialise in L2,
// one word per counter put a ~200 us floor under a 1M-slot launch); the
// block sums first, one atomic per counter per block.
__global__ __launch_bounds__(kBlock) void k_shade(
    spray_rt_shader P, const spray_rt_bsdf* __restrict__ bsdfs, int nbsdf, int bounce,
    int ns, spray_rt_ray* __restrict__ rays, const spray_rt_hit* __restrict__ hits,
    float4* __restrict__ w, uint8_t* __restrict__ valid, const int32_t* __restrict__ pixid,
    const int32_t* __restrict__ samid, size_t M, spray_rt_ray* __restrict__ sh,
    float4* __restrict__ sw, uint8_t* __restrict__ sv, unsigned long long* __restrict__ stats,
    int stripes) {
  __shared__ uint32_t part[kBlock / 64][4];
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  ShadeCount cnt;
  if (i < M)
    shade_slot(P, bsdfs, nbsdf, bounce, ns, rays, hits, w, valid, pixid, samid, i, sh, sw, sv,
               cnt);
  if (!stats) return;
  const uint32_t v[4] = {wave_sum(cnt.bad), wave_sum(cnt.shadows), wave_sum(cnt.next),
                         wave_sum(cnt.live)};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0)
    for (int k = 0; k < 4; ++k) part[wave][k] = v[k];
  __syncthreads();
  if (threadIdx.x < 4) {
    uint32_t t = 0;
    for (int x = 0; x < kBlock / 64; ++x) t += part[x][threadIdx.x];
    if (t)
      atomicAdd(stats + threadIdx.x * stripes + blockIdx.x % unsigned(stripes),
                (unsigned long long)t);
  }
}

// path weights (1, 1, 1) and all slots live: the camera rays of a tile
__global__ __launch_bounds__(kBlock) void k_path_init(float4* __restrict__ w,
                                                      uint8_t* __restrict__ valid, size_t M) {
  const size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= M) return;
  w[i] = make_float4(1.f, 1.f, 1.f, 0.f);
  valid[i] = 1;
}

// TContext::retire + HdrImage::add(pixid, w, double scale): one thread per
// pixel group of spp slots, adds in slot then shadow order.
__global__ __launch_bounds__(kBlock) void k_film(float4* __restrict__ image,
                                                 const int32_t* __restrict__ pixid,
                                                 size_t ngroups, int spp, int ns,
                                                 const float4* __restrict__ sw,
                                                 const uint8_t* __restrict__ sv,
                                                 const uint8_t* __restrict__ occ,
                                                 double scale) {
  const size_t g = size_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= ngroups) return;
  const size_t i0 = g * size_t(spp);
  const size_t per = size_t(spp) * ns;
  bool any = false;
  for (size_t j = i0 * ns; j < i0 * ns + per; ++j) any |= sv[j] && !occ[j];
  if (!any) return;
  const int32_t p = pixid[i0];
  float4 px = image[p];
  for (size_t j = i0 * ns; j < i0 * ns + per; ++j) {
    if (!sv[j] || occ[j]) continue;
    const float4 L = sw[j];
    px.x = float(double(px.x) + scale * double(L.x));
    px.y = float(double(px.y) + scale * double(L.y));
    px.z = float(double(px.z) + scale * double(L.z));
  }
  image[p] = px;
}

}  // namespace

hipError_t launch_shade(hipStream_t s, const spray_rt_shader& P, const spray_rt_bsdf* bsdfs,
                        int nbsdf, int bounce, int ns, spray_rt_ray* rays,
                        const spray_rt_hit* hits, float* w, uint8_t* valid,
                        const int32_t* pixid, const int32_t* samid, size_t M,
                        spray_rt_ray* shadows, float* sw, uint8_t* svalid,
                        unsigned long long* stats, int stripes) {
  if (M == 0) return hipSuccess;
  k_shade<<<grid_for(M), kBlock, 0, s>>>(P, bsdfs, nbsdf, bounce, ns, rays, hits,
                                         reinterpret_cast<float4*>(w), valid, pixid, samid, M,
                                         shadows, reinterpret_cast<float4*>(sw), svalid, stats,
                                         stripes < 1 ? 1 : stripes);
  return hipGetLastError();
}

hipError_t launch_path_init(hipStream_t s, float* w, uint8_t* valid, size_t M) {
  if (M == 0) return hipSuccess;
  k_path_init<<<grid_for(M), kBlock, 0, s>>>(reinterpret_cast<float4*>(w), valid, M);
  return hipGetLastError();
}

hipError_t launch_film(hipStream_t s, float* image, const int32_t* pixid, size_t M, int spp,
                       int ns, const float* sw, const uint8_t* svalid, const uint8_t* occ,
                       double scale) {
  const size_t ng = M / size_t(spp);
  if (ng == 0) return hipSuccess;
  k_film<<<grid_for(ng), kBlock, 0, s>>>(reinterpret_cast<float4*>(image), pixid, ng, spp, ns,
                                         reinterpret_cast<const float4*>(sw), svalid, occ,
                                         scale);
  return hipGetLastError();
}

}  // namespace spray_rt
