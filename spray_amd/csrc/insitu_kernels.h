// insitu_kernels.h -- launchers of the in-situ exchange kernels
// (insitu_kernels.hip); the protocol that sequences them is insitu.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_kernels.h"
#include "spray_rt.h"

namespace spray_rt {

constexpr uint64_t kInsituMissKey = 0x7FFFFFFFFFFFFFFFull;  // keyed closest hit: a miss
constexpr size_t kRadRecBytes = 48;                         // org, dir, w, pixid, samid
constexpr size_t kShadowRecBytes = 24;                      // org, dir

// out[j] = radiance record of ray idx[j]
hipError_t launch_pack_rad(hipStream_t s, const spray_rt_ray* rays, const float* w,
                           const int32_t* pix, const int32_t* sam, const int64_t* idx, size_t n,
                           void* out);
hipError_t launch_unpack_rad(hipStream_t s, const void* in, size_t m, spray_rt_ray* rays,
                             float* w, int32_t* pix, int32_t* sam);
// out[j] = shadow record of slot sel[idx[j]]
hipError_t launch_pack_shadow(hipStream_t s, const spray_rt_ray* slots, const uint32_t* sel,
                              const int64_t* idx, size_t n, void* out);
hipError_t launch_unpack_shadow(hipStream_t s, const void* in, size_t m, spray_rt_ray* rays);
// out[j] = slots[sel[j]]
hipError_t launch_gather_shadow(hipStream_t s, const spray_rt_ray* slots, const uint32_t* sel,
                                size_t n, spray_rt_ray* out);
// the rank's own copies without the wire: orays[j] etc. = holder record idx[j]
// as k_unpack_rad leaves it; out[j] = shadow slot sel[idx[j]] as k_unpack_shadow
hipError_t launch_gather_rad(hipStream_t s, const spray_rt_ray* rays, const float* w,
                             const int32_t* pix, const int32_t* sam, const int64_t* idx, size_t n,
                             spray_rt_ray* orays, float* ow, int32_t* opix, int32_t* osam);
hipError_t launch_gather_shadow_self(hipStream_t s, const spray_rt_ray* slots,
                                     const uint32_t* sel, const int64_t* idx, size_t n,
                                     spray_rt_ray* out);
// best[idx[j]] = min(best[idx[j]], keys[j]) over the returned keys
hipError_t launch_key_min(hipStream_t s, const int64_t* idx, const uint64_t* keys, size_t n,
                          uint64_t* best);
hipError_t launch_fill_u64(hipStream_t s, uint64_t* p, size_t n, uint64_t v);
// win[j] = key[j] is a hit and equals the composite minimum best[j]
hipError_t launch_winners(hipStream_t s, const uint64_t* key, const uint64_t* best, size_t m,
                          uint8_t* win);
// occ[sel[idx[j]]] = 1 where ret[j]
hipError_t launch_occ_return(hipStream_t s, const int64_t* idx, const uint8_t* ret, size_t n,
                             const uint32_t* sel, uint8_t* occ);
// image + stride * pix[i] (+0, +1, +2) += the unoccluded weights of copy i;
// tot (optional): {nrad, *nsh, 0} written by the first lane (a fused
// frame's totals without a counters pass)
hipError_t launch_film_atomic(hipStream_t s, float* image, const int32_t* pix, size_t m, int ns,
                              const float* sw, const uint8_t* sv, const uint8_t* occ,
                              double scale, int stride = 4, unsigned long long* tot = nullptr,
                              const uint32_t* nsh = nullptr, unsigned long long nrad = 0);
hipError_t launch_record(hipStream_t s, const uint8_t* win, size_t m, int bounce, int ns,
                         const int32_t* sam, const spray_rt_hit* hits, const uint8_t* sv,
                         const uint8_t* occ, const spray_rt_insitu_rec& rec);
hipError_t launch_gather_next(hipStream_t s, const spray_rt_ray* rays, const float* w,
                              const int32_t* pix, const int32_t* sam, const uint32_t* sel,
                              size_t n, spray_rt_ray* orays, float* ow, int32_t* opix,
                              int32_t* osam);
hipError_t launch_weights_one(hipStream_t s, float* w, size_t n);
// win[i] = (valid == null || valid[i]) && hits[i] is a hit
hipError_t launch_hit_flags(hipStream_t s, const uint8_t* valid, const spray_rt_hit* hits,
                            size_t n, uint8_t* win);
// ---- replicated-ray frames (insitu.cpp, trace_replicated) ----
// scene bounding box (the replicated frame's cull)
struct SceneBox {
  float lo[3], hi[3];
};
// fc[i] = ray i enters the box (or has a zero direction component)
hipError_t launch_rep_cull(hipStream_t s, const spray_rt_ray* rays, size_t n, const SceneBox& b,
                           uint8_t* fc);
// lp[j] = list position of keys[j] where its t bits equal tmin[j], else 0xFF
hipError_t launch_rep_lp(hipStream_t s, const uint64_t* keys, const uint32_t* tmin, size_t nc,
                         uint8_t* lp);
// The winners' shadow count: kWinCounters u64 counters kWinStride u64
// apart (one block adds to counter blockIdx % kWinCounters: a pass over C'
// with one address would serialise ~nc / 64 atomics at one L2 channel);
// launch_rep_totals sums them.  Zero kWinCounterBytes before the pass.
constexpr int kWinCounters = 64;
constexpr int kWinStride = 32;  // 256 B
constexpr size_t kWinCounterBytes = size_t(kWinCounters) * kWinStride * 8;
// win[j] = keys[j] is the group's minimum (t bits == tmin and list position
// == lpmin, or, lpmin null, keys == kmin); svw = win && sv; nshadow += svw
hipError_t launch_rep_win(hipStream_t s, const uint64_t* keys, const uint32_t* tmin,
                          const uint8_t* lpmin, const uint64_t* kmin, const uint8_t* sv, size_t nc,
                          uint8_t* win, uint8_t* svw, unsigned long long* nshadow);
// ---- replicated PT frames from the camera (trace_camera): passes over the
// rank's eye table T, the shared arrays addressed by U slot (rt_kernels.h)
// lp[u] = own list position where own t bits tk[u] == tmin[u] (lp prefilled
// 0xFF); defer (the keyed launch's defer_lp): the position computed here on
// the regenerated eye ray (the domain boxes and the top-level tree over them)
// and written into the key
hipError_t launch_cam_lp(hipStream_t s, const CamTable& T, int spp, uint64_t* keys,
                        const uint32_t* tk, const uint32_t* tmin, uint8_t* lp,
                        const CamFrame* defer, const float* boxes, const BvhNode* tlas,
                        int ntlas);
// win / svw at u as launch_rep_win (own t bits tk: 0xFFFFFFFF = no own hit)
hipError_t launch_cam_win(hipStream_t s, const CamTable& T, int spp, const uint64_t* keys,
                         const uint32_t* tk, const uint32_t* tmin, const uint8_t* lpmin,
                         const uint64_t* kmin, const uint8_t* sv, uint8_t* win, uint8_t* svw,
                         unsigned long long* nshadow);
// compact[3 q ..] += scale * sw of the unoccluded winners' shadows, q = u / spp
hipError_t launch_cam_film(hipStream_t s, const CamTable& T, int spp, float* compact,
                          const float* sw, const uint8_t* svw, const uint8_t* occ, double scale);
// image pixel of U pixel q += compact[3 q ..] (U: the frame's U table)
hipError_t launch_cam_expand(hipStream_t s, const CamTable& U, int image_w, const float* compact,
                            float* image);
hipError_t launch_cam_record(hipStream_t s, const CamTable& T, int spp, int image_w,
                            const uint8_t* win, const spray_rt_hit* hits, const uint8_t* svw,
                            const uint8_t* occ, const spray_rt_insitu_rec& rec);
// eye rays, pixel and sample ids of table T's work items at their U slots
hipError_t launch_cam_eye_rays(hipStream_t s, const CamTable& T, const CamFrame& F,
                              spray_rt_ray* rays, int32_t* pixid, int32_t* samid);
// tmin[j] = t bits of kmin[j] (0xFFFFFFFF: a miss)
hipError_t launch_tmin_from_keys(hipStream_t s, const uint64_t* kmin, size_t nc, uint32_t* tmin);
// *out = max(pix[0..n)) (bmax: grid_for(n) u32 of scratch)
hipError_t launch_pix_max(hipStream_t s, const int32_t* pix, size_t n, uint32_t* bmax,
                          uint32_t* out);
// dst[j] = src[idx[j]]
hipError_t launch_gather_i32(hipStream_t s, const uint32_t* idx, size_t n, const int32_t* src,
                             int32_t* dst);
// The compact film's slots: the runs of equal pixels along C.  slot_c[j] =
// run of ray j, slot_pix[run] = its pixel, *d_np = runs; incl: [nc] u32
// scratch; temp == nullptr: *temp_bytes <- the scan's scratch size.
hipError_t launch_rep_slots(hipStream_t s, const uint32_t* idx_c, const int32_t* pix, size_t nc,
                            uint32_t* incl, void* temp, size_t* temp_bytes,
                            int32_t* slot_c, int32_t* slot_pix, uint32_t* d_np);
// image[4 slot_pix[q] + k] += compact[3 q + k], q < np
hipError_t launch_rep_expand(hipStream_t s, float* image, const int32_t* slot_pix,
                             const float* compact, size_t np);
// tail[64 c + k] = bit k of {nrad, the nshadow counters' sum, 0}[c] (192 bytes)
// Image frames' interleaved bands (band b of the frame = rows b * band16 * 16
// bytes on; rank r holds bands r, r + W, ...): pack = 1 copies rank r0's
// bands from the image into pk (its bands in order); pack = 0 copies ranks
// r0 .. r0 + nr - 1's segments of the gathered pk (rank k's bands at
// k * bands * band16 uint4) into the image.  One launch for every band.
hipError_t launch_bands_copy(hipStream_t s, float* image, void* pk, int W, int bands,
                             size_t band_bytes, int r0, int nr, int pack);
// Image frames' compact gather: the RGB of table T's pixels (footprint.h
// runs, in table order) packed from / unpacked into the image, 12 B a pixel
hipError_t launch_pack_rgb(hipStream_t s, const CamTable& T, int image_w, const float* image,
                           float* out);
hipError_t launch_unpack_rgb(hipStream_t s, const CamTable& T, int image_w, const float* in,
                             float* image);
// tot = {stats[3] (live slots shaded), stats[1] (shadows), stats[0] (aborts)}
hipError_t launch_totals_of_stats(hipStream_t s, const unsigned long long* stats,
                                  unsigned long long* tot);
hipError_t launch_rep_totals(hipStream_t s, uint8_t* tail, unsigned long long nrad,
                             const unsigned long long* nshadow);
// ---- replicated-ray AO frames (insitu.cpp, trace_replicated_ao) ----
struct RepAoArgs {
  size_t nc;
  int rank;
  int ns;                       // AO samples per hit (<= 32)
  int fb;                       // bits per occlusion count field (2, 4 or 8)
  const uint32_t* idx_c;        // [nc] ray ids of C
  const uint64_t* keys_c;       // [nc] winning keys (after the MIN all-reduce)
  const uint64_t* keys_n;       // [nc] this rank's keys
  const uint64_t* mask;         // unused
  const float4* rays;           // [n] eye rays (32 B)
  const spray_rt_hit* hits_n;   // [nc] this rank's hit records
  const int32_t* pix;           // [n]
  const int32_t* sam;           // [n]
  uint4* pub;                   // [nc] winner's normal bits + colour, zeros elsewhere
  uint8_t* win;                 // [nc] 1: this rank won ray j
  float4* rays_c;               // [nc] C's rays (32 B)
  int32_t* pix_c;               // [nc]
  int32_t* sam_c;               // [nc]
  spray_rt_hit* hit_c;          // [nc] winners' hit records (optional: records)
  spray_rt_hit* hits_all;       // [nc] every ray's hit as the group sees it
  const float4* rec_ao;         // [nc] AO spawn records (launch_spawn_ao_pairs)
  const float4* lv;             // (pixel, sample) table (launch_spawn_ao_pairs)
  const uint32_t* fields;       // occlusion count fields, position j * ns + l
};
hipError_t launch_rep_ao_publish(hipStream_t s, const RepAoArgs& a);
hipError_t launch_rep_ao_hits(hipStream_t s, const RepAoArgs& a);
// bits[w] bit b = occ[32 w + b] != 0 for k = 32 w + b < n
hipError_t launch_pack_bits(hipStream_t s, const uint8_t* occ, size_t n, uint32_t* bits);
hipError_t launch_rep_ao_film(hipStream_t s, const RepAoArgs& a, float* image, double scale);
// camera frames: the film of U pixels [q0, q1) into compact (3 floats per U
// pixel; slot j of pixel q = q spp + sample), the other pixels untouched
hipError_t launch_rep_ao_film_pix(hipStream_t s, const RepAoArgs& a, int spp, size_t q0,
                                  size_t q1, float* compact, double scale);
hipError_t launch_rep_ao_record(hipStream_t s, const RepAoArgs& a, const spray_rt_insitu_rec& rec);
// counts[r] = starts[r + 1] - starts[r], r < world (<= 64)
hipError_t launch_counts_from_starts(hipStream_t s, const int64_t* starts, int world,
                                     int64_t* counts);

}  // namespace spray_rt
