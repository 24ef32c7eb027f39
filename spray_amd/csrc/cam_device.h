// cam_device.h -- the eye rays of the replicated in-situ frames generated
// in the lanes (insitu.cpp trace_camera): camera record, jitter and the
// run tables that map a launch's work items to pixels and U slots.  The same
// operations as k_eye_rays_insitu, so the rays are bit-identical.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_kernels.h"
#include "shade_device.h"

namespace spray_rt {
namespace {

// ---- the replicated frames' camera rays (trace_camera) ---------------------
// Camera record (camera_init): eye, image-plane corner, u and v axes, w, h.
struct Cam {
  float p[14];
};
// Camera::generateRay (camera.h:168-209), glm operand order: the normalised
// direction through image point (fx, fy)
__device__ __forceinline__ void cam_dir(const Cam& cam, float fx, float fy, float* d) {
  const float* c = cam.p;
  const float u = fx / c[12], v = fy / c[13];
  float dx = ((c[3] + c[6] * u) + c[9] * v) - c[0];
  float dy = ((c[4] + c[7] * u) + c[10] * v) - c[1];
  float dz = ((c[5] + c[8] * u) + c[11] * v) - c[2];
  const float inv = 1.0f / sqrtf((dx * dx + dy * dy) + dz * dz);
  d[0] = dx * inv;
  d[1] = dy * inv;
  d[2] = dz * inv;
}
// insitu::genMultiSampleEyeRays (insitu_ray.h:103-182): sample s of pixel
// (x, y) jittered by the (pixid, s) seed; one sample per pixel: the corner
__device__ __forceinline__ void insitu_jitter(int image_w, int spp, int x, int y, int s,
                                              float& fx, float& fy) {
  fx = float(x);
  fy = float(y);
  if (spp > 1) {
    uint32_t st = mm_fin(mm_mix(mm_mix(0u, uint32_t(image_w * y + x)), uint32_t(s)));
    fx = float(x) + sampler_1d(st);
    fy = float(y) + sampler_1d(st);
  }
}
// Work item j of run table T (CamTable): its pixel (x, y), sample s and U slot
__device__ __forceinline__ void cam_item(const CamTable& T, int spp, size_t j, int& x, int& y,
                                         int& s, size_t& slot) {
  const uint32_t pj = uint32_t(j / uint32_t(spp));
  s = int(j - size_t(pj) * uint32_t(spp));
  uint32_t r = T.first[pj >> 3];
  while (T.runs[r + 1].pbase <= pj) ++r;  // the sentinel run ends the scan
  const CamRun run = T.runs[r];
  const uint32_t off = pj - run.pbase;
  x = run.x0 + int(off);
  y = run.y;
  slot = size_t(run.ubase + off) * uint32_t(spp) + uint32_t(s);
}

}  // namespace
}  // namespace spray_rt
