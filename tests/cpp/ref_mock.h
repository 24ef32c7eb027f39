// ref_mock.h -- stand-ins for the reference application's own types, for
// tests/cpp/scene_adapter_test.cpp (test infrastructure, not product).
//
// The reference's tracers and shaders hold the scene's lights and materials
// as spray::Light* / const spray::Bsdf* (src/render/light.h:31-89,
// reflection.h:219-364) over glm.  Neither glm nor those files exist in this
// image, so this header restates the few pieces a shader touches -- a glm
// subset with glm's operand order, the RandomSampler, cosine-hemisphere
// sampling (sampler.h:49-128, sampler.cc:54-60), the two lights, the diffuse
// and mirror BSDFs -- and a ShaderPt whose body uses the reference's own
// expressions against SceneT (ooc_shader_pt.h:45-52, 99-226):
//
//   lights_ = scene->getLights();                  // std::vector<Light*>
//   lights_[l]->isAreaLight(); lights_[l]->sample(pos, &wi, &pdf);
//   lights_[l]->sampleArea(light_sampler, normal_ff, &wi, &pdf);
//   const Bsdf *bsdf = scene_->getBsdf(domain_id); bsdf->isDelta();
//   bsdf->sampleRandom(normal_ff, &sampler, &wi, &pdf);
//
// Transcendentals are rounded once from double, as the oracle's are
// (DESIGN.md section 1), so the shader's output is comparable bit for bit
// with or_shade.  Build with -ffp-contract=off.
#pragma once

#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "spray_scene.hpp"

// Embree 2's opaque scene handle (embree2/rtcore_scene.h), which the
// reference's Scene::SceneInfo holds (src/render/scene.h:57-60).
typedef struct __RTCScene* RTCScene;

namespace glm {

struct vec2 {
  float x, y;
  vec2(float a, float b) : x(a), y(b) {}
};
struct vec3 {
  float x = 0, y = 0, z = 0;
  vec3() = default;
  explicit vec3(float s) : x(s), y(s), z(s) {}
  vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  const float& operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline vec3 operator-(const vec3& a) { return vec3(-a.x, -a.y, -a.z); }
inline vec3 operator*(const vec3& a, const vec3& b) { return vec3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline vec3 operator*(const vec3& a, float s) { return vec3(a.x * s, a.y * s, a.z * s); }
inline vec3 operator*(float s, const vec3& a) { return vec3(s * a.x, s * a.y, s * a.z); }
inline vec3 operator/(const vec3& a, float s) { return vec3(a.x / s, a.y / s, a.z / s); }
inline float dot(const vec3& a, const vec3& b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline vec3 cross(const vec3& a, const vec3& b) {
  return vec3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline vec3 normalize(const vec3& v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float max(float a, float b) { return a < b ? b : a; }
inline float min(float a, float b) { return b < a ? b : a; }
inline float clamp(float x, float lo, float hi) { return min(max(x, lo), hi); }
inline float sqrt(float x) { return std::sqrt(x); }
inline float abs(float x) { return std::fabs(x); }
inline float cos(float x) { return float(std::cos(double(x))); }
inline float sin(float x) { return float(std::sin(double(x))); }
inline float pow(float x, float y) { return float(std::pow(double(x), double(y))); }

}  // namespace glm

namespace spray {

// Scene::SceneInfo as the reference declares it (scene.h:57-60); the
// tracers hold `spray::SceneInfo sinfo_` (ooc_pcontext.h:83) and pass
// sinfo.rtc_scene / sinfo.cache_block to the scene (ooc_tcontext.inl:37,
// 59, 79).  The adapter takes it as is: its handle carries the slot.
struct SceneInfo {
  RTCScene rtc_scene;
  int cache_block;
};

#define MOCK_SPRAY_PI 3.14159265358979323846       // SPRAY_PI = M_PI (spray.h:48)
#define MOCK_SPRAY_ONE_OVER_PI 0.3183098861837907f  // spray.h:50
#define MOCK_SPRAY_1_OVER_255 0.00392156862745098   // spray.h:54

// deps/embree/random_sampler.h:30-113
struct RandomSampler {
  uint32_t s;
};
inline uint32_t murmur_mix(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = (k << 15) | (k >> 17);
  k *= 0x1b873593u;
  h ^= k;
  return ((h << 13) | (h >> 19)) * 5u + 0xe6546b64u;
}
inline void RandomSampler_init(RandomSampler& self, int id) {
  uint32_t h = murmur_mix(0u, uint32_t(id));
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  self.s = h;
}
inline float RandomSampler_get1D(RandomSampler& self) {
  self.s = self.s * 1664525u + 1013904223u;
  return float(int(self.s >> 1)) * 4.656612873077392578125e-10f;
}
inline glm::vec2 RandomSampler_get2D(RandomSampler& self) {
  const float u = RandomSampler_get1D(self);
  const float v = RandomSampler_get1D(self);
  return glm::vec2(u, v);
}

// getCosineHemisphereSample (sampler.cc:54-60): concentric disk, lifted,
// normalised, rotated into N's frame (localToWorld, sampler.h:104-115)
inline void getCosineHemisphereSample(float u1, float u2, const glm::vec3& N, glm::vec3* wi,
                                      float* pdf) {
  glm::vec3 v;
  const float sx = 2 * u1 - 1, sy = 2 * u2 - 1;
  if (!(sx == 0.0 && sy == 0.0)) {
    float r, theta;
    if (sx >= -sy) {
      if (sx > sy) {
        r = sx;
        theta = sy > 0.0 ? sy / r : 8.0f + sy / r;
      } else {
        r = sy;
        theta = 2.0f - sx / r;
      }
    } else if (sx <= sy) {
      r = -sx;
      theta = 4.0f - sy / r;
    } else {
      r = -sy;
      theta = 6.0f + sx / r;
    }
    theta *= MOCK_SPRAY_PI / 4.f;
    v.x = r * glm::cos(theta);
    v.y = r * glm::sin(theta);
  }
  v.z = glm::sqrt(glm::max(0.f, 1.f - v.x * v.x - v.y * v.y));
  v = glm::normalize(v);
  const glm::vec3 dx0(0, N.z, -N.y), dx1(-N.z, 0, N.x);
  const glm::vec3 dx = glm::normalize(glm::dot(dx0, dx0) > glm::dot(dx1, dx1) ? dx0 : dx1);
  const glm::vec3 dy = glm::normalize(glm::cross(N, dx));
  *wi = glm::normalize(dx * v.x + dy * v.y + N * v.z);  // mat3(dx, dy, N) * v
  *pdf = v.z * MOCK_SPRAY_ONE_OVER_PI;
}

class Light {
 public:
  virtual ~Light() {}
  virtual glm::vec3 sample(const glm::vec3& p, glm::vec3* wi, float* pdf) const = 0;
  virtual bool isAreaLight() const = 0;
  virtual glm::vec3 sampleArea(RandomSampler& sampler, const glm::vec3& normal, glm::vec3* wi,
                               float* pdf) const = 0;
};
class PointLight : public Light {
 public:
  PointLight(const glm::vec3& p, const glm::vec3& r) : position_(p), radiance_(r) {}
  glm::vec3 sample(const glm::vec3& p, glm::vec3* wi, float* pdf) const override {
    *wi = glm::normalize(position_ - p);
    *pdf = 1.0;
    return radiance_;
  }
  bool isAreaLight() const override { return false; }
  glm::vec3 sampleArea(RandomSampler&, const glm::vec3&, glm::vec3*, float*) const override {
    throw std::logic_error("forbidden");
  }

 private:
  glm::vec3 position_, radiance_;
};
class DiffuseHemisphereLight : public Light {
 public:
  explicit DiffuseHemisphereLight(const glm::vec3& r) : radiance_(r) {}
  bool isAreaLight() const override { return true; }
  glm::vec3 sample(const glm::vec3&, glm::vec3*, float*) const override {
    throw std::logic_error("forbidden");
  }
  glm::vec3 sampleArea(RandomSampler& sampler, const glm::vec3& normal, glm::vec3* wi,
                       float* pdf) const override {
    glm::vec2 u = RandomSampler_get2D(sampler);
    getCosineHemisphereSample(u.x, u.y, normal, wi, pdf);
    return radiance_;
  }

 private:
  glm::vec3 radiance_;
};

class Bsdf {
 public:
  virtual ~Bsdf() {}
  virtual void sampleRandom(const glm::vec3& normal, RandomSampler* sampler, glm::vec3* wi,
                            float* pdf) const = 0;
  virtual bool isDelta() const = 0;
};
class DiffuseBsdf : public Bsdf {
 public:
  explicit DiffuseBsdf(const glm::vec3& albedo) : albedo_(albedo) {}
  void sampleRandom(const glm::vec3& normal, RandomSampler* sampler, glm::vec3* wi,
                    float* pdf) const override {
    glm::vec2 u = RandomSampler_get2D(*sampler);
    getCosineHemisphereSample(u.x, u.y, normal, wi, pdf);
  }
  bool isDelta() const override { return false; }

 private:
  glm::vec3 albedo_;
};
class DeltaBsdf : public Bsdf {  // mirror / glass / transmission: not sampled here
 public:
  void sampleRandom(const glm::vec3&, RandomSampler*, glm::vec3*, float*) const override {
    throw std::logic_error("forbidden");
  }
  bool isDelta() const override { return true; }
};

struct Aabb {
  glm::vec3 bounds[2];
};

// reflection.h:202-214
inline glm::vec3 blinnPhong(float costheta, const glm::vec3 kd, const glm::vec3 ks,
                            float shininess, const glm::vec3& li, const glm::vec3& wi,
                            const glm::vec3& n_hat, const glm::vec3 wo) {
  glm::vec3 half_hat = glm::normalize(wi + wo);
  float n_dot_h = glm::clamp(glm::dot(n_hat, half_hat), 0.0f, 1.0f);
  glm::vec3 cs = ks * glm::pow(n_dot_h, shininess);
  glm::vec3 cd = kd * costheta;
  return li * (cd + cs);
}
inline bool hasPositive(const glm::vec3& v) { return v.x > 0.0f || v.y > 0.0f || v.z > 0.0f; }

// the application's type policy for spray_amd::Scene<Types>
struct RefTypes {
  typedef spray::Light Light;
  typedef spray::Bsdf Bsdf;
  typedef spray::Aabb Aabb;
  static Light* makeLight(const spray_amd::LightDesc& d) {
    const glm::vec3 r(d.radiance[0], d.radiance[1], d.radiance[2]);
    if (d.type == SPRAY_RT_LIGHT_HEMISPHERE) return new DiffuseHemisphereLight(r);
    return new PointLight(glm::vec3(d.position[0], d.position[1], d.position[2]), r);
  }
  static Bsdf* makeBsdf(const spray_rt_bsdf& b) {
    if (b.type == SPRAY_RT_BSDF_DIFFUSE) return new DiffuseBsdf(glm::vec3(b.p[0], b.p[1], b.p[2]));
    return new DeltaBsdf;
  }
  static Aabb makeAabb(const float b[6]) {
    Aabb a;
    a.bounds[0] = glm::vec3(b[0], b[1], b[2]);
    a.bounds[1] = glm::vec3(b[3], b[4], b[5]);
    return a;
  }
};

namespace ooc {

struct Ray {  // ooc_ray.h:28-40, the fields a shader reads and writes
  float org[3], dir[3], w[3];
  int pixid, samid, depth;
  int light;
};

// ShaderPt (ooc_shader_pt.h:40-226) for non-delta surfaces: direct lighting
// of every light, then the diffuse continuation; shadows and the next ray go
// to vectors instead of the arena queues.
template <typename SceneT>
class ShaderPt {
 public:
  typedef SceneT SceneType;
  struct Config {
    int bounces, ao_samples;
    glm::vec3 ks;
    float shininess;
  };
  void init(const Config& cfg, const SceneT* scene) {
    bounces_ = cfg.bounces;
    samples_ = cfg.ao_samples;
    ks_ = cfg.ks;
    shininess_ = cfg.shininess;
    scene_ = scene;
    lights_ = scene->getLights();  // copy lights
  }
  void operator()(int domain_id, const Ray& rayin, const spray_rt_ray_intersection& isect,
                  std::vector<Ray>* sq, std::vector<Ray>* rq, int ray_depth) const {
    glm::vec3 pos(rayin.dir[0] * isect.tfar + rayin.org[0], rayin.dir[1] * isect.tfar + rayin.org[1],
                  rayin.dir[2] * isect.tfar + rayin.org[2]);  // RTCRayUtil::hitPosition
    glm::vec3 surf_radiance;
    surf_radiance[0] = ((isect.color >> 16) & 0xff) * MOCK_SPRAY_1_OVER_255;  // util::unpack
    surf_radiance[1] = ((isect.color >> 8) & 0xff) * MOCK_SPRAY_1_OVER_255;
    surf_radiance[2] = (isect.color & 0xff) * MOCK_SPRAY_1_OVER_255;
    glm::vec3 normal(isect.Ns[0], isect.Ns[1], isect.Ns[2]);
    glm::vec3 wo(-rayin.dir[0], -rayin.dir[1], -rayin.dir[2]);
    glm::vec3 Lin(rayin.w[0], rayin.w[1], rayin.w[2]);
    float cos_theta_i = glm::dot(wo, normal);
    bool entering = (cos_theta_i > 0.0f);
    glm::vec3 normal_ff = entering ? normal : -normal;
    normal_ff = glm::normalize(normal_ff);
    glm::vec3 wi, light_radiance, Lr;
    float pdf, costheta;
    int nlights = lights_.size();
    const Bsdf* bsdf = scene_->getBsdf(domain_id);
    bool delta_dist = bsdf->isDelta();
    int next_virtual_depth = rayin.depth + 1;
    int next_actual_depth = ray_depth + next_virtual_depth;
    if (!delta_dist) {
      RandomSampler light_sampler;
      RandomSampler_init(light_sampler, rayin.samid * next_actual_depth);
      for (int l = 0; l < nlights; ++l) {
        if (lights_[l]->isAreaLight()) {
          for (int s = 0; s < samples_; ++s) {
            light_radiance = lights_[l]->sampleArea(light_sampler, normal_ff, &wi, &pdf);
            if (pdf > 0.0f) {
              costheta = glm::clamp(glm::dot(normal_ff, wi), 0.0f, 1.0f);
              Lr = Lin * blinnPhong(costheta, surf_radiance, ks_, shininess_, light_radiance, wi,
                                    normal_ff, wo) *
                   (1.0f / (pdf * samples_));
              if (hasPositive(Lr)) sq->push_back(make(rayin, l, pos, wi, Lr));
            }
          }
        } else {
          light_radiance = lights_[l]->sample(pos, &wi, &pdf);
          if (pdf > 0.0f) {
            costheta = glm::clamp(glm::dot(normal_ff, wi), 0.0f, 1.0f);
            Lr = Lin * blinnPhong(costheta, surf_radiance, ks_, shininess_, light_radiance, wi,
                                  normal_ff, wo) *
                 (1.0f / pdf);
            if (hasPositive(Lr)) sq->push_back(make(rayin, l, pos, wi, Lr));
          }
        }
      }
    }
    if (next_actual_depth < bounces_ && !delta_dist) {
      RandomSampler sampler;
      RandomSampler_init(sampler, rayin.samid * next_actual_depth);
      bsdf->sampleRandom(normal_ff, &sampler, &wi, &pdf);
      costheta = glm::clamp(glm::dot(normal_ff, wi), 0.0f, 1.0f);
      Lr = Lin * surf_radiance * MOCK_SPRAY_ONE_OVER_PI * costheta / pdf;
      if (hasPositive(Lr)) {
        Ray r2 = make(rayin, -1, pos, wi, Lr);
        r2.depth = next_virtual_depth;
        rq->push_back(r2);
      }
    }
  }

 private:
  static Ray make(const Ray& in, int l, const glm::vec3& p, const glm::vec3& d,
                  const glm::vec3& w) {
    Ray r = in;
    for (int k = 0; k < 3; ++k) {
      r.org[k] = p[k];
      r.dir[k] = d[k];
      r.w[k] = w[k];
    }
    r.light = l;
    return r;
  }
  const SceneT* scene_ = nullptr;
  std::vector<Light*> lights_;
  int bounces_ = 1, samples_ = 1;
  glm::vec3 ks_;
  float shininess_ = 1.f;
};

}  // namespace ooc
}  // namespace spray
