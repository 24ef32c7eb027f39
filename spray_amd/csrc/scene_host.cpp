// scene_host.cpp -- scene files, PLY meshes, domain cache and the GpuScene
// adapter (see scene_host.h), plus a C ABI (spray_scene_*) for bindings.
#include "scene_host.h"
#include "rt_ctx.h"
#include "spray_scene.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <algorithm>
#include <atomic>
#include <sstream>
#include <thread>

namespace spray_host {

// ---------------------------------------------------------------------------
// column-major 4x4 helpers (glm 0.9.8 operand order)
// ---------------------------------------------------------------------------
static void mat_identity(float m[16]) {
  for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.0f : 0.0f;
}

// glm::translate(m, v): m[3] = m[0]*v0 + m[1]*v1 + m[2]*v2 + m[3]
static void mat_translate(float m[16], const float v[3]) {
  for (int r = 0; r < 4; ++r) {
    float a = m[0 * 4 + r] * v[0], b = m[1 * 4 + r] * v[1],
          c = m[2 * 4 + r] * v[2];
    m[3 * 4 + r] = ((a + b) + c) + m[3 * 4 + r];
  }
}

// glm::scale(m, v): m[i] *= v[i], i < 3
static void mat_scale(float m[16], const float v[3]) {
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 4; ++r) m[c * 4 + r] = m[c * 4 + r] * v[c];
}

// glm::rotate(m, angle, axis)
static void mat_rotate(float m[16], float angle, const float axis_in[3]) {
  const float c = std::cos(angle), s = std::sin(angle);
  float len = 1.0f / std::sqrt((axis_in[0] * axis_in[0] + axis_in[1] * axis_in[1]) +
                               axis_in[2] * axis_in[2]);
  float ax[3] = {axis_in[0] * len, axis_in[1] * len, axis_in[2] * len};
  float t[3] = {(1.0f - c) * ax[0], (1.0f - c) * ax[1], (1.0f - c) * ax[2]};
  float R[3][3];
  R[0][0] = c + t[0] * ax[0];
  R[0][1] = t[0] * ax[1] + s * ax[2];
  R[0][2] = t[0] * ax[2] - s * ax[1];
  R[1][0] = t[1] * ax[0] - s * ax[2];
  R[1][1] = c + t[1] * ax[1];
  R[1][2] = t[1] * ax[2] + s * ax[0];
  R[2][0] = t[2] * ax[0] + s * ax[1];
  R[2][1] = t[2] * ax[1] - s * ax[0];
  R[2][2] = c + t[2] * ax[2];
  float out[16];
  for (int i = 0; i < 3; ++i)
    for (int r = 0; r < 4; ++r)
      out[i * 4 + r] = (m[0 * 4 + r] * R[i][0] + m[1 * 4 + r] * R[i][1]) +
                       m[2 * 4 + r] * R[i][2];
  for (int r = 0; r < 4; ++r) out[12 + r] = m[12 + r];
  std::memcpy(m, out, sizeof(out));
}

void transform_vertices(const float m[16], float* v, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const float x = v[3 * i], y = v[3 * i + 1], z = v[3 * i + 2];
    float o[3];
    for (int r = 0; r < 3; ++r)
      o[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * 1.0f);
    v[3 * i] = o[0];
    v[3 * i + 1] = o[1];
    v[3 * i + 2] = o[2];
  }
}

void compute_normals(Mesh* mesh) {
  const size_t nv = mesh->vertices.size() / 3, nf = mesh->faces.size() / 3;
  mesh->normals.assign(3 * nv, 0.0f);
  const float* v = mesh->vertices.data();
  float* n = mesh->normals.data();
  for (size_t i = 0; i < nf; ++i) {
    const size_t a = 3 * size_t(mesh->faces[3 * i]),
                 b = 3 * size_t(mesh->faces[3 * i + 1]),
                 c = 3 * size_t(mesh->faces[3 * i + 2]);
    const float ux = v[b] - v[a], uy = v[b + 1] - v[a + 1], uz = v[b + 2] - v[a + 2];
    const float wx = v[c] - v[a], wy = v[c + 1] - v[a + 1], wz = v[c + 2] - v[a + 2];
    const float nx = uy * wz - uz * wy;
    const float ny = uz * wx - ux * wz;
    const float nz = ux * wy - uy * wx;
    for (size_t k : {a, b, c}) {
      n[k] += nx;
      n[k + 1] += ny;
      n[k + 2] += nz;
    }
  }
}

static void vnorm(float v[3]) {
  const float inv = 1.0f / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
  v[0] *= inv;
  v[1] *= inv;
  v[2] *= inv;
}
static void vcross(const float a[3], const float b[3], float r[3]) {
  r[0] = a[1] * b[2] - b[1] * a[2];
  r[1] = a[2] * b[0] - b[2] * a[0];
  r[2] = a[0] * b[1] - b[0] * a[1];
}

void camera_init(const float pos[3], const float lookat[3], const float up[3],
                 float vfov, int image_w, int image_h, float cam[14]) {
  const float aspect = float(image_w) / float(image_h);
  const float theta = float(double(vfov) * 3.14159265358979323846 / 180.0);
  const float half_h = float(std::tan(double(theta / 2.0f)));
  const float half_w = aspect * half_h;
  float w[3] = {pos[0] - lookat[0], pos[1] - lookat[1], pos[2] - lookat[2]};
  float u[3], v[3];
  vcross(up, w, u);
  vcross(w, u, v);
  vnorm(w);
  vnorm(u);
  vnorm(v);
  for (int k = 0; k < 3; ++k) {
    const float center = pos[k] - w[k];
    cam[k] = pos[k];
    cam[3 + k] = (center - u[k] * half_w) - v[k] * half_h;
    cam[6 + k] = u[k] * (2.0f * half_w);
    cam[9 + k] = v[k] * (2.0f * half_h);
  }
  cam[12] = float(image_w);
  cam[13] = float(image_h);
}

// ---------------------------------------------------------------------------
// .spray scene description
// ---------------------------------------------------------------------------
bool load_scene_file(const std::string& desc, const std::string& ply_path,
                     std::vector<Domain>* domains, std::vector<Light>* lights,
                     std::string* err) {
  std::ifstream in(desc);
  if (!in.is_open()) {
    *err = "unable to open input file " + desc;
    return false;
  }
  domains->clear();
  lights->clear();
  std::string line;
  while (std::getline(in, line)) {
    std::vector<std::string> tok;
    {
      std::istringstream ss(line);
      std::string t;
      while (ss >> t) tok.push_back(t);
    }
    if (tok.empty() || tok[0][0] == '#') continue;
    const std::string& k = tok[0];
    auto need = [&](size_t n) {
      if (tok.size() != n) {
        *err = "malformed '" + k + "' line: " + line;
        return false;
      }
      if (k != "light" && k != "domain" && domains->empty()) {
        *err = "'" + k + "' before any 'domain'";
        return false;
      }
      return true;
    };
    auto f = [&](size_t i) { return float(std::atof(tok[i].c_str())); };
    if (k == "domain") {
      Domain d;
      d.id = int(domains->size());
      mat_identity(d.transform);
      domains->push_back(d);
    } else if (k == "file") {
      if (!need(2)) return false;
      domains->back().filename = ply_path.empty() ? tok[1] : ply_path + "/" + tok[1];
    } else if (k == "mtl") {
      if (domains->empty()) {
        *err = "'mtl' before any 'domain'";
        return false;
      }
      domains->back().material.assign(tok.begin() + 1, tok.end());
    } else if (k == "bound") {
      if (!need(7)) return false;
      for (int j = 0; j < 6; ++j) domains->back().object_aabb[j] = f(1 + j);
    } else if (k == "scale") {
      if (!need(4)) return false;
      float v[3] = {f(1), f(2), f(3)};
      mat_scale(domains->back().transform, v);
    } else if (k == "rotate") {
      if (!need(3)) return false;
      float axis[3] = {0, 0, 0};
      if (tok[1] == "x") axis[0] = 1;
      else if (tok[1] == "y") axis[1] = 1;
      else if (tok[1] == "z") axis[2] = 1;
      else {
        *err = "invalid axis name " + tok[1];
        return false;
      }
      float rad = float(double(std::atof(tok[2].c_str())) * 0.017453292519943295);
      mat_rotate(domains->back().transform, rad, axis);
    } else if (k == "translate") {
      if (!need(4)) return false;
      float v[3] = {f(1), f(2), f(3)};
      mat_translate(domains->back().transform, v);
    } else if (k == "face") {
      if (!need(2)) return false;
      domains->back().num_faces = std::stoul(tok[1]);
    } else if (k == "vertex") {
      if (!need(2)) return false;
      domains->back().num_vertices = std::stoul(tok[1]);
    } else if (k == "light") {
      Light l;
      if (tok.size() == 8 && tok[1] == "point") {
        l.type = 0;
        for (int j = 0; j < 3; ++j) {
          l.position[j] = f(2 + j);
          l.radiance[j] = f(5 + j);
        }
      } else if (tok.size() == 5 && tok[1] == "diffuse") {
        l.type = 1;
        for (int j = 0; j < 3; ++j) l.radiance[j] = f(2 + j);
      } else {
        *err = "unknown light source: " + line;
        return false;
      }
      lights->push_back(l);
    } else {
      *err = "unknown tag name " + k;
      return false;
    }
  }
  if (domains->empty()) {
    *err = "no domains in " + desc;
    return false;
  }
  for (Domain& d : *domains) {  // scene_loader.cc:351-357: two corners only
    float lo[3] = {d.object_aabb[0], d.object_aabb[1], d.object_aabb[2]};
    float hi[3] = {d.object_aabb[3], d.object_aabb[4], d.object_aabb[5]};
    transform_vertices(d.transform, lo, 1);
    transform_vertices(d.transform, hi, 1);
    std::memcpy(d.world_aabb, lo, 12);
    std::memcpy(d.world_aabb + 3, hi, 12);
  }
  return true;
}

// ---------------------------------------------------------------------------
// PLY
// ---------------------------------------------------------------------------
namespace {
int type_size(const std::string& t) {
  if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
  if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
  if (t == "int" || t == "uint" || t == "float" || t == "int32" ||
      t == "uint32" || t == "float32")
    return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}
double read_scalar(const char* p, const std::string& t) {
  if (t == "char" || t == "int8") return double(*reinterpret_cast<const int8_t*>(p));
  if (t == "uchar" || t == "uint8") return double(*reinterpret_cast<const uint8_t*>(p));
  int16_t s16;
  uint16_t u16;
  int32_t s32;
  uint32_t u32;
  float f32;
  double f64;
  if (t == "short" || t == "int16") { std::memcpy(&s16, p, 2); return s16; }
  if (t == "ushort" || t == "uint16") { std::memcpy(&u16, p, 2); return u16; }
  if (t == "int" || t == "int32") { std::memcpy(&s32, p, 4); return s32; }
  if (t == "uint" || t == "uint32") { std::memcpy(&u32, p, 4); return u32; }
  if (t == "float" || t == "float32") { std::memcpy(&f32, p, 4); return f32; }
  std::memcpy(&f64, p, 8);
  return f64;
}
struct Prop {
  std::string name, type, count_type;
  bool list = false;
};
struct Elem {
  std::string name;
  size_t n = 0;
  std::vector<Prop> props;
};
}  // namespace

bool load_ply(const std::string& filename, Mesh* mesh, std::string* err) {
  std::ifstream in(filename, std::ios::binary);
  if (!in.is_open()) {
    *err = "cannot open " + filename;
    return false;
  }
  std::string line, format;
  std::getline(in, line);
  if (line != "ply") {
    *err = "unknown file type " + filename;
    return false;
  }
  std::vector<Elem> elems;
  bool end = false;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string w;
    ss >> w;
    if (w == "format") {
      ss >> format;
    } else if (w == "element") {
      Elem e;
      ss >> e.name >> e.n;
      elems.push_back(e);
    } else if (w == "property") {
      if (elems.empty()) {
        *err = "property before element";
        return false;
      }
      Prop p;
      std::string t;
      ss >> t;
      if (t == "list") {
        p.list = true;
        ss >> p.count_type >> p.type >> p.name;
      } else {
        p.type = t;
        ss >> p.name;
      }
      elems.back().props.push_back(p);
    } else if (w == "end_header") {
      end = true;
      break;
    }
  }
  if (!end || (format != "binary_little_endian" && format != "ascii")) {
    *err = "unsupported PLY header/format in " + filename;
    return false;
  }
  const bool binary = format == "binary_little_endian";
  mesh->vertices.clear();
  mesh->faces.clear();
  mesh->colors.clear();
  for (const Elem& e : elems) {
    if (e.name == "vertex") {
      mesh->vertices.resize(3 * e.n);
      mesh->colors.assign(e.n, 0u);
      int ix = -1, iy = -1, iz = -1, ir = -1, ig = -1, ib = -1;
      for (size_t k = 0; k < e.props.size(); ++k) {
        const std::string& nm = e.props[k].name;
        if (nm == "x") ix = int(k);
        if (nm == "y") iy = int(k);
        if (nm == "z") iz = int(k);
        if (nm == "red") ir = int(k);
        if (nm == "green") ig = int(k);
        if (nm == "blue") ib = int(k);
      }
      if (ix < 0 || iy < 0 || iz < 0) {
        *err = "vertex element without x/y/z";
        return false;
      }
      std::vector<double> val(e.props.size());
      std::vector<char> rec;
      size_t rsz = 0;
      std::vector<size_t> off(e.props.size());
      for (size_t k = 0; k < e.props.size(); ++k) {
        off[k] = rsz;
        rsz += type_size(e.props[k].type);
      }
      rec.resize(rsz);
      for (size_t n = 0; n < e.n; ++n) {
        if (binary) {
          if (!in.read(rec.data(), rsz)) {
            *err = "truncated vertex data";
            return false;
          }
          for (size_t k = 0; k < e.props.size(); ++k)
            val[k] = read_scalar(rec.data() + off[k], e.props[k].type);
        } else {
          std::getline(in, line);
          std::istringstream ss(line);
          for (size_t k = 0; k < e.props.size(); ++k) ss >> val[k];
        }
        mesh->vertices[3 * n] = float(val[ix]);
        mesh->vertices[3 * n + 1] = float(val[iy]);
        mesh->vertices[3 * n + 2] = float(val[iz]);
        if (ir >= 0 && ig >= 0 && ib >= 0)
          mesh->colors[n] = (uint32_t(val[ir]) << 16) | (uint32_t(val[ig]) << 8) |
                            uint32_t(val[ib]);
      }
    } else if (e.name == "face") {
      if (e.props.size() != 1 || !e.props[0].list) {
        *err = "face element must be one index list";
        return false;
      }
      const Prop& p = e.props[0];
      const int cs = type_size(p.count_type), is = type_size(p.type);
      mesh->faces.resize(3 * e.n);
      char buf[16];
      for (size_t n = 0; n < e.n; ++n) {
        long cnt;
        uint32_t idx[3];
        if (binary) {
          if (!in.read(buf, cs)) {
            *err = "truncated face data";
            return false;
          }
          cnt = long(read_scalar(buf, p.count_type));
          if (cnt != 3) {
            *err = "only triangles are supported";
            return false;
          }
          for (int j = 0; j < 3; ++j) {
            in.read(buf, is);
            idx[j] = uint32_t(read_scalar(buf, p.type));
          }
        } else {
          std::getline(in, line);
          std::istringstream ss(line);
          ss >> cnt;
          if (cnt != 3) {
            *err = "only triangles are supported";
            return false;
          }
          ss >> idx[0] >> idx[1] >> idx[2];
        }
        std::memcpy(&mesh->faces[3 * n], idx, 12);
      }
    } else {
      *err = "unknown element name " + e.name;
      return false;
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// cache
// ---------------------------------------------------------------------------
void DomainCache::init(int num_domains, int cache_size) {
  lru_ = !(cache_size < 0 || cache_size >= num_domains);
  capacity_ = lru_ ? cache_size : num_domains;
  size_ = 0;
  status_.assign(num_domains, 0);
  blocks_.clear();
  where_.clear();
}

bool DomainCache::load(int domid, int* block) {
  if (!lru_) {  // InfiniteCache::load (infinite_cache.cc:47-60)
    *block = domid;
    const bool hit = status_[domid] != 0;
    status_[domid] = 1;
    return hit;
  }
  // LruCache::load (lru_cache.cc:65-171)
  if (status_[domid]) {
    auto it = where_[domid];
    Block b = *it;
    blocks_.erase(it);
    blocks_.push_back(b);
    where_[domid] = std::prev(blocks_.end());
    *block = b.block;
    return true;
  }
  status_[domid] = 1;
  Block nb{0, domid};
  if (size_ < capacity_) {
    nb.block = size_++;
  } else {
    Block old = blocks_.front();
    blocks_.pop_front();
    where_.erase(old.domain);
    status_[old.domain] = 0;
    nb.block = old.block;
  }
  blocks_.push_back(nb);
  where_[domid] = std::prev(blocks_.end());
  *block = nb.block;
  return false;
}

// ---------------------------------------------------------------------------
// GpuScene
// ---------------------------------------------------------------------------
GpuScene::~GpuScene() {
  if (rt_) spray_rt_destroy(rt_);
  for (void* p : pinned_)
    if (p) (void)hipHostFree(p);
}

int GpuScene::fail(int code, const std::string& msg) {
  err_ = msg;
  return code;
}

int GpuScene::init(const std::string& desc, const std::string& ply_path,
                   int cache_size, int hip_device) {
  std::string e;
  if (!load_scene_file(desc, ply_path, &domains_, &lights_, &e))
    return fail(SPRAY_RT_ERR_ARG, e);
  // mergeDomainBounds (scene.inl:295-349)
  for (int j = 0; j < 3; ++j) {
    bound_[j] = domains_[0].world_aabb[j];
    bound_[3 + j] = domains_[0].world_aabb[3 + j];
  }
  for (const Domain& d : domains_)
    for (int j = 0; j < 3; ++j) {
      bound_[j] = std::fmin(bound_[j], d.world_aabb[j]);
      bound_[3 + j] = std::fmax(bound_[3 + j], d.world_aabb[3 + j]);
    }
  int r = spray_rt_create(hip_device, &rt_);
  if (r) return fail(r, "spray_rt_create failed (no HIP device?)");
  std::vector<float> boxes(6 * domains_.size());
  for (size_t i = 0; i < domains_.size(); ++i)
    std::memcpy(&boxes[6 * i], domains_[i].world_aabb, 24);
  r = spray_rt_domain_bounds(rt_, int(domains_.size()), boxes.data());
  if (r) return fail(r, spray_rt_last_error(rt_));
  cache_.init(int(domains_.size()), cache_size);
  block_domain_.assign(cache_.capacity(), -1);
  images_.resize(domains_.size());
  pinned_.assign(domains_.size(), nullptr);
  r = prebuild_images();
  if (r) return r;
  if (!cache_.lru()) {  // warm-up (scene.inl:86-93)
    for (size_t id = 0; id < domains_.size(); ++id) {
      SceneInfo s;
      r = load(int(id), &s);
      if (r) return r;
    }
    // every domain is resident for good: no miss will read a pinned image
    // again (an upload after all would rebuild it, build_image)
    if (hipDeviceSynchronize() != hipSuccess) return fail(SPRAY_RT_ERR_HIP, "warm-up uploads");
    for (void*& p : pinned_)
      if (p) {
        (void)hipHostFree(p);
        p = nullptr;
      }
  }
  return SPRAY_RT_OK;
}

// A cache miss uploads the domain's device image.  TriMeshBuffer::load
// (trimesh_buffer.cc:117-169) re-reads, transforms and rebuilds on every
// miss; the image is a pure function of the domain, so it is built on the
// first load only and kept in pinned host memory -- a later miss is one
// async DMA (the bytes, hence every result, are the same).
int GpuScene::build_image(int id, std::string* err) {
  spray_rt::detail::SlotImage& img = images_[size_t(id)];
  const Domain& d = domains_[id];
  const auto it = ply_cache_.find(d.filename);
  if (it == ply_cache_.end()) {
    *err = "domain " + std::to_string(id) + ": mesh not loaded";
    return SPRAY_RT_ERR_STATE;
  }
  Mesh mesh = it->second;  // world-space copy
  float ident[16];
  mat_identity(ident);
  if (std::memcmp(ident, d.transform, sizeof(ident)) != 0)
    transform_vertices(d.transform, mesh.vertices.data(), mesh.vertices.size() / 3);
  compute_normals(&mesh);
  if (const char* why = spray_rt::detail::build_slot_image(
          mesh.vertices.data(), mesh.vertices.size() / 3, mesh.faces.data(),
          mesh.faces.size() / 3, mesh.colors.data(), mesh.normals.data(), &img)) {
    *err = std::string("domain ") + std::to_string(id) + ": " + why;
    return SPRAY_RT_ERR_ARG;
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, img.nbytes, hipHostMallocDefault) != hipSuccess) {
    *err = "pinned host memory for a domain image";
    return SPRAY_RT_ERR_NOMEM;
  }
  std::memcpy(p, img.bytes.data(), img.nbytes);
  pinned_[size_t(id)] = p;
  std::vector<char>().swap(img.bytes);  // one host copy: the pinned one
  return SPRAY_RT_OK;
}

// The misses of an LRU cache would each build a domain image inside the
// tracer's `omp single` while every other thread waits; building them all up
// front (in parallel: the meshes first, then one image per task) leaves a
// miss one async DMA.  Bounded by a budget of page-locked host memory (the
// images' bytes ~ 100 B per triangle, one pinned copy each); past it images
// are built on their first miss, and the skip is logged.  The default, 8 GB,
// keeps the triangle capacity of the earlier 16 GB budget that held each
// image twice (a vector and a pinned copy): ~86 M triangles.
int GpuScene::prebuild_images() {
  const char* e = std::getenv("SPRAY_SCENE_PREBUILD_MB");
  const double budget_mb = e ? std::atof(e) : 8192.0;
  if (budget_mb <= 0.0) return SPRAY_RT_OK;
  double tris = 0.0;
  for (const Domain& d : domains_) {
    auto it = ply_cache_.find(d.filename);
    if (it == ply_cache_.end()) {
      Mesh m;
      std::string err;
      if (!load_ply(d.filename, &m, &err)) return fail(SPRAY_RT_ERR_ARG, err);
      it = ply_cache_.emplace(d.filename, std::move(m)).first;
    }
    tris += double(it->second.faces.size() / 3);
  }
  if (tris * 100.0 > budget_mb * 1048576.0) {
    std::fprintf(stderr,
                 "spray_scene: %.0f triangles need ~%.0f MB of pinned domain images, over the "
                 "SPRAY_SCENE_PREBUILD_MB budget of %.0f MB: images are built on their first "
                 "cache miss\n", tris, tris * 100.0 / 1048576.0, budget_mb);
    return SPRAY_RT_OK;
  }
  const int nd = int(domains_.size());
  const int nt = std::max(1, std::min(nd, int(std::min(16u, std::thread::hardware_concurrency()))));
  std::vector<int> rc(nd, SPRAY_RT_OK);
  std::vector<std::string> err(nd);
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&] {
      for (int id = next++; id < nd; id = next++) rc[id] = build_image(id, &err[id]);
    });
  for (std::thread& th : pool) th.join();
  for (int id = 0; id < nd; ++id)
    if (rc[id]) return fail(rc[id], err[id]);
  return SPRAY_RT_OK;
}

int GpuScene::upload(int id, int block) {
  spray_rt::detail::SlotImage& img = images_[size_t(id)];
  if (!pinned_[size_t(id)]) {
    const Domain& d = domains_[id];
    if (ply_cache_.find(d.filename) == ply_cache_.end()) {
      Mesh m;
      std::string e;
      if (!load_ply(d.filename, &m, &e)) return fail(SPRAY_RT_ERR_ARG, e);
      ply_cache_.emplace(d.filename, std::move(m));
    }
    std::string e;
    const int r = build_image(id, &e);
    if (r) return fail(r, e);
  }
  int r = spray_rt::detail::upload_slot_image(rt_, block, img, pinned_[size_t(id)], true);
  if (r) return fail(r, spray_rt_last_error(rt_));
  // keep the scene path's domain -> slot map in step with the cache
  if (block_domain_[block] >= 0)
    spray_rt_map_domain(rt_, block_domain_[block], -1);
  block_domain_[block] = id;
  r = spray_rt_map_domain(rt_, id, block);
  if (r) return fail(r, spray_rt_last_error(rt_));
  return SPRAY_RT_OK;
}

int GpuScene::load(int id, SceneInfo* sinfo) {
  if (id < 0 || size_t(id) >= domains_.size())
    return fail(SPRAY_RT_ERR_ARG, "domain id out of range");
  int block;
  if (!cache_.load(id, &block)) {
    int r = upload(id, block);
    if (r) return r;
  }
  sinfo->cache_block = block;
  return SPRAY_RT_OK;
}

static void make_radiance_ray(const float org[3], const float dir[3],
                              spray_rt_ray_intersection* r) {
  // RTCRayUtil::makeRadianceRay (rays.h:345-363)
  for (int k = 0; k < 3; ++k) {
    r->org[k] = org[k];
    r->dir[k] = dir[k];
  }
  r->tnear = 0.001f;
  r->tfar = INFINITY;
  r->instID = r->geomID = r->primID = SPRAY_RT_INVALID_ID;
  r->mask = 0xFFFFFFFFu;
  r->time = 0.0f;
}

bool GpuScene::intersect(const SceneInfo& s, const float org[3],
                         const float dir[3], spray_rt_ray_intersection* isect) {
  make_radiance_ray(org, dir, isect);
  if (spray_rt_intersect1M(rt_, s.cache_block, isect, 1, sizeof(*isect))) return false;
  return isect->geomID != SPRAY_RT_INVALID_ID;
}

bool GpuScene::occluded(const SceneInfo& s, const float org[3],
                        const float dir[3], spray_rt_ray_intersection* ray) {
  make_radiance_ray(org, dir, ray);  // makeShadowRay: same fields (rays.h:389-423)
  if (spray_rt_occluded1M(rt_, s.cache_block, ray, 1, sizeof(*ray))) return false;
  return ray->geomID != SPRAY_RT_INVALID_ID;
}

int GpuScene::intersectDomains(const float org[3], const float dir[3], int* ids,
                               float* ts, int maxhits) {
  int count = 0;
  int r = spray_rt_domains1M(rt_, org, dir, 1, ids, ts, &count, maxhits);
  return r ? r : count;
}

int GpuScene::intersect1M(int block, spray_rt_ray_intersection* rays, size_t n) {
  return spray_rt_intersect1M(rt_, block, rays, n, sizeof(*rays));
}

int GpuScene::occluded1M(int block, spray_rt_ray_intersection* rays, size_t n) {
  return spray_rt_occluded1M(rt_, block, rays, n, sizeof(*rays));
}

}  // namespace spray_host

// ---------------------------------------------------------------------------
// C ABI for bindings (include/spray_scene.h)
// ---------------------------------------------------------------------------
using spray_host::GpuScene;

extern "C" {

int spray_scene_create(const char* desc, const char* ply_path, int cache_size,
                       int hip_device, spray_scene_t* out, char* err,
                       size_t errlen) {
  if (!out || !desc) return SPRAY_RT_ERR_ARG;
  GpuScene* s = new GpuScene;
  int r = s->init(desc, ply_path ? ply_path : "", cache_size, hip_device);
  if (r) {
    if (err && errlen) std::snprintf(err, errlen, "%s", s->error().c_str());
    delete s;
    *out = nullptr;
    return r;
  }
  *out = reinterpret_cast<spray_scene_t>(s);
  return SPRAY_RT_OK;
}

int spray_scene_destroy(spray_scene_t h) {
  delete reinterpret_cast<GpuScene*>(h);
  return SPRAY_RT_OK;
}

const char* spray_scene_last_error(spray_scene_t h) {
  return h ? reinterpret_cast<GpuScene*>(h)->error().c_str() : "null scene";
}

spray_rt_ctx_t spray_scene_rt(spray_scene_t h) {
  return reinterpret_cast<GpuScene*>(h)->rt();
}

int spray_scene_num_domains(spray_scene_t h) {
  return int(reinterpret_cast<GpuScene*>(h)->getNumDomains());
}

int spray_scene_cache_capacity(spray_scene_t h) {
  return reinterpret_cast<GpuScene*>(h)->cacheCapacity();
}

// boxes[n][6] world bounds; bound[6] scene bound
int spray_scene_bounds(spray_scene_t h, float* boxes, float* bound) {
  GpuScene* s = reinterpret_cast<GpuScene*>(h);
  if (boxes)
    for (size_t i = 0; i < s->getNumDomains(); ++i)
      std::memcpy(boxes + 6 * i, s->getDomains()[i].world_aabb, 24);
  if (bound) std::memcpy(bound, s->getBound(), 24);
  return SPRAY_RT_OK;
}

int spray_scene_num_lights(spray_scene_t h) {
  return int(reinterpret_cast<GpuScene*>(h)->getLights().size());
}

// out7 = type, position[3], radiance[3]
int spray_scene_light(spray_scene_t h, int i, float* out7) {
  GpuScene* s = reinterpret_cast<GpuScene*>(h);
  if (i < 0 || size_t(i) >= s->getLights().size()) return SPRAY_RT_ERR_ARG;
  const auto& l = s->getLights()[i];
  out7[0] = float(l.type);
  std::memcpy(out7 + 1, l.position, 12);
  std::memcpy(out7 + 4, l.radiance, 12);
  return SPRAY_RT_OK;
}

int spray_scene_load(spray_scene_t h, int id, int* cache_block) {
  GpuScene* s = reinterpret_cast<GpuScene*>(h);
  spray_host::SceneInfo si;
  int r = s->load(id, &si);
  if (!r && cache_block) *cache_block = si.cache_block;
  return r;
}

int spray_scene_intersect1(spray_scene_t h, int cache_block, const float* org,
                           const float* dir, spray_rt_ray_intersection* isect) {
  spray_host::SceneInfo si;
  si.cache_block = cache_block;
  return reinterpret_cast<GpuScene*>(h)->intersect(si, org, dir, isect) ? 1 : 0;
}

int spray_scene_occluded1(spray_scene_t h, int cache_block, const float* org,
                          const float* dir, spray_rt_ray_intersection* ray) {
  spray_host::SceneInfo si;
  si.cache_block = cache_block;
  return reinterpret_cast<GpuScene*>(h)->occluded(si, org, dir, ray) ? 1 : 0;
}

int spray_camera_init(const float* pos, const float* lookat, const float* up,
                      float vfov, int w, int h, float* cam14) {
  spray_host::camera_init(pos, lookat, up, vfov, w, h, cam14);
  return SPRAY_RT_OK;
}

// Host mesh preparation (PLY + transform + normals) for a domain, exposed
// for callers that manage uploads themselves.  Sizes first (arrays NULL).
int spray_scene_domain_mesh(spray_scene_t h, int id, size_t* nverts,
                            size_t* nfaces, float* verts, uint32_t* faces,
                            uint32_t* colors, float* normals);

static int prep_mesh(const spray_host::Domain& d, spray_host::Mesh* m) {
  std::string e;
  if (!spray_host::load_ply(d.filename, m, &e)) return SPRAY_RT_ERR_ARG;
  float ident[16];
  for (int i = 0; i < 16; ++i) ident[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  if (std::memcmp(ident, d.transform, sizeof(ident)) != 0)
    spray_host::transform_vertices(d.transform, m->vertices.data(), m->vertices.size() / 3);
  spray_host::compute_normals(m);
  return SPRAY_RT_OK;
}

static void copy_mesh(const spray_host::Mesh& m, size_t* nverts, size_t* nfaces,
                      float* verts, uint32_t* faces, uint32_t* colors,
                      float* normals) {
  *nverts = m.vertices.size() / 3;
  *nfaces = m.faces.size() / 3;
  if (verts) std::memcpy(verts, m.vertices.data(), m.vertices.size() * 4);
  if (faces) std::memcpy(faces, m.faces.data(), m.faces.size() * 4);
  if (colors) std::memcpy(colors, m.colors.data(), m.colors.size() * 4);
  if (normals) std::memcpy(normals, m.normals.data(), m.normals.size() * 4);
}

int spray_host_parse_scene(const char* desc, const char* ply_path,
                           int* ndomains, int* nlights, float* boxes,
                           float* transforms, float* lights, char* err,
                           size_t errlen) {
  if (!desc) return SPRAY_RT_ERR_ARG;
  std::vector<spray_host::Domain> doms;
  std::vector<spray_host::Light> ls;
  std::string e;
  if (!spray_host::load_scene_file(desc, ply_path ? ply_path : "", &doms, &ls, &e)) {
    if (err && errlen) std::snprintf(err, errlen, "%s", e.c_str());
    return SPRAY_RT_ERR_ARG;
  }
  if (ndomains) *ndomains = int(doms.size());
  if (nlights) *nlights = int(ls.size());
  for (size_t i = 0; i < doms.size(); ++i) {
    if (boxes) std::memcpy(boxes + 6 * i, doms[i].world_aabb, 24);
    if (transforms) std::memcpy(transforms + 16 * i, doms[i].transform, 64);
  }
  if (lights)
    for (size_t i = 0; i < ls.size(); ++i) {
      lights[7 * i] = float(ls[i].type);
      std::memcpy(lights + 7 * i + 1, ls[i].position, 12);
      std::memcpy(lights + 7 * i + 4, ls[i].radiance, 12);
    }
  return SPRAY_RT_OK;
}

int spray_host_scene_bsdfs(const char* desc, int* ndomains, spray_rt_bsdf* bsdfs, char* err,
                           size_t errlen) {
  if (!desc || !ndomains) return SPRAY_RT_ERR_ARG;
  std::vector<spray_host::Domain> doms;
  std::vector<spray_host::Light> ls;
  std::string e;
  if (!spray_host::load_scene_file(desc, "", &doms, &ls, &e)) {
    if (err && errlen) std::snprintf(err, errlen, "%s", e.c_str());
    return SPRAY_RT_ERR_ARG;
  }
  *ndomains = int(doms.size());
  if (!bsdfs) return SPRAY_RT_OK;
  // SceneLoader::parseMaterial (src/io/scene_loader.cc:88-130)
  for (size_t i = 0; i < doms.size(); ++i) {
    const std::vector<std::string>& t = doms[i].material;
    spray_rt_bsdf& b = bsdfs[i];
    b.type = SPRAY_RT_BSDF_DIFFUSE;
    b.p[0] = b.p[1] = b.p[2] = 0.f;
    auto bad = [&](const char* why) {
      if (err && errlen) std::snprintf(err, errlen, "domain %zu: %s", i, why);
      return SPRAY_RT_ERR_ARG;
    };
    if (t.empty()) return bad("no material (the reference's getBsdf would be null)");
    const std::string& k = t[0];
    const size_t want = (k == "diffuse" || k == "mirror") ? 4 : 3;
    if (k == "diffuse") b.type = SPRAY_RT_BSDF_DIFFUSE;
    else if (k == "mirror") b.type = SPRAY_RT_BSDF_MIRROR;
    else if (k == "glass") b.type = SPRAY_RT_BSDF_GLASS;
    else if (k == "transmission") b.type = SPRAY_RT_BSDF_TRANSMISSION;
    else return bad("unknown material type");
    if (t.size() != want) return bad("wrong number of material parameters");
    for (size_t j = 1; j < want; ++j) b.p[j - 1] = float(std::atof(t[j].c_str()));
  }
  return SPRAY_RT_OK;
}

int spray_host_domain_mesh(const char* desc, const char* ply_path, int id,
                           size_t* nverts, size_t* nfaces, float* verts,
                           uint32_t* faces, uint32_t* colors, float* normals) {
  std::vector<spray_host::Domain> doms;
  std::vector<spray_host::Light> ls;
  std::string e;
  if (!desc || !nverts || !nfaces ||
      !spray_host::load_scene_file(desc, ply_path ? ply_path : "", &doms, &ls, &e))
    return SPRAY_RT_ERR_ARG;
  if (id < 0 || size_t(id) >= doms.size()) return SPRAY_RT_ERR_ARG;
  spray_host::Mesh m;
  int r = prep_mesh(doms[id], &m);
  if (r) return r;
  copy_mesh(m, nverts, nfaces, verts, faces, colors, normals);
  return SPRAY_RT_OK;
}

int spray_scene_domain_mesh(spray_scene_t h, int id, size_t* nverts,
                            size_t* nfaces, float* verts, uint32_t* faces,
                            uint32_t* colors, float* normals) {
  GpuScene* s = reinterpret_cast<GpuScene*>(h);
  if (!s || id < 0 || size_t(id) >= s->getNumDomains() || !nverts || !nfaces)
    return SPRAY_RT_ERR_ARG;
  spray_host::Mesh m;
  int r = prep_mesh(s->getDomains()[id], &m);
  if (r) return r;
  copy_mesh(m, nverts, nfaces, verts, faces, colors, normals);
  return SPRAY_RT_OK;
}

}  // extern "C"
