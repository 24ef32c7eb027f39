/*
 * oracle.h -- CPU restatement of SpRay's intersect/occluded hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under spray_amd/ links, loads or calls
 * this library; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * Parity status: the reference's arithmetic lives in Embree 2.17.1 (third
 * party, not vendored, not installed here -- SURVEY.md 8(c)) and the reference
 * has no tests or golden vectors, so parity against Embree itself is
 * UNPINNED.  This oracle restates the published Embree 2 Moeller-Trumbore
 * intersector and the reference's own host code (cited per function in
 * oracle.c) and is cross-checked three ways in tests/: BVH traversal against
 * brute force (bit-exact), against a float64 watertight checker (1e-4), and
 * against the known-answer numbers of SURVEY.md 8(c) (primary hit fraction,
 * domains per ray).
 *
 * Build: oracle/Makefile -> oracle/_build/liboracle.so (gcc, -ffp-contract=off,
 * OpenMP).  Every float expression is written in the operand order the GPU
 * kernels use, with explicit fmaf() where a fused multiply-add is intended, so
 * results are bit-identical to the HIP path.
 */
#ifndef SPRAY_ORACLE_H_
#define SPRAY_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Whole-scene hit record (48 B), identical to spray_rt_hit_t in
 * include/spray_rt.h.  t = +inf and prim = domain = -1 on a miss. */
typedef struct or_hit {
  float t, u, v;
  uint32_t prim;
  float ng[3];
  uint32_t color;
  float ns[3];
  int32_t domain;
} or_hit;

/* Per-ray traversal counters of the canonical BVH2. */
typedef struct or_counts {
  uint64_t nodes;  /* 64 B node fetches */
  uint64_t tris;   /* 48 B triangle tests */
  uint64_t visits; /* (ray, domain) visits */
  uint64_t rays;
} or_counts;

/* ---- host-side data preparation (restated reference host code) ---- */
void or_transform_vertices(const float m[16], float* v, size_t nverts);
void or_compute_normals(const float* v, size_t nverts, const uint32_t* f,
                        size_t nfaces, float* n_out);
void or_world_aabb(const float m[16], const float obj_lo[3],
                   const float obj_hi[3], float out_lo_hi[6]);

/* ---- camera + sampler + eye rays ---- */
/* cam_out[14] = pos[3], lowerleft[3], wvec[3], hvec[3], image_w, image_h */
void or_camera_init(const float pos[3], const float lookat[3],
                    const float up[3], float vfov, int image_w, int image_h,
                    float cam_out[14]);
uint32_t or_sampler_init1(int id);
uint32_t or_sampler_init2(int pixel_id, int sample_id);
float or_sampler_get1d(uint32_t* state);
void or_camera_ray(const float cam[14], float x, float y, float dir[3]);
/* ooc::Tracer::genMultiEyes / genSingleEyes over one blocking tile.
 * n = tw*th*spp rays in bufid order. */
void or_eye_rays_ooc(const float cam[14], int image_w, int spp, int tx, int ty,
                     int tw, int th, float* org, float* dir, int32_t* pixid,
                     int32_t* samid);
/* insitu::genMultiSampleEyeRays over a tile inside a blocking tile. */
void or_eye_rays_insitu(const float cam[14], int image_w, int spp, int bx,
                        int by, int bw, int bh, int tx, int ty, int tw, int th,
                        float* org, float* dir, int32_t* pixid,
                        int32_t* samid);

/* ---- domain query (a5) ---- */
/* boxes[ndom][6] = lo.xyz hi.xyz.  ids/ts are [n][maxhits].  Returns the
 * number of rays whose hit count exceeded maxhits (lists truncated). */
int or_domain_query(const float* org, const float* dir, size_t n,
                    const float* boxes, int ndom, int maxhits, int32_t* ids,
                    float* ts, int32_t* counts);

/* ---- triangle primitives ---- */
/* tri_out[nf][12] = v0.xyz e1.xyz e2.xyz ng.xyz (e1=v0-v1, e2=v2-v0, ng=e1xe2) */
void or_prep_tris(const float* v, const uint32_t* f, size_t nf, float* tri_out);
/* Brute-force closest hit over all nf triangles of one domain. */
void or_brute_intersect(const float* tri, size_t nf, const float* org,
                        const float* dir, const float* tnear,
                        const float* tfar, size_t n, float* t_out,
                        float* u_out, float* v_out, uint32_t* prim_out);
void or_brute_occluded(const float* tri, size_t nf, const float* org,
                       const float* dir, const float* tnear,
                       const float* tfar, size_t n, uint8_t* occ_out);
/* float64 reference: closest hit with |t| error bound and an edge margin
 * flag (1 if the winning hit lies within rel. 1e-5 of a triangle edge). */
void or_f64_intersect(const float* v, const uint32_t* f, size_t nf,
                      const float* org, const float* dir, float tnear,
                      size_t n, double* t_out, int32_t* prim_out,
                      uint8_t* margin_out);

/* TriMeshBuffer::updateIntersection for n hits of one domain (prim = face
 * index; prim == 0xFFFFFFFF rows are skipped). */
void or_epilogue(const uint32_t* faces, const uint32_t* colors,
                 const float* normals, const uint32_t* prim, const float* u,
                 const float* v, size_t n, uint32_t* color_out, float* ns_out);

/* ---- canonical BVH2 (binned SAH, 32 bins, <=4 tris/leaf) ---- */
typedef struct or_bvh or_bvh;
or_bvh* or_bvh_build(const float* v, const uint32_t* f, size_t nf);
void or_bvh_free(or_bvh*);
size_t or_bvh_num_nodes(const or_bvh*);
int or_bvh_depth(const or_bvh*);
/* nodes_out[num_nodes][16] (64 B nodes), order_out[nf] (leaf-order prim ids)*/
void or_bvh_export(const or_bvh*, float* nodes_out, uint32_t* order_out);
void or_bvh_intersect(const or_bvh*, const float* org, const float* dir,
                      const float* tnear, const float* tfar, size_t n,
                      float* t_out, float* u_out, float* v_out,
                      uint32_t* prim_out, or_counts* cnt);
void or_bvh_occluded(const or_bvh*, const float* org, const float* dir,
                     const float* tnear, const float* tfar, size_t n,
                     uint8_t* occ_out, or_counts* cnt);

/* ---- whole scene: domain list + per-domain traversal + a4 epilogue ---- */
typedef struct or_scene or_scene;
or_scene* or_scene_create(int ndomains);
void or_scene_free(or_scene*);
/* verts already in world space; colors 0xRRGGBB per vertex; normals per
 * vertex (unnormalised, or_compute_normals); box = the .spray world bound. */
int or_scene_set_domain(or_scene*, int id, const float* v, size_t nv,
                        const uint32_t* f, size_t nf, const uint32_t* colors,
                        const float* normals, const float box[6]);
int or_scene_set_box(or_scene* s, int id, const float box[6]);
/* Closest hit over every domain the ray's sorted domain list holds
 * (ooc_isector.h:126-145 enqueues the ray to all of them; ooc_vbuf.cc:54-112
 * keeps the nearest), ties -> earlier list entry.  nthreads<=0: all. */
void or_scene_intersect(const or_scene*, const float* org, const float* dir,
                        size_t n, or_hit* hits, or_counts* cnt, int nthreads);
void or_scene_occluded(const or_scene*, const float* org, const float* dir,
                       size_t n, uint8_t* occ, or_counts* cnt, int nthreads);
/* PT point-light shadow spawn (ooc_shader_pt.h:93-171).  Writes rays for
 * primaries that hit and pass hasPositive(Lr); returns the count.
 * src_index_out[k] = primary index of shadow ray k (ascending). */
size_t or_spawn_shadows_pt(const float* org, const float* dir,
                           const or_hit* hits, size_t n,
                           const float light_pos[3],
                           const float light_rad[3], const float ks[3],
                           float shininess, float* sorg, float* sdir,
                           int32_t* src_index_out);
/* AO shadow spawn (ooc_shader_ao.h:120-146): up to nsamples per hit. */
size_t or_spawn_shadows_ao(const float* org, const float* dir,
                           const int32_t* pixid, const or_hit* hits, size_t n,
                           int nsamples, float* sorg, float* sdir,
                           int32_t* src_index_out);

/* ---- path shading + film (ooc::ShaderPt / ShaderAo, TContext::retire) ---- */
#define OR_SHADER_PT 0
#define OR_SHADER_AO 1
#define OR_LIGHT_POINT 0      /* PointLight, render/light.h:38-62 */
#define OR_LIGHT_HEMISPHERE 1 /* DiffuseHemisphereLight, light.h:64-90 */
#define OR_BSDF_DIFFUSE 0
#define OR_BSDF_MIRROR 1
#define OR_BSDF_GLASS 2        /* p = eta_exterior, eta_interior */
#define OR_BSDF_TRANSMISSION 3 /* p = eta_exterior, eta_interior */
#define OR_MAX_LIGHTS 8
typedef struct or_light {
  int32_t type;
  float pos[3];
  float radiance[3];
} or_light;
typedef struct or_bsdf {
  int32_t type;
  float p[3];
} or_bsdf;
typedef struct or_shader {
  int32_t shader;  /* OR_SHADER_* */
  int32_t bounces; /* cfg.bounces */
  int32_t samples; /* cfg.ao_samples */
  int32_t nlights;
  float ks[3];
  float shininess;
  or_light lights[OR_MAX_LIGHTS];
} or_shader;
int or_shadow_slots(const or_shader* P);
/* w[n][3] path weights, sw[n*nshadow][3]; see oracle.c */
int or_shade(const or_shader* P, const or_bsdf* bsdf, int nbsdf, int bounce,
             float* org, float* dir, const or_hit* hits, float* w, uint8_t* valid,
             const int32_t* pixid, const int32_t* samid, size_t n, float* sorg,
             float* sdir, float* sw, uint8_t* svalid);
void or_film(float* image_rgba, const int32_t* pixid, size_t n, int spp, int nshadow,
             const float* sw, const uint8_t* svalid, const uint8_t* occ,
             double scale);

#ifdef __cplusplus
}
#endif
#endif
