"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker or the timed CPU baseline.  The product
(spray_amd/) never imports it.

Besides the C entry points of oracle.c it restates, in numpy, the two input
parsers the hot path consumes:
  * ``parse_spray``  -- SceneLoader::load, src/io/scene_loader.cc:42-358
  * ``load_ply``     -- PlyLoader::load/parseVertices/parseFaces,
                        src/io/ply_loader.cc:114-324
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

HIT_DTYPE = np.dtype([("t", "<f4"), ("u", "<f4"), ("v", "<f4"), ("prim", "<u4"),
                      ("ng", "<f4", 3), ("color", "<u4"), ("ns", "<f4", 3),
                      ("domain", "<i4")])
assert HIT_DTYPE.itemsize == 48


class Counts(C.Structure):
    _fields_ = [("nodes", C.c_uint64), ("tris", C.c_uint64),
                ("visits", C.c_uint64), ("rays", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class _Lib:
    """Forwards calls to the CDLL and drops the temporaries _p() parked."""

    def __init__(self, cdll):
        self._cdll = cdll

    def __getattr__(self, name):
        fn = getattr(self._cdll, name)

        def call(*args):
            try:
                return fn(*args)
            finally:
                _release()
        return call


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        cdll = C.CDLL(LIB_PATH)
        _declare(cdll)
        _lib = _Lib(cdll)
    return _lib


P = C.c_void_p
SZ = C.c_size_t


def _declare(L):
    sig = {
        "or_transform_vertices": (None, [P, P, SZ]),
        "or_compute_normals": (None, [P, SZ, P, SZ, P]),
        "or_world_aabb": (None, [P, P, P, P]),
        "or_camera_init": (None, [P, P, P, C.c_float, C.c_int, C.c_int, P]),
        "or_sampler_init1": (C.c_uint32, [C.c_int]),
        "or_sampler_init2": (C.c_uint32, [C.c_int, C.c_int]),
        "or_sampler_get1d": (C.c_float, [P]),
        "or_camera_ray": (None, [P, C.c_float, C.c_float, P]),
        "or_eye_rays_ooc": (None, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, P, P, P, P]),
        "or_eye_rays_insitu": (None, [P, C.c_int, C.c_int] + [C.c_int] * 8 + [P, P, P, P]),
        "or_domain_query": (C.c_int, [P, P, SZ, P, C.c_int, C.c_int, P, P, P]),
        "or_prep_tris": (None, [P, P, SZ, P]),
        "or_brute_intersect": (None, [P, SZ, P, P, P, P, SZ, P, P, P, P]),
        "or_brute_occluded": (None, [P, SZ, P, P, P, P, SZ, P]),
        "or_f64_intersect": (None, [P, P, SZ, P, P, C.c_float, SZ, P, P, P]),
        "or_epilogue": (None, [P, P, P, P, P, P, SZ, P, P]),
        "or_bvh_build": (P, [P, P, SZ]),
        "or_bvh_free": (None, [P]),
        "or_bvh_num_nodes": (SZ, [P]),
        "or_bvh_depth": (C.c_int, [P]),
        "or_bvh_export": (None, [P, P, P]),
        "or_bvh_intersect": (None, [P, P, P, P, P, SZ, P, P, P, P, P]),
        "or_bvh_occluded": (None, [P, P, P, P, P, SZ, P, P]),
        "or_scene_create": (P, [C.c_int]),
        "or_scene_free": (None, [P]),
        "or_scene_set_domain": (C.c_int, [P, C.c_int, P, SZ, P, SZ, P, P, P]),
        "or_scene_set_box": (C.c_int, [P, C.c_int, P]),
        "or_scene_intersect": (None, [P, P, P, SZ, P, P, C.c_int]),
        "or_scene_occluded": (None, [P, P, P, SZ, P, P, C.c_int]),
        "or_spawn_shadows_pt": (SZ, [P, P, P, SZ, P, P, P, C.c_float, P, P, P]),
        "or_spawn_shadows_ao": (SZ, [P, P, P, P, SZ, C.c_int, P, P, P]),
        "or_shadow_slots": (C.c_int, [P]),
        "or_shade": (C.c_int, [P, P, C.c_int, C.c_int, P, P, P, P, P, P, P, SZ, P, P, P, P]),
        "or_film": (None, [P, P, SZ, C.c_int, C.c_int, P, P, P, C.c_double]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


_KEEP = []


def _p(a):
    """Address of a C-contiguous array.  Converted temporaries are parked in
    _KEEP until the enclosing wrapper returns (see _call)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays must be C-contiguous"
    _KEEP.append(a)
    return a.ctypes.data


def _release():
    del _KEEP[:]


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


# --------------------------------------------------------------------------
# input parsing (numpy restatements)
# --------------------------------------------------------------------------

def load_ply(path):
    """PlyLoader::load (src/io/ply_loader.cc:179-324): binary little endian
    or ascii; float x y z (+ optional uchar r g b); triangle list faces.
    Returns (verts float32[nv,3], faces uint32[nf,3], colors uint32[nv])."""
    data = open(path, "rb").read()
    end = data.index(b"end_header")
    end = data.index(b"\n", end) + 1
    header = data[:end].decode("ascii").splitlines()
    assert header[0] == "ply", "unknown file type"
    fmt = None
    elems = []
    for line in header[1:]:
        w = line.split()
        if not w:
            continue
        if w[0] == "format":
            fmt = w[1]
        elif w[0] == "element":
            elems.append({"name": w[1], "n": int(w[2]), "props": []})
        elif w[0] == "property":
            elems[-1]["props"].append(w[1:])
    assert fmt in ("binary_little_endian", "ascii"), fmt
    verts = faces = colors = None
    tmap = {"char": "i1", "uchar": "u1", "short": "<i2", "ushort": "<u2",
            "int": "<i4", "uint": "<u4", "float": "<f4", "double": "<f8",
            "int8": "i1", "uint8": "u1", "int32": "<i4", "uint32": "<u4",
            "float32": "<f4"}
    if fmt == "ascii":
        body = data[end:].decode("ascii").split("\n")
        li = 0
        for e in elems:
            rows = body[li:li + e["n"]]
            li += e["n"]
            if e["name"] == "vertex":
                arr = np.array([r.split() for r in rows], dtype=np.float64)
                verts = arr[:, :3].astype(np.float32)
                if arr.shape[1] >= 6:
                    c = arr[:, 3:6].astype(np.uint32)
                    colors = (c[:, 0] << 16) | (c[:, 1] << 8) | c[:, 2]
            else:
                arr = np.array([r.split() for r in rows], dtype=np.int64)
                assert (arr[:, 0] == 3).all()
                faces = arr[:, 1:4].astype(np.uint32)
    else:
        off = end
        for e in elems:
            if e["name"] == "vertex":
                dt = np.dtype([(p[-1], tmap[p[0]]) for p in e["props"]])
                v = np.frombuffer(data, dtype=dt, count=e["n"], offset=off)
                off += dt.itemsize * e["n"]
                verts = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float32)
                if "red" in dt.names:
                    colors = ((v["red"].astype(np.uint32) << 16) |
                              (v["green"].astype(np.uint32) << 8) |
                              v["blue"].astype(np.uint32))
            else:
                p = e["props"][0]
                assert p[0] == "list"
                dt = np.dtype([("n", tmap[p[1]]), ("i", tmap[p[2]], 3)])
                f = np.frombuffer(data, dtype=dt, count=e["n"], offset=off)
                off += dt.itemsize * e["n"]
                assert (f["n"] == 3).all()
                faces = f["i"].astype(np.uint32)
    if colors is None:
        colors = np.zeros(len(verts), np.uint32)
    return (np.ascontiguousarray(verts), np.ascontiguousarray(faces),
            np.ascontiguousarray(colors.astype(np.uint32)))


def _translate(m, t):
    # glm::translate(m, v): m[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
    m = m.copy()
    c = (m[0] * np.float32(t[0]) + m[1] * np.float32(t[1])) + m[2] * np.float32(t[2])
    m[3] = (c + m[3]).astype(np.float32)
    return m


def _scale(m, s):
    m = m.copy()
    for i in range(3):
        m[i] = (m[i] * np.float32(s[i])).astype(np.float32)
    return m


def _rotate(m, angle_rad, axis):
    # glm::rotate (0.9.8, gtc/matrix_transform.inl)
    a = np.float32(angle_rad)
    c = np.float32(math.cos(a))
    s = np.float32(math.sin(a))
    ax = np.asarray(axis, np.float32)
    ax = ax * np.float32(1.0 / math.sqrt(float(np.dot(ax, ax))))
    temp = (np.float32(1) - c) * ax
    R = np.zeros((3, 3), np.float32)
    R[0, 0] = c + temp[0] * ax[0]
    R[0, 1] = temp[0] * ax[1] + s * ax[2]
    R[0, 2] = temp[0] * ax[2] - s * ax[1]
    R[1, 0] = temp[1] * ax[0] - s * ax[2]
    R[1, 1] = c + temp[1] * ax[1]
    R[1, 2] = temp[1] * ax[2] + s * ax[0]
    R[2, 0] = temp[2] * ax[0] + s * ax[1]
    R[2, 1] = temp[2] * ax[1] - s * ax[0]
    R[2, 2] = c + temp[2] * ax[2]
    out = m.copy()
    for i in range(3):
        out[i] = (m[0] * R[i, 0] + m[1] * R[i, 1]) + m[2] * R[i, 2]
    return out.astype(np.float32)


def parse_spray(path, ply_path=None):
    """SceneLoader::load (src/io/scene_loader.cc:42-358).  Returns
    (domains, lights); each domain dict has id, file, transform (float32
    [4 cols][4 rows], glm column-major), object/world bound, nverts, nfaces,
    mtl tokens."""
    domains, lights = [], []
    for line in open(path):
        tok = [t for t in line.rstrip("\n").split(" ") if t]
        if not tok or tok[0].startswith("#"):
            continue
        k = tok[0]
        if k == "domain":
            domains.append({"id": len(domains), "transform": np.eye(4, dtype=np.float32),
                            "file": None, "mtl": None, "bound": None,
                            "nverts": 0, "nfaces": 0})
        elif k == "file":
            f = tok[1]
            domains[-1]["file"] = f if not ply_path else os.path.join(ply_path, f)
        elif k == "mtl":
            domains[-1]["mtl"] = tok[1:]
        elif k == "bound":
            b = [np.float32(float(x)) for x in tok[1:7]]
            domains[-1]["bound"] = np.array(b, np.float32)
        elif k == "scale":
            domains[-1]["transform"] = _scale(domains[-1]["transform"],
                                              [float(x) for x in tok[1:4]])
        elif k == "rotate":
            axis = {"x": (1, 0, 0), "y": (0, 1, 0), "z": (0, 0, 1)}[tok[1]]
            domains[-1]["transform"] = _rotate(domains[-1]["transform"],
                                               math.radians(float(tok[2])), axis)
        elif k == "translate":
            domains[-1]["transform"] = _translate(domains[-1]["transform"],
                                                  [float(x) for x in tok[1:4]])
        elif k == "face":
            domains[-1]["nfaces"] = int(tok[1])
        elif k == "vertex":
            domains[-1]["nverts"] = int(tok[1])
        elif k == "light":
            if tok[1] == "point":
                lights.append({"type": "point",
                               "pos": np.array([float(x) for x in tok[2:5]], np.float32),
                               "rad": np.array([float(x) for x in tok[5:8]], np.float32)})
            else:
                lights.append({"type": "diffuse",
                               "rad": np.array([float(x) for x in tok[2:5]], np.float32)})
        else:
            raise ValueError("unknown tag name " + k)
    for d in domains:
        b = d["bound"]
        wb = np.zeros(6, np.float32)
        lib().or_world_aabb(_p(f32(d["transform"]).reshape(16)),
                            _p(f32(b[:3])), _p(f32(b[3:])), _p(wb))
        d["world_bound"] = wb
    return domains, lights


def load_domain_mesh(d):
    """TriMeshBuffer::load (trimesh_buffer.cc:117-169): PLY, transform,
    normals.  Returns (verts_world, faces, colors, normals)."""
    v, f, c = load_ply(d["file"])
    v = v.copy()
    m = f32(d["transform"]).reshape(16)
    if not np.array_equal(d["transform"], np.eye(4, dtype=np.float32)):
        lib().or_transform_vertices(_p(m), _p(v), len(v))
    n = np.zeros_like(v)
    lib().or_compute_normals(_p(v), len(v), _p(f), len(f), _p(n))
    return v, f, c, n


# --------------------------------------------------------------------------
# C entry points
# --------------------------------------------------------------------------

def camera_init(pos, lookat, up, vfov, w, h):
    cam = np.zeros(14, np.float32)
    lib().or_camera_init(_p(f32(pos)), _p(f32(lookat)), _p(f32(up)),
                         float(vfov), int(w), int(h), _p(cam))
    return cam


def eye_rays_ooc(cam, image_w, spp, tile):
    tx, ty, tw, th = tile
    n = tw * th * spp
    org = np.zeros((n, 3), np.float32)
    d = np.zeros((n, 3), np.float32)
    pix = np.zeros(n, np.int32)
    sam = np.zeros(n, np.int32)
    lib().or_eye_rays_ooc(_p(cam), image_w, spp, tx, ty, tw, th, _p(org), _p(d),
                          _p(pix), _p(sam))
    return org, d, pix, sam


def eye_rays_insitu(cam, image_w, spp, btile, tile):
    tx, ty, tw, th = tile
    n = tw * th * spp
    org = np.zeros((n, 3), np.float32)
    d = np.zeros((n, 3), np.float32)
    pix = np.zeros(n, np.int32)
    sam = np.zeros(n, np.int32)
    lib().or_eye_rays_insitu(_p(cam), image_w, spp, *btile, tx, ty, tw, th,
                             _p(org), _p(d), _p(pix), _p(sam))
    return org, d, pix, sam


def domain_query(org, d, boxes, maxhits):
    org, d, boxes = f32(org), f32(d), f32(boxes)
    n = len(org)
    ids = np.full((n, maxhits), -1, np.int32)
    ts = np.zeros((n, maxhits), np.float32)
    cnt = np.zeros(n, np.int32)
    over = lib().or_domain_query(_p(org), _p(d), n, _p(boxes), len(boxes), maxhits,
                                 _p(ids), _p(ts), _p(cnt))
    return ids, ts, cnt, over


def prep_tris(v, f):
    tri = np.zeros((len(f), 12), np.float32)
    lib().or_prep_tris(_p(f32(v)), _p(u32(f)), len(f), _p(tri))
    return tri


def brute_intersect(tri, org, d, tnear=None, tfar=None):
    n = len(org)
    t = np.zeros(n, np.float32)
    u = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    p = np.zeros(n, np.uint32)
    lib().or_brute_intersect(_p(f32(tri)), len(tri), _p(f32(org)), _p(f32(d)),
                             _p(None if tnear is None else f32(tnear)),
                             _p(None if tfar is None else f32(tfar)), n,
                             _p(t), _p(u), _p(v), _p(p))
    return t, u, v, p


def brute_occluded(tri, org, d, tnear=None, tfar=None):
    n = len(org)
    o = np.zeros(n, np.uint8)
    lib().or_brute_occluded(_p(f32(tri)), len(tri), _p(f32(org)), _p(f32(d)),
                            _p(None if tnear is None else f32(tnear)),
                            _p(None if tfar is None else f32(tfar)), n, _p(o))
    return o


def f64_intersect(v, f, org, d, tnear=0.001):
    n = len(org)
    t = np.zeros(n, np.float64)
    p = np.zeros(n, np.int32)
    m = np.zeros(n, np.uint8)
    lib().or_f64_intersect(_p(f32(v)), _p(u32(f)), len(f), _p(f32(org)), _p(f32(d)),
                           float(tnear), n, _p(t), _p(p), _p(m))
    return t, p, m


def epilogue(faces, colors, normals, prim, u, v):
    n = len(prim)
    col = np.zeros(n, np.uint32)
    ns = np.zeros((n, 3), np.float32)
    lib().or_epilogue(_p(u32(faces)), _p(u32(colors)), _p(f32(normals)), _p(u32(prim)),
                      _p(f32(u)), _p(f32(v)), n, _p(col), _p(ns))
    return col, ns


class Bvh:
    def __init__(self, v, f):
        self._v, self._f = f32(v), u32(f)
        self.h = lib().or_bvh_build(_p(self._v), _p(self._f), len(self._f))
        self.nf = len(f)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_bvh_free(self.h)
            self.h = None

    @property
    def num_nodes(self):
        return lib().or_bvh_num_nodes(self.h)

    @property
    def depth(self):
        return lib().or_bvh_depth(self.h)

    def export(self):
        nodes = np.zeros((self.num_nodes, 16), np.float32)
        order = np.zeros(self.nf, np.uint32)
        lib().or_bvh_export(self.h, _p(nodes), _p(order))
        return nodes, order

    def intersect(self, org, d, tnear=None, tfar=None):
        n = len(org)
        t = np.zeros(n, np.float32)
        u = np.zeros(n, np.float32)
        v = np.zeros(n, np.float32)
        p = np.zeros(n, np.uint32)
        c = Counts()
        lib().or_bvh_intersect(self.h, _p(f32(org)), _p(f32(d)),
                               _p(None if tnear is None else f32(tnear)),
                               _p(None if tfar is None else f32(tfar)), n,
                               _p(t), _p(u), _p(v), _p(p), C.byref(c))
        return t, u, v, p, c.as_dict()

    def occluded(self, org, d, tnear=None, tfar=None):
        n = len(org)
        o = np.zeros(n, np.uint8)
        c = Counts()
        lib().or_bvh_occluded(self.h, _p(f32(org)), _p(f32(d)),
                              _p(None if tnear is None else f32(tnear)),
                              _p(None if tfar is None else f32(tfar)), n, _p(o),
                              C.byref(c))
        return o, c.as_dict()


class Scene:
    """Whole-scene oracle: every domain resident, domain list per ray."""

    def __init__(self, ndomains):
        self.h = lib().or_scene_create(ndomains)
        self.ndomains = ndomains

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_scene_free(self.h)
            self.h = None

    def set_domain(self, i, v, f, colors, normals, box):
        r = lib().or_scene_set_domain(self.h, i, _p(f32(v)), len(v), _p(u32(f)), len(f),
                                      _p(u32(colors)), _p(f32(normals)), _p(f32(box)))
        assert r == 0

    def set_box(self, i, box):
        """A domain owned elsewhere: listed by the domain query, no mesh."""
        assert lib().or_scene_set_box(self.h, i, _p(f32(box))) == 0

    def intersect(self, org, d, nthreads=0):
        n = len(org)
        hits = np.zeros(n, HIT_DTYPE)
        c = Counts()
        lib().or_scene_intersect(self.h, _p(f32(org)), _p(f32(d)), n, _p(hits),
                                 C.byref(c), int(nthreads))
        return hits, c.as_dict()

    def occluded(self, org, d, nthreads=0):
        n = len(org)
        o = np.zeros(n, np.uint8)
        c = Counts()
        lib().or_scene_occluded(self.h, _p(f32(org)), _p(f32(d)), n, _p(o), C.byref(c),
                                int(nthreads))
        return o, c.as_dict()


def load_scene(spray_path, ply_path=None, only=None):
    """Parse a .spray file and build the whole-scene oracle; ``only``: the
    domain ids whose meshes are resident (the others keep just their box)."""
    domains, lights = parse_spray(spray_path, ply_path)
    sc = Scene(len(domains))
    cache = {}
    for d in domains:
        if only is not None and d["id"] not in only:
            sc.set_box(d["id"], d["world_bound"])
            continue
        key = (d["file"], d["transform"].tobytes())
        if key not in cache:
            cache[key] = load_domain_mesh(d)
        v, f, c, n = cache[key]
        sc.set_domain(d["id"], v, f, c, n, d["world_bound"])
    return sc, domains, lights


def spawn_shadows_pt(org, d, hits, light_pos, light_rad, ks, shininess):
    n = len(org)
    so = np.zeros((n, 3), np.float32)
    sd = np.zeros((n, 3), np.float32)
    src = np.zeros(n, np.int32)
    m = lib().or_spawn_shadows_pt(_p(f32(org)), _p(f32(d)), _p(hits), n,
                                  _p(f32(light_pos)), _p(f32(light_rad)), _p(f32(ks)),
                                  float(shininess), _p(so), _p(sd), _p(src))
    return so[:m].copy(), sd[:m].copy(), src[:m].copy()


def spawn_shadows_ao(org, d, pixid, hits, nsamples):
    n = len(org)
    so = np.zeros((n * nsamples, 3), np.float32)
    sd = np.zeros((n * nsamples, 3), np.float32)
    src = np.zeros(n * nsamples, np.int32)
    m = lib().or_spawn_shadows_ao(_p(f32(org)), _p(f32(d)),
                                  _p(np.ascontiguousarray(pixid, np.int32)), _p(hits),
                                  n, int(nsamples), _p(so), _p(sd), _p(src))
    return so[:m].copy(), sd[:m].copy(), src[:m].copy()


# ---------------------------------------------------------------------------
# frames: path shading, film, tiles (ooc::ShaderPt / ShaderAo, TContext::
# retire, TileList) -- the CPU restatement the frame-layer tests check
# ---------------------------------------------------------------------------
SHADER_PT, SHADER_AO = 0, 1
LIGHT_POINT, LIGHT_HEMISPHERE = 0, 1
BSDF = {"diffuse": 0, "mirror": 1, "glass": 2, "transmission": 3}


class OrLight(C.Structure):
    _fields_ = [("type", C.c_int32), ("pos", C.c_float * 3), ("radiance", C.c_float * 3)]


class OrBsdf(C.Structure):
    _fields_ = [("type", C.c_int32), ("p", C.c_float * 3)]


class OrShader(C.Structure):
    _fields_ = [("shader", C.c_int32), ("bounces", C.c_int32), ("samples", C.c_int32),
                ("nlights", C.c_int32), ("ks", C.c_float * 3), ("shininess", C.c_float),
                ("lights", OrLight * 8)]


def shader(kind="pt", bounces=1, samples=1, ks=(0.4, 0.4, 0.4), shininess=10.0, lights=()):
    """lights: rows (type, x, y, z, r, g, b)."""
    s = OrShader()
    s.shader = SHADER_AO if kind == "ao" else SHADER_PT
    s.bounces, s.samples, s.nlights = int(bounces), int(samples), len(lights)
    for k in range(3):
        s.ks[k] = float(ks[k])
    s.shininess = float(shininess)
    for i, l in enumerate(lights):
        s.lights[i].type = int(l[0])
        for k in range(3):
            s.lights[i].pos[k] = float(l[1 + k])
            s.lights[i].radiance[k] = float(l[4 + k])
    return s


def scene_lights(lights):
    """parse_spray lights -> rows (type, x, y, z, r, g, b)."""
    rows = []
    for l in lights:
        if l["type"] == "point":
            rows.append((LIGHT_POINT, *l["pos"], *l["rad"]))
        else:
            rows.append((LIGHT_HEMISPHERE, 0, 0, 0, *l["rad"]))
    return rows


def scene_bsdfs(domains):
    """SceneLoader::parseMaterial (scene_loader.cc:88-130) -> (type, p0, p1, p2)."""
    out = []
    for d in domains:
        t = d["mtl"]
        if not t:
            raise ValueError("domain %d has no material" % d["id"])
        if t[0] not in BSDF:
            raise ValueError("unknown material type " + t[0])
        want = 4 if t[0] in ("diffuse", "mirror") else 3
        if len(t) != want:
            raise ValueError("wrong number of material parameters")
        p = [float(x) for x in t[1:]] + [0.0] * (4 - want)
        out.append((BSDF[t[0]], *[np.float32(x) for x in p]))
    return out


def _bsdf_array(bsdfs):
    arr = (OrBsdf * max(len(bsdfs), 1))()
    for i, b in enumerate(bsdfs):
        arr[i].type = int(b[0])
        for k in range(3):
            arr[i].p[k] = float(b[1 + k])
    return arr


def shadow_slots(sh):
    return lib().or_shadow_slots(C.byref(sh))


def shade(sh, bsdfs, bounce, org, d, hits, w, valid, pixid, samid):
    """One shading pass; org/d/w/valid updated in place (next rays).
    Returns (sorg, sdir, sw, svalid, aborts)."""
    n = len(org)
    ns = shadow_slots(sh)
    so = np.zeros((n * ns, 3), np.float32)
    sd = np.zeros((n * ns, 3), np.float32)
    sw = np.zeros((n * ns, 3), np.float32)
    sv = np.zeros(n * ns, np.uint8)
    arr = _bsdf_array(bsdfs)
    for a in (org, d, w, valid):
        assert a.flags["C_CONTIGUOUS"]
    bad = lib().or_shade(C.byref(sh), C.addressof(arr), len(bsdfs), int(bounce), _p(org),
                         _p(d), _p(hits), _p(w), _p(valid),
                         _p(np.ascontiguousarray(pixid, np.int32)),
                         _p(np.ascontiguousarray(samid, np.int32)), n, _p(so), _p(sd),
                         _p(sw), _p(sv))
    return so, sd, sw, sv, bad


def film(image, pixid, spp, ns, sw, svalid, occ, scale):
    assert image.dtype == np.float32 and image.flags["C_CONTIGUOUS"]
    lib().or_film(_p(image), _p(np.ascontiguousarray(pixid, np.int32)), len(pixid), int(spp),
                  int(ns), _p(f32(sw)), _p(np.ascontiguousarray(svalid, np.uint8)),
                  _p(np.ascontiguousarray(occ, np.uint8)), float(scale))


def tile_list(image_w, image_h, spp, nranks=1, rank=0, max_samples_per_rank=1024 * 1024,
              schedule="image"):
    """"image": ImageScheduleTileList::init + makeVerticalStripe
    (src/render/tile.cc:208-230, 317-391); "blocking": BlockingTileList::init
    + TileList::init + makeHorizontalStripe (tile.cc:52-206)."""
    if schedule == "image":
        sw = max(image_w // nranks, 1)
        sx = rank * sw
        if sx >= image_w:
            return []
        vw = image_w - sx if (sx + sw > image_w or rank == nranks - 1) else sw
        est = (vw * image_h * spp + max_samples_per_rank - 1) // max_samples_per_rank
        th = image_h // est
        assert th > 0
        return [(sx, y, vw, min(th, image_h - y)) for y in range(0, image_h, th)]
    total = image_w * image_h * spp
    per_cluster = max_samples_per_rank * nranks
    ntiles = (total + per_cluster - 1) // per_cluster
    n1 = int(math.ceil(math.sqrt(float(ntiles))))
    assert 0 < n1 <= image_w and n1 <= image_h
    tw, th = image_w // n1, image_h // n1
    out = []
    for y in range(0, image_h, th):
        for x in range(0, image_w, tw):
            w, h = min(tw, image_w - x), min(th, image_h - y)
            assert w * h * spp <= per_cluster
            sh = max(h // nranks, 1)
            sy = y + rank * sh
            if sy >= y + h:
                out.append((0, sy, 0, 0))
            else:
                hh = (y + h - sy) if (sy + sh > y + h or rank == nranks - 1) else sh
                out.append((x, sy, w, hh))
    return out


def render_tile(scene, sh, bsdfs, cam, image_w, spp, tile, image):
    """One tile of an ooc-mode frame (ooc::Tracer::trace with exact
    resolution): eye rays, then per bounce closest hit of the live slots ->
    shade -> any hit of the shadows -> film.  Returns (radiance rays,
    shadow rays, aborts)."""
    org, d, pix, sam = eye_rays_ooc(cam, image_w, spp, tile)
    n = len(org)
    w = np.ones((n, 3), np.float32)
    valid = np.ones(n, np.uint8)
    hits = np.zeros(n, HIT_DTYPE)
    ns = shadow_slots(sh)
    nrad, nsh, bad = 0, 0, 0
    for b in range(sh.bounces):
        live = np.flatnonzero(valid)
        nrad += len(live)
        if len(live):
            h, _ = scene.intersect(org[live], d[live])
            hits[live] = h
        so, sd, sw, sv, k = shade(sh, bsdfs, b, org, d, hits, w, valid, pix, sam)
        bad += k
        occ = np.zeros(n * ns, np.uint8)
        sel = np.flatnonzero(sv)
        nsh += len(sel)
        if len(sel):
            o, _ = scene.occluded(so[sel], sd[sel])
            occ[sel] = o
        film(image, pix, spp, ns, sw, sv, occ, 1.0 / spp)
    return nrad, nsh, bad
