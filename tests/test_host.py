"""CPU tests of the product's host side (no GPU): the C-ABI library loads and
exports every symbol include/*.h declares, and its host logic (scene file,
PLY, transform, normals, camera, BVH builder) equals the oracle bit for bit."""
import ctypes as C
import os
import re
import sys

import numpy as np
import pytest

from conftest import BENCH_CAMERA, ROOT, SCENES, WAVELET2, WAVELETS64


@pytest.fixture(scope="module")
def native():
    from spray_amd import build
    build.build()
    from spray_amd import _native
    return _native


def header_symbols():
    syms = set()
    for h in ("spray_rt.h", "spray_scene.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(spray_\w+)\s*\(", txt, re.M):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_header_symbol(native):
    L = native.lib()
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing
    # and the binding declares each of them
    assert syms <= set(native.SIGNATURES), sorted(syms - set(native.SIGNATURES))


def test_no_oracle_in_product():
    """The product never references the oracle (test infrastructure)."""
    for d, _, files in os.walk(os.path.join(ROOT, "spray_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(d, f)).read()
                assert "pyoracle" not in txt and "liboracle" not in txt, f


def _parse(native, desc):
    L = native.lib()
    nd, nl = C.c_int(), C.c_int()
    err = C.create_string_buffer(256)
    assert L.spray_host_parse_scene(desc.encode(), SCENES.encode(), C.byref(nd), C.byref(nl),
                                    None, None, None, err, 256) == 0, err.value
    boxes = np.zeros((nd.value, 6), np.float32)
    tr = np.zeros((nd.value, 16), np.float32)
    lights = np.zeros((nl.value, 7), np.float32)
    L.spray_host_parse_scene(desc.encode(), SCENES.encode(), None, None, boxes.ctypes.data,
                             tr.ctypes.data, lights.ctypes.data, None, 0)
    return boxes, tr, lights


@pytest.mark.parametrize("desc", [WAVELETS64, WAVELET2])
def test_scene_file_matches_oracle(native, oracle, desc):
    boxes, tr, lights = _parse(native, desc)
    doms, ls = oracle.parse_spray(desc, SCENES)
    assert np.array_equal(boxes, np.array([d["world_bound"] for d in doms]))
    assert np.array_equal(tr, np.array([d["transform"].reshape(16) for d in doms]))
    assert len(lights) == len(ls)
    for l, o in zip(lights, ls):
        assert (l[0] == 0) == (o["type"] == "point")
        assert np.array_equal(l[4:7], o["rad"])


def test_scene_file_errors(native, tmp_path):
    L = native.lib()
    bad = tmp_path / "bad.spray"
    bad.write_text("domain\nfile a.ply\nbogus 1 2\n")
    err = C.create_string_buffer(256)
    nd = C.c_int()
    assert L.spray_host_parse_scene(str(bad).encode(), b"", C.byref(nd), None, None, None,
                                    None, err, 256) != 0
    assert b"unknown tag" in err.value
    assert L.spray_host_parse_scene(b"/nonexistent.spray", b"", C.byref(nd), None, None, None,
                                    None, err, 256) != 0


def _mesh(native, desc, i):
    L = native.lib()
    nv, nf = C.c_size_t(), C.c_size_t()
    assert L.spray_host_domain_mesh(desc.encode(), SCENES.encode(), i, C.byref(nv), C.byref(nf),
                                    None, None, None, None) == 0
    v = np.zeros((nv.value, 3), np.float32)
    f = np.zeros((nf.value, 3), np.uint32)
    c = np.zeros(nv.value, np.uint32)
    n = np.zeros((nv.value, 3), np.float32)
    L.spray_host_domain_mesh(desc.encode(), SCENES.encode(), i, C.byref(nv), C.byref(nf),
                             v.ctypes.data, f.ctypes.data, c.ctypes.data, n.ctypes.data)
    return v, f, c, n


@pytest.mark.parametrize("desc,i", [(WAVELETS64, 0), (WAVELETS64, 37), (WAVELET2, 1)])
def test_domain_mesh_matches_oracle(native, oracle, desc, i):
    v, f, c, n = _mesh(native, desc, i)
    doms, _ = oracle.parse_spray(desc, SCENES)
    ov, of, oc, on = oracle.load_domain_mesh(doms[i])
    assert np.array_equal(v, ov) and np.array_equal(f, of)
    assert np.array_equal(c, oc) and np.array_equal(n.view(np.uint32), on.view(np.uint32))


def test_ascii_ply(native, oracle, tmp_path):
    """ASCII PLY path of PlyLoader (ply_loader.cc:249-270, :304-320)."""
    v, f, c = oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))
    p = tmp_path / "w.ply"
    with open(p, "w") as fh:
        fh.write("ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
                 "property float z\nproperty uchar red\nproperty uchar green\n"
                 "property uchar blue\nelement face %d\nproperty list uchar int "
                 "vertex_indices\nend_header\n" % (len(v), len(f)))
        for k in range(len(v)):
            fh.write("%.9g %.9g %.9g %d %d %d\n" % (v[k, 0], v[k, 1], v[k, 2],
                                                   c[k] >> 16, (c[k] >> 8) & 255, c[k] & 255))
        for t in f:
            fh.write("3 %d %d %d\n" % tuple(t))
    s = tmp_path / "a.spray"
    s.write_text("domain\nfile w.ply\nbound -10 -10 -10 10 10 10\nface %d\nvertex %d\n"
                 "translate 1 2 3\n" % (len(f), len(v)))
    L = native.lib()
    nv, nf = C.c_size_t(), C.c_size_t()
    assert L.spray_host_domain_mesh(str(s).encode(), str(tmp_path).encode(), 0, C.byref(nv),
                                    C.byref(nf), None, None, None, None) == 0
    mv = np.zeros((nv.value, 3), np.float32)
    mf = np.zeros((nf.value, 3), np.uint32)
    mc = np.zeros(nv.value, np.uint32)
    L.spray_host_domain_mesh(str(s).encode(), str(tmp_path).encode(), 0, C.byref(nv),
                             C.byref(nf), mv.ctypes.data, mf.ctypes.data, mc.ctypes.data, None)
    assert np.array_equal(mv, v + np.array([1, 2, 3], np.float32))
    assert np.array_equal(mf, f) and np.array_equal(mc, c)


def test_camera_matches_oracle(native, oracle):
    import spray_amd
    for w, h, fov in [(1024, 1024, 90.0), (640, 480, 60.0), (512, 512, 45.0)]:
        a = spray_amd.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"],
                                  BENCH_CAMERA["up"], fov, w, h)
        b = oracle.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"], BENCH_CAMERA["up"],
                               fov, w, h)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _bvh(native, v, f):
    L = native.lib()
    nn, dep = C.c_size_t(), C.c_int()
    assert L.spray_rt_bvh_build_host(v.ctypes.data, len(v), f.ctypes.data, len(f),
                                     C.byref(nn), C.byref(dep), None, None, None) == 0
    nodes = np.zeros((nn.value, 16), np.float32)
    tris = np.zeros((len(f), 12), np.float32)
    prims = np.zeros(len(f), np.uint32)
    L.spray_rt_bvh_build_host(v.ctypes.data, len(v), f.ctypes.data, len(f), None, None,
                              nodes.ctypes.data, tris.ctypes.data, prims.ctypes.data)
    return nodes, tris, prims, dep.value


@pytest.mark.parametrize("kind", ["wavelet", "random", "degenerate", "tiny"])
def test_bvh_builder_matches_canonical(native, oracle, kind):
    """The product builder produces the oracle's canonical tree node for node
    (same refs, same triangle order, boxes = padded canonical boxes)."""
    rng = np.random.default_rng(9)
    if kind == "wavelet":
        v, f, _ = oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))
    elif kind == "random":
        v = rng.uniform(-5, 5, size=(6000, 3)).astype(np.float32)
        f = rng.integers(0, 6000, size=(20000, 3)).astype(np.uint32)
    elif kind == "degenerate":  # all centroids equal on two axes, duplicates
        v = np.zeros((900, 3), np.float32)
        v[:, 0] = np.repeat(np.arange(300), 3) * 0.0
        v[:, 1] = rng.uniform(0, 1, 900)
        f = np.arange(900, dtype=np.uint32).reshape(-1, 3)
    else:
        v = rng.uniform(-1, 1, size=(9, 3)).astype(np.float32)
        f = np.arange(9, dtype=np.uint32).reshape(-1, 3)
    nodes, tris, prims, depth = _bvh(native, v, f)
    ob = oracle.Bvh(v, f)
    onodes, order = ob.export()
    assert depth == ob.depth <= 24
    assert np.array_equal(prims, order)
    assert np.array_equal(nodes[:, 12:14].view(np.int32), onodes[:, 12:14].view(np.int32))
    fin = np.isfinite(onodes[:, :12])
    assert (nodes[:, 0:3][fin[:, 0:3]] <= onodes[:, 0:3][fin[:, 0:3]]).all()
    assert (nodes[:, 3:6][fin[:, 3:6]] >= onodes[:, 3:6][fin[:, 3:6]]).all()
    assert np.array_equal(tris, oracle.prep_tris(v, f[order]))


def test_bvh_depth_bound_on_skewed_input(native, oracle):
    """A chain of nested slivers drives SAH deep; the builder's median
    fallback keeps leaves at depth <= 24 (the kernels' 24-entry stack)."""
    n = 40000
    x = (np.arange(n, dtype=np.float64) ** 3 / n ** 2).astype(np.float32)
    v = np.zeros((3 * n, 3), np.float32)
    v[0::3, 0] = x
    v[1::3, 0] = x + 1e-3
    v[1::3, 1] = 1e-3
    v[2::3, 2] = 1e-3
    v[2::3, 0] = x
    f = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    nodes, tris, prims, depth = _bvh(native, v, f)
    assert depth <= 24
    assert depth == oracle.Bvh(v, f).depth
    assert np.array_equal(prims, oracle.Bvh(v, f).export()[1])


def test_face_index_validation(native):
    L = native.lib()
    v = np.zeros((3, 3), np.float32)
    f = np.array([[0, 1, 3]], np.uint32)
    assert L.spray_rt_bvh_build_host(v.ctypes.data, 3, f.ctypes.data, 1, None, None, None,
                                     None, None) != 0


QNODE_DTYPE = np.dtype([("q", "<u2", 12), ("left", "<i4"), ("right", "<i4")])


def _qnodes(native, v, f):
    L = native.lib()
    nn = C.c_size_t()
    grid = np.zeros(6, np.float32)
    rc = L.spray_rt_qnodes_host(v.ctypes.data, len(v), f.ctypes.data, len(f), C.byref(nn),
                                grid.ctypes.data, None)
    assert rc == 0, rc
    q = np.zeros(nn.value, QNODE_DTYPE)
    assert L.spray_rt_qnodes_host(v.ctypes.data, len(v), f.ctypes.data, len(f), None, None,
                                  q.ctypes.data) == 0
    return q, grid


def _quad(axis, value, lo=-1.0, hi=1.0):
    """Two triangles spanning [lo, hi]^2 in the plane coordinate[axis] = value."""
    o = [a for a in range(3) if a != axis]
    v = np.zeros((4, 3), np.float32)
    for k, (s, t) in enumerate([(lo, lo), (hi, lo), (hi, hi), (lo, hi)]):
        v[k, axis] = value
        v[k, o[0]], v[k, o[1]] = s, t
    return v, np.array([[0, 1, 2], [0, 2, 3]], np.uint32)


@pytest.mark.parametrize("case", ["ground_y-1", "wall_x5", "wall_z-1e3", "patch_1e4",
                                  "ground_y0", "wavelet_far", "tilted"])
def test_quantized_nodes_contain_fp32_boxes(native, oracle, case):
    """flat / tiny domains away from the origin quantize
    (the upload used to fail on them), and every decoded quantized child box
    (base + q * scale, exact in float64) contains its padded fp32 box with at
    least one grid step to spare -- the per-lane any hit's culling stays
    conservative."""
    rng = np.random.default_rng(3)
    if case == "ground_y-1":
        v, f = _quad(1, -1.0, -100, 100)
    elif case == "wall_x5":
        v, f = _quad(0, 5.0)
    elif case == "wall_z-1e3":
        v, f = _quad(2, -1000.0, -0.5, 0.25)
    elif case == "patch_1e4":
        v, f = _quad(1, 1e4, 1e4, 1e4 + 0.01)
    elif case == "ground_y0":
        v, f = _quad(1, 0.0)
    elif case == "wavelet_far":
        v, f, _ = oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))
        v = (v + np.float32(3.0e4)).astype(np.float32)
    else:
        v = rng.uniform(-1, 1, size=(30, 3)).astype(np.float32) + np.float32(7.0)
        f = np.arange(30, dtype=np.uint32).reshape(-1, 3)
    nodes, _, _, _ = _bvh(native, v, f)
    q, grid = _qnodes(native, v, f)
    assert len(q) == len(nodes)
    base, scale = grid[:3].astype(np.float64), grid[3:].astype(np.float64)
    assert np.isfinite(base).all() and (scale > 0).all()
    assert np.array_equal(q["left"], nodes[:, 12].view(np.int32))
    assert np.array_equal(q["right"], nodes[:, 13].view(np.int32))
    for side in (0, 1):
        lo32 = nodes[:, 6 * side:6 * side + 3].astype(np.float64)
        hi32 = nodes[:, 6 * side + 3:6 * side + 6].astype(np.float64)
        ql = q["q"][:, 6 * side:6 * side + 3].astype(np.float64)
        qh = q["q"][:, 6 * side + 3:6 * side + 6].astype(np.float64)
        live = np.isfinite(lo32).all(1)  # the builder's never-hit box stays 0xFFFF
        assert (q["q"][~live, 6 * side:6 * side + 6] == 0xFFFF).all()
        dlo = base + ql[live] * scale
        dhi = base + qh[live] * scale
        assert (dlo + scale <= lo32[live]).all()
        assert (dhi - scale >= hi32[live]).all()


QNODE4_DTYPE = np.dtype([("q", "<u2", 24), ("child", "<i4", 4)])
Q4_STACK = 40  # rt_common.h kQ4Stack
NO_CHILD = np.int32(-2 ** 31)


@pytest.mark.parametrize("case", ["wavelet", "ground_y-1", "patch_1e4", "skewed", "tiny"])
def test_quantized_4wide_collapse(native, oracle, case):
    """The 4-wide quantized collapse the per-lane any hit walks (QNode4):
    every node is reached once from the root, the leaves are exactly the
    BVH2's leaves (same refs, each once), every decoded child box contains
    all triangles below it with a grid step to spare (culling conservative),
    and the walk's pending stack -- recomputed here as the sum of (entered
    children - 1) along each path -- equals the reported bound <= kQ4Stack."""
    rng = np.random.default_rng(5)
    if case == "wavelet":
        v, f, _ = oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))
    elif case == "ground_y-1":
        v, f = _quad(1, -1.0, -100, 100)
    elif case == "patch_1e4":
        v, f = _quad(1, 1e4, 1e4, 1e4 + 0.01)
    elif case == "skewed":  # the deep chain of test_bvh_depth_bound_on_skewed_input
        n = 20000
        x = (np.arange(n, dtype=np.float64) ** 3 / n ** 2).astype(np.float32)
        v = np.zeros((3 * n, 3), np.float32)
        v[0::3, 0] = x
        v[1::3, 0] = x + 1e-3
        v[1::3, 1] = 1e-3
        v[2::3, 2] = 1e-3
        v[2::3, 0] = x
        f = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    else:
        v = rng.uniform(-1, 1, size=(6, 3)).astype(np.float32)
        f = np.arange(6, dtype=np.uint32).reshape(-1, 3)
    v = np.ascontiguousarray(v, np.float32)
    f = np.ascontiguousarray(f, np.uint32)
    nodes, _, prims, _ = _bvh(native, v, f)
    L = native.lib()
    nn, bound = C.c_size_t(), C.c_int()
    grid = np.zeros(6, np.float32)
    assert L.spray_rt_qnodes4_host(v.ctypes.data, len(v), f.ctypes.data, len(f), C.byref(nn),
                                   C.byref(bound), grid.ctypes.data, None) == 0
    q = np.zeros(nn.value, QNODE4_DTYPE)
    assert L.spray_rt_qnodes4_host(v.ctypes.data, len(v), f.ctypes.data, len(f), None, None,
                                   None, q.ctypes.data) == 0
    base, scale = grid[:3].astype(np.float64), grid[3:].astype(np.float64)
    refs = nodes[:, 12:14].view(np.int32)
    live = np.stack([np.isfinite(nodes[:, 0]), np.isfinite(nodes[:, 6])], 1)  # never-hit boxes drop
    bvh2_leaves = sorted(int(r) for r in refs[live & (refs < 0) & (refs != NO_CHILD)])
    tri_v = v[f[prims]].astype(np.float64)  # leaf order, [ntris][3][3]
    seen = np.zeros(len(q), np.int32)
    leaves, worst = [], 0

    def walk(i, pend):
        nonlocal worst
        seen[i] += 1
        kids = [int(c) for c in q["child"][i] if c != NO_CHILD]
        assert 1 <= len(kids) <= 4
        p2 = pend + len(kids) - 1
        worst = max(worst, p2)
        lo_all, hi_all = [], []
        for k, c in enumerate(q["child"][i]):
            if c == NO_CHILD:
                continue
            if c >= 0:
                lo, hi = walk(int(c), p2)
            else:
                enc = ~int(c)
                first, cnt = int(enc) >> 2, (int(enc) & 3) + 1
                leaves.append(int(c))
                pts = tri_v[first:first + cnt].reshape(-1, 3)
                lo, hi = pts.min(0), pts.max(0)
            qq = q["q"][i, 6 * k:6 * k + 6].astype(np.float64)
            assert (base + qq[:3] * scale + scale <= lo).all()
            assert (base + qq[3:] * scale - scale >= hi).all()
            lo_all.append(lo)
            hi_all.append(hi)
        return np.min(lo_all, 0), np.max(hi_all, 0)

    sys.setrecursionlimit(10000)
    walk(0, 0)
    assert (seen == 1).all()
    assert sorted(leaves) == bvh2_leaves
    assert worst == bound.value <= Q4_STACK
    if case == "wavelet":  # the collapse halves the node count of a real mesh
        assert len(q) < 0.6 * len(nodes)


def test_scene_adapter_header_compiles():
    """include/spray_scene.hpp (the SceneT drop-in) is self-contained C++17
    over the C ABI: it compiles on its own, and the C++ caller test
    (tests/cpp/scene_adapter_test.cpp) builds against it."""
    import subprocess
    inc = os.path.join(ROOT, "include")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I" + inc,
                        "-x", "c++", "-"], input='#include "spray_scene.hpp"\n'
                       "template class spray_amd::Scene<>;\nint main() { return 0; }\n",
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    src = os.path.join(ROOT, "tests", "cpp", "scene_adapter_test.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-fopenmp", "-Wall", "-I" + inc,
                        "-I" + os.path.join(ROOT, "oracle"), src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
