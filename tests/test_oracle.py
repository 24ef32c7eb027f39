"""CPU tests of the oracle itself (no GPU): golden vectors, internal
consistency (BVH == brute force bit for bit), the float64 checker (the
north-star 1e-4 tolerance), and the survey's known answers."""
import json
import os

import numpy as np
import pytest

from conftest import BENCH_CAMERA, SCENES, WAVELET2, WAVELETS64, axis_rays, edge_rays, random_rays

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INV = 0xFFFFFFFF


@pytest.fixture(scope="module")
def wavelet(oracle):
    return oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))


def test_ply_loader(oracle, wavelet):
    v, f, c = wavelet
    assert v.shape == (2840, 3) and f.shape == (5480, 3) and c.shape == (2840,)
    assert f.max() == 2839 and f.min() == 0
    # object bound of the .spray description (examples/wavelets64/*.spray)
    assert np.allclose(v.min(0), [-10, -10, -10]) and np.allclose(v.max(0), [10, 9.324713, 10])


def test_golden_single_domain(oracle, wavelet):
    g = np.load(os.path.join(GOLDEN, "vectors_wavelet.npz"))
    v, f, _ = wavelet
    tri = oracle.prep_tris(v, f)
    t, u, vv, p = oracle.brute_intersect(tri, g["org"], g["dir"])
    assert np.array_equal(p, g["prim"])
    assert np.array_equal(t.view(np.uint32), g["t"].view(np.uint32))
    assert np.array_equal(u.view(np.uint32), g["u"].view(np.uint32))
    assert np.array_equal(vv.view(np.uint32), g["v"].view(np.uint32))
    o = oracle.brute_occluded(tri, g["org"], g["dir"])
    assert np.array_equal(o, g["occluded"])


def test_golden_scene(oracle):
    g = np.load(os.path.join(GOLDEN, "vectors_wavelets64.npz"))
    sc, doms, lights = oracle.load_scene(WAVELETS64, SCENES)
    h, _ = sc.intersect(g["org"], g["dir"])
    assert np.array_equal(h.view(np.uint8).reshape(-1, 48), g["hits"])
    so, sd, src = oracle.spawn_shadows_pt(g["org"], g["dir"], h, [0, 500, 1000], [1, 1, 1],
                                          [0.4, 0.4, 0.4], 10.0)
    assert np.array_equal(so, g["shadow_org"]) and np.array_equal(sd, g["shadow_dir"])
    assert np.array_equal(src, g["shadow_src"])
    o, _ = sc.occluded(so, sd)
    assert np.array_equal(o, g["occluded"])


@pytest.mark.parametrize("seed", [0, 1])
def test_bvh_equals_brute_force(oracle, wavelet, seed):
    v, f, _ = wavelet
    rng = np.random.default_rng(seed)
    c = (v.min(0) + v.max(0)) / 2
    o1, d1 = random_rays(rng, 3000, c, 25.0)
    o2, d2 = edge_rays(rng, v, f, 3000)
    o3, d3 = axis_rays(v, 300)
    org = np.concatenate([o1, o2, o3])
    d = np.concatenate([d1, d2, d3])
    tfar = np.full(len(org), np.inf, np.float32)
    tfar[::4] = 28.0
    tri = oracle.prep_tris(v, f)
    bvh = oracle.Bvh(v, f)
    t, u, vv, p = oracle.brute_intersect(tri, org, d, None, tfar)
    bt, bu, bv, bp, cnt = bvh.intersect(org, d, None, tfar)
    assert np.array_equal(p, bp)
    assert np.array_equal(t.view(np.uint32), bt.view(np.uint32))
    assert np.array_equal(u.view(np.uint32), bu.view(np.uint32))
    assert np.array_equal(vv.view(np.uint32), bv.view(np.uint32))
    o = oracle.brute_occluded(tri, org, d, None, tfar)
    bo, _ = bvh.occluded(org, d, None, tfar)
    assert np.array_equal(o, bo)
    assert cnt["nodes"] < len(org) * bvh.num_nodes / 10  # culling works


@pytest.mark.parametrize("scale,shift", [(0.05, 0.0), (0.05, 1.0e4), (1.0, 3.0e4)])
def test_bvh_equals_brute_force_far_origins(oracle, wavelet, scale, shift):
    """Culling stays conservative for origins hundreds to thousands of domain
    extents away and for domains at large coordinates (the per-ray origin
    slack of the slab test, oracle.c ray_prep): rays aimed at vertices and
    edge midpoints -- the triangles touching their leaf boxes' faces."""
    v, f, _ = wavelet
    v = (v * np.float32(scale) + np.float32(shift)).astype(np.float32)
    ext = float((v.max(0) - v.min(0)).max())
    rng = np.random.default_rng(17)
    org, d = [], []
    for k in (370.0, 2000.0, 9000.0):
        fi = f[rng.integers(0, len(f), 2000)]
        a, b = v[fi[:, 0]], v[fi[:, 1]]
        w = rng.integers(0, 3, len(fi))[:, None]
        tgt = np.where(w == 0, a, np.where(w == 1, (a + b) * np.float32(0.5), b)).astype(float)
        u = rng.normal(size=(len(fi), 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        o = tgt + u * k * ext
        dd = tgt - o
        org.append(o.astype(np.float32))
        d.append((dd / np.linalg.norm(dd, axis=1, keepdims=True)).astype(np.float32))
    org, d = np.concatenate(org), np.concatenate(d)
    tri = oracle.prep_tris(v, f)
    bvh = oracle.Bvh(v, f)
    t, _, _, p = oracle.brute_intersect(tri, org, d)
    bt, _, _, bp, _ = bvh.intersect(org, d)
    assert (p != INV).mean() > 0.3
    assert np.array_equal(p, bp) and np.array_equal(t.view(np.uint32), bt.view(np.uint32))
    assert np.array_equal(oracle.brute_occluded(tri, org, d), bvh.occluded(org, d)[0])


def test_float64_checker_tolerance(oracle, wavelet):
    """North-star: hit t within 1e-4 relative (and the same primitive) of an
    exact evaluation, except flagged near-edge hits (the crack cases where
    any non-watertight intersector -- Embree 2 included -- may pick a
    neighbour)."""
    v, f, _ = wavelet
    rng = np.random.default_rng(3)
    c = (v.min(0) + v.max(0)) / 2
    org, d = random_rays(rng, 6000, c, 25.0)
    t, u, vv, p = oracle.brute_intersect(oracle.prep_tris(v, f), org, d)
    t64, p64, margin = oracle.f64_intersect(v, f, org, d)
    hit = p != INV
    ok = ~margin.astype(bool)
    assert np.array_equal(hit[ok], (p64 >= 0)[ok])
    h = hit & ok
    assert np.array_equal(p[h].astype(np.int64), p64[h].astype(np.int64))
    rel = np.abs(t[h] - t64[h]) / np.abs(t64[h])
    assert rel.max() < 1e-4
    # barycentrics reconstruct the hit point: (1-u-v) v0 + u v1 + v v2
    P = org[h] + t[h, None] * d[h]
    tri = f[p[h]]
    Q = ((1 - u[h] - vv[h])[:, None] * v[tri[:, 0]] + u[h, None] * v[tri[:, 1]] +
         vv[h, None] * v[tri[:, 2]])
    assert np.abs(P - Q).max() < 1e-3
    assert margin.sum() < len(org) * 0.01


def test_geometry_normal_convention(oracle):
    """Ng = (v0 - v1) x (v2 - v0) (Embree 2 MoellerTrumbore, e1 = v0 - v1,
    e2 = v2 - v0), unnormalised; hits from both sides (no backface culling)."""
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    f = np.array([[0, 1, 2]], np.uint32)
    tri = oracle.prep_tris(v, f)
    assert np.array_equal(tri[0, 9:12], np.array([0, 0, -1], np.float32))
    org = np.array([[0.25, 0.25, 2], [0.25, 0.25, -2]], np.float32)
    d = np.array([[0, 0, -1], [0, 0, 1]], np.float32)
    t, u, vv, p = oracle.brute_intersect(tri, org, d)
    assert (p == 0).all() and np.allclose(t, 2) and np.allclose(u, 0.25) and np.allclose(vv, 0.25)


def test_tnear_tfar_semantics(oracle):
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    f = np.array([[0, 1, 2]], np.uint32)
    tri = oracle.prep_tris(v, f)
    org = np.tile(np.array([[0.25, 0.25, 2]], np.float32), (4, 1))
    d = np.tile(np.array([[0, 0, -1]], np.float32), (4, 1))
    tnear = np.array([0.001, 2.0, 0.001, 0.001], np.float32)
    tfar = np.array([np.inf, np.inf, 2.0, 1.999], np.float32)
    _, _, _, p = oracle.brute_intersect(tri, org, d, tnear, tfar)
    # t must exceed tnear strictly; t == tfar is accepted (T <= |den| tfar)
    assert p.tolist() == [0, INV, 0, INV]
    o = oracle.brute_occluded(tri, org, d, tnear, tfar)
    assert o.tolist() == [1, 0, 1, 0]


def test_closest_hit_tie_breaks_on_face_index(oracle):
    """Two coincident triangles: the smaller face index wins, whatever the
    traversal order (order-independent closest hit)."""
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    f = np.array([[0, 1, 2], [0, 1, 2], [0, 1, 2]], np.uint32)
    org = np.array([[0.25, 0.25, 2]], np.float32)
    d = np.array([[0, 0, -1]], np.float32)
    _, _, _, p = oracle.brute_intersect(oracle.prep_tris(v, f), org, d)
    assert p[0] == 0
    _, _, _, bp, _ = oracle.Bvh(v, f).intersect(org, d)
    assert bp[0] == 0


def test_survey_known_answers(oracle):
    """48x48 pixel-centre probe of wavelets64 at 1024^2:
    primary hit fraction ~0.274, mean 1.38 domains per ray, max 10."""
    sc, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    cam = oracle.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"], BENCH_CAMERA["up"],
                             BENCH_CAMERA["fov"], 1024, 1024)
    xs = (np.arange(48) + 0.5) * 1024 / 48
    d = np.zeros((48 * 48, 3), np.float32)
    for i, y in enumerate(xs):
        for j, x in enumerate(xs):
            dv = np.zeros(3, np.float32)
            oracle.lib().or_camera_ray(oracle._p(cam), float(x), float(y), oracle._p(dv))
            d[i * 48 + j] = dv
    org = np.tile(cam[:3], (len(d), 1)).astype(np.float32)
    h, _ = sc.intersect(org, d)
    boxes = np.array([x["world_bound"] for x in doms], np.float32)
    _, _, cnt, _ = oracle.domain_query(org, d, boxes, 64)
    assert abs((h["domain"] >= 0).mean() - 0.274) < 0.002
    assert abs(cnt.mean() - 1.38) < 0.01 and cnt.max() == 10


def test_domain_lists_sorted(oracle):
    _, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    boxes = np.array([x["world_bound"] for x in doms], np.float32)
    rng = np.random.default_rng(4)
    org, d = random_rays(rng, 5000, np.array([30, 28, 30], np.float32), 70.0)
    ids, ts, cnt, over = oracle.domain_query(org, d, boxes, 64)
    assert over == 0 and cnt.max() > 3
    for i in np.nonzero(cnt > 1)[0][:500]:
        k = cnt[i]
        key = list(zip(ts[i, :k].tolist(), ids[i, :k].tolist()))
        assert key == sorted(key)
    # truncation keeps the nearest entries
    ids2, ts2, cnt2, over2 = oracle.domain_query(org, d, boxes, 2)
    assert over2 > 0
    m = cnt >= 2
    assert np.array_equal(ids2[m], ids[m, :2])


def test_eye_rays_seeding(oracle):
    """ooc jitter is seeded by the TILE-LOCAL bufid (ooc_tracer.inl:151), so
    equal offsets in different blocking tiles get equal jitter."""
    cam = oracle.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"], BENCH_CAMERA["up"],
                             BENCH_CAMERA["fov"], 1024, 1024)
    _, d0, p0, s0 = oracle.eye_rays_ooc(cam, 1024, 8, (0, 0, 16, 4))
    _, d1, p1, s1 = oracle.eye_rays_ooc(cam, 1024, 8, (0, 128, 16, 4))
    assert np.array_equal(s0, s1) and not np.array_equal(p0, p1)
    st = np.zeros(1, np.uint32)
    st[0] = oracle.lib().or_sampler_init1(5)
    a = oracle.lib().or_sampler_get1d(oracle._p(st))
    assert 0.0 <= a < 1.0
    # 1 spp: no jitter, pixel corner (genSingleEyes)
    _, d2, _, _ = oracle.eye_rays_ooc(cam, 1024, 1, (3, 5, 1, 1))
    dv = np.zeros(3, np.float32)
    oracle.lib().or_camera_ray(oracle._p(cam), 3.0, 5.0, oracle._p(dv))
    assert np.array_equal(d2[0], dv)


def test_workload_counts_fixture(oracle):
    """The committed per-config counts of the bench workload (first tile
    re-derived here; the whole frame is regenerated by make_golden.py)."""
    c = json.load(open(os.path.join(GOLDEN, "workload_counts.json")))
    assert c["primary"]["rays"] == 8388608
    assert 0.26 < c["primary_hits"] / c["primary"]["rays"] < 0.29
    assert c["shadow"]["rays"] <= c["primary_hits"]
    sc, _, _ = oracle.load_scene(WAVELETS64, SCENES)
    cam = oracle.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"], BENCH_CAMERA["up"],
                             BENCH_CAMERA["fov"], 1024, 1024)
    org, d, _, _ = oracle.eye_rays_ooc(cam, 1024, 8, (0, 0, 1024, 128))
    _, c0 = sc.intersect(org, d)
    assert 0 < c0["nodes"] < c["primary"]["nodes"]


def test_two_domain_scene(oracle):
    sc, doms, lights = oracle.load_scene(WAVELET2, SCENES)
    assert len(doms) == 2 and len(lights) == 2
    assert lights[1]["type"] == "diffuse"
    cam = oracle.camera_init([0, 0, 40], [0, 0, 0], [0, 1, 0], 60, 64, 64)
    org, d, _, _ = oracle.eye_rays_ooc(cam, 64, 1, (0, 0, 64, 64))
    h, _ = sc.intersect(org, d)
    assert set(np.unique(h["domain"])) == {-1, 0, 1}
