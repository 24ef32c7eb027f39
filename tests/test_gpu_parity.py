"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Integer/index results (primID, geomID, color, domain lists, counts) must be
identical; float results (t, u, v, Ng, Ns) are required BIT-identical too,
because the kernels and the oracle evaluate the same operations in the same
order (-ffp-contract=off, explicit fmaf) -- the reference's VBuf compares t
with == (ooc_vbuf.cc:41-52).  North-star tolerance vs Embree (1e-4 relative)
is checked against the float64 checker in test_oracle.py.
"""
import numpy as np
import pytest

from conftest import (BENCH_CAMERA, SCENES, WAVELET2, WAVELETS64, axis_rays,
                      edge_rays, random_rays)

pytestmark = pytest.mark.gpu

INV = 0xFFFFFFFF


@pytest.fixture(scope="module")
def spray():
    import torch  # noqa: F401  (one HIP runtime in the process)
    import spray_amd
    return spray_amd


@pytest.fixture(scope="module")
def wavelet(oracle):
    v, f, c = oracle.load_ply(SCENES + "/wavelet.ply")
    n = np.zeros_like(v)
    oracle.lib().or_compute_normals(oracle._p(v), len(v), oracle._p(f), len(f), oracle._p(n))
    return v, f, c, n


@pytest.fixture(scope="module")
def ctx1(spray, wavelet):
    v, f, c, n = wavelet
    ctx = spray.RtContext(0)
    ctx.upload_domain(0, v, f, c, n)
    # a translated copy in slot 3 (segments test)
    ctx.upload_domain(3, v + np.float32(30.0), f, c, n)
    yield ctx
    ctx.close()


def ray_batch(rng, wavelet, n=4000):
    v, f, _, _ = wavelet
    c = (v.min(0) + v.max(0)) / 2
    o1, d1 = random_rays(rng, n, c, 25.0)
    o2, d2 = edge_rays(rng, v, f, n // 2)
    o3, d3 = axis_rays(v, 400)
    # rays starting inside the mesh bound
    o4 = (c + rng.uniform(-8, 8, size=(n // 4, 3))).astype(np.float32)
    d4 = rng.normal(size=(n // 4, 3)).astype(np.float32)
    d4 /= np.linalg.norm(d4, axis=1, keepdims=True)
    org = np.concatenate([o1, o2, o3, o4]).astype(np.float32)
    d = np.concatenate([d1, d2, d3, d4]).astype(np.float32)
    return org, d


def rtc_records(spray, org, d, tnear=0.001, tfar=np.inf):
    """RTCRayUtil::makeRadianceRay (rays.h:345-363) records."""
    r = np.zeros(len(org), spray.RTC_ISECT_DTYPE)
    r["org"] = org
    r["dir"] = d
    r["tnear"] = tnear
    r["tfar"] = tfar
    r["geomID"] = INV
    r["primID"] = INV
    r["instID"] = INV
    r["mask"] = 0xFFFFFFFF
    return r


def test_intersect1M_matches_oracle(spray, oracle, wavelet, ctx1):
    v, f, c, n = wavelet
    rng = np.random.default_rng(1)
    org, d = ray_batch(rng, wavelet)
    # per-ray tnear / tfar variations (Embree accepts tnear < t <= tfar)
    tnear = np.full(len(org), 0.001, np.float32)
    tfar = np.full(len(org), np.inf, np.float32)
    tnear[::7] = 5.0
    tfar[::5] = 30.0
    recs = rtc_records(spray, org, d, tnear, tfar)
    before = recs.copy()
    ctx1.intersect1M(0, recs)
    tri = oracle.prep_tris(v, f)
    t, u, vv, p = oracle.brute_intersect(tri, org, d, tnear, tfar)
    hit = p != INV
    assert 0.2 < hit.mean() < 0.9
    assert np.array_equal(recs["primID"], p)
    assert np.array_equal(recs["geomID"][hit], np.zeros(hit.sum(), np.uint32))
    assert np.array_equal(recs["tfar"].view(np.uint32), t.view(np.uint32))
    assert np.array_equal(recs["u"][hit].view(np.uint32), u[hit].view(np.uint32))
    assert np.array_equal(recs["v"][hit].view(np.uint32), vv[hit].view(np.uint32))
    assert np.array_equal(recs["Ng"][hit], tri[p[hit], 9:12])
    col, ns = oracle.epilogue(f, c, n, p, u, vv)
    assert np.array_equal(recs["color"][hit], col[hit])
    assert np.array_equal(recs["Ns"][hit].view(np.uint32), ns[hit].view(np.uint32))
    # misses: record untouched (tfar stays, geomID stays invalid)
    assert np.array_equal(recs[~hit].view(np.uint8), before[~hit].view(np.uint8))
    # instID is never written
    assert (recs["instID"] == INV).all()


def test_occluded1M_matches_oracle(spray, oracle, wavelet, ctx1):
    v, f, _, _ = wavelet
    rng = np.random.default_rng(2)
    org, d = ray_batch(rng, wavelet)
    tfar = np.full(len(org), np.inf, np.float32)
    tfar[::3] = 10.0
    recs = rtc_records(spray, org, d, 0.001, tfar)
    ctx1.occluded1M(0, recs)
    occ = oracle.brute_occluded(oracle.prep_tris(v, f), org, d, None, tfar)
    got = recs["geomID"] != INV
    assert np.array_equal(got, occ.astype(bool))
    assert (recs["geomID"][got] == 0).all()
    assert np.array_equal(recs["tfar"], tfar)  # occlusion never writes tfar


def test_segments_two_slots(spray, oracle, wavelet, ctx1):
    v, f, c, n = wavelet
    rng = np.random.default_rng(3)
    org, d = ray_batch(rng, wavelet, 1000)
    m = len(org) // 2
    org2 = org.copy()
    org2[m:] += np.float32(30.0)  # second half aimed at slot 3's copy
    recs = rtc_records(spray, org2, d)
    ctx1.intersect_segments([0, 3], [0, m, len(org)], recs)
    tri0 = oracle.prep_tris(v, f)
    tri3 = oracle.prep_tris(v + np.float32(30.0), f)
    t0, _, _, p0 = oracle.brute_intersect(tri0, org2[:m], d[:m])
    t3, _, _, p3 = oracle.brute_intersect(tri3, org2[m:], d[m:])
    assert np.array_equal(recs["primID"][:m], p0)
    assert np.array_equal(recs["primID"][m:], p3)
    assert np.array_equal(recs["tfar"][:m], t0)
    assert np.array_equal(recs["tfar"][m:], t3)
    # occluded segments
    recs = rtc_records(spray, org2, d)
    ctx1.occluded_segments([0, 3], [0, m, len(org)], recs)
    o0 = oracle.brute_occluded(tri0, org2[:m], d[:m])
    o3 = oracle.brute_occluded(tri3, org2[m:], d[m:])
    assert np.array_equal(recs["geomID"] != INV, np.concatenate([o0, o3]).astype(bool))


def test_empty_and_errors(spray, ctx1):
    recs = np.zeros(0, spray.RTC_ISECT_DTYPE)
    ctx1.intersect1M(0, recs)  # M = 0 is a no-op
    with pytest.raises(spray.SprayRtError):
        ctx1.intersect1M(7, np.zeros(4, spray.RTC_ISECT_DTYPE))  # unloaded slot
    with pytest.raises(spray.SprayRtError):
        ctx1.upload_domain(1, np.zeros((3, 3), np.float32), np.array([[0, 1, 5]]))


def test_tiny_meshes(spray, oracle):
    """1..5 triangles: root-leaf layout and tiny trees."""
    ctx = spray.RtContext(0)
    rng = np.random.default_rng(4)
    for nt in [1, 2, 4, 5, 9]:
        v = rng.uniform(-1, 1, size=(3 * nt, 3)).astype(np.float32)
        f = np.arange(3 * nt, dtype=np.uint32).reshape(-1, 3)
        ctx.upload_domain(0, v, f)
        org, d = random_rays(rng, 512, np.zeros(3), 3.0)
        recs = rtc_records(spray, org, d)
        ctx.intersect1M(0, recs)
        t, u, vv, p = oracle.brute_intersect(oracle.prep_tris(v, f), org, d)
        assert np.array_equal(recs["primID"], p), nt
        assert np.array_equal(recs["tfar"], t), nt
    ctx.close()


@pytest.fixture(scope="module")
def scene64(spray, oracle):
    sc = spray.Scene(WAVELETS64, SCENES, cache_size=-1, device=0)
    osc, doms, lights = oracle.load_scene(WAVELETS64, SCENES)
    yield sc, osc, doms, lights
    sc.close()


def bench_tile(oracle, tile=(384, 448, 256, 64), spp=8):
    cam = oracle.camera_init(BENCH_CAMERA["pos"], BENCH_CAMERA["lookat"], BENCH_CAMERA["up"],
                             BENCH_CAMERA["fov"], 1024, 1024)
    org, d, pix, sam = oracle.eye_rays_ooc(cam, 1024, spp, tile)
    return cam, org, d, pix


def test_domains1M_matches_oracle(spray, oracle, scene64):
    sc, osc, doms, _ = scene64
    boxes = np.array([x["world_bound"] for x in doms], np.float32)
    _, org, d, _ = bench_tile(oracle)
    rng = np.random.default_rng(5)
    o2, d2 = random_rays(rng, 3000, np.array([30, 28, 30], np.float32), 70.0)
    org = np.concatenate([org[::7], o2])
    d = np.concatenate([d[::7], d2])
    ids, ts, cnt = sc.intersectDomains(org, d, maxhits=64)
    oids, ots, ocnt, _ = oracle.domain_query(org, d, boxes, 64)
    assert np.array_equal(cnt, ocnt)
    for k in range(64):
        m = cnt > k
        assert np.array_equal(ids[m, k], oids[m, k])
        assert np.array_equal(ts[m, k].view(np.uint32), ots[m, k].view(np.uint32))
    # truncated lists keep the nearest entries
    ids3, ts3, cnt3 = sc.rt.domains1M(org, d, 3)
    oids3, ots3, ocnt3, _ = oracle.domain_query(org, d, boxes, 3)
    assert np.array_equal(cnt3, ocnt3)
    assert np.array_equal(np.where(np.arange(3) < cnt3[:, None], ids3, -1),
                          np.where(np.arange(3) < ocnt3[:, None], oids3, -1))


def test_eye_rays_match_oracle(spray, oracle):
    import torch
    cam, org, d, pix = bench_tile(oracle, (128, 256, 200, 40), 8)
    ctx = spray.RtContext(0)
    n = len(org)
    rays = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    pixid = torch.zeros(n, dtype=torch.int32, device="cuda")
    samid = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.eye_rays_ooc(cam, 1024, 8, (128, 256, 200, 40), rays, pixid, samid)
    ctx.sync()
    r = rays.cpu().numpy().view(spray.RAY_DTYPE)
    assert np.array_equal(r["org"], org)
    assert np.array_equal(r["dir"].view(np.uint32), d.view(np.uint32))
    assert np.array_equal(pixid.cpu().numpy(), pix)
    assert np.array_equal(samid.cpu().numpy(), np.arange(n))
    assert (r["tnear"] == np.float32(0.001)).all() and np.isinf(r["tfar"]).all()
    ctx.close()


def compare_hits(h, oh):
    assert np.array_equal(h["domain"], oh["domain"])
    assert np.array_equal(h["prim"], oh["prim"])
    for k in ("t", "u", "v", "ng", "ns"):
        assert np.array_equal(h[k].view(np.uint32), oh[k].view(np.uint32)), k
    assert np.array_equal(h["color"], oh["color"])


def test_scene_intersect_matches_oracle(spray, oracle, scene64):
    sc, osc, doms, _ = scene64
    _, org, d, _ = bench_tile(oracle)
    rng = np.random.default_rng(6)
    o2, d2 = random_rays(rng, 4000, np.array([30, 28, 30], np.float32), 60.0)
    org = np.concatenate([org, o2])
    d = np.concatenate([d, d2])
    rays = spray.make_rays(org, d)
    hits = sc.rt.intersect_scene(rays)
    oh, ocnt = osc.intersect(org, d)
    assert (oh["domain"] >= 0).mean() > 0.2
    compare_hits(hits, oh)


def test_scene_counts_match_canonical(spray, oracle, scene64):
    """The counting build of the GPU kernel reproduces the oracle's canonical
    node/triangle/visit counts exactly (same BVH, same traversal order)."""
    import torch
    sc, osc, _, _ = scene64
    _, org, d, _ = bench_tile(oracle, (0, 512, 512, 32), 8)
    rays = spray.make_rays(org, d)
    cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
    hits = sc.rt.intersect_scene(rays, counters=cnt)
    torch.cuda.synchronize()
    _, oc = osc.intersect(org, d)
    assert cnt.cpu().tolist() == [oc["nodes"], oc["tris"], oc["visits"]]
    so, sd, _ = oracle.spawn_shadows_pt(org, d, hits, [0, 500, 1000], [1, 1, 1],
                                        [0.4, 0.4, 0.4], 10.0)
    cnt.zero_()
    sc.rt.occluded_scene(spray.make_rays(so, sd), counters=cnt)
    torch.cuda.synchronize()
    _, oc2 = osc.occluded(so, sd)
    assert cnt.cpu().tolist() == [oc2["nodes"], oc2["tris"], oc2["visits"]]


def test_scene_occluded_and_spawn_match_oracle(spray, oracle, scene64):
    import torch
    sc, osc, doms, lights = scene64
    _, org, d, _ = bench_tile(oracle, (256, 448, 384, 48), 8)
    n = len(org)
    rays_h = spray.make_rays(org, d)
    rays = torch.from_numpy(rays_h.view(np.uint8)).cuda()
    hits = torch.zeros(n * 48, dtype=torch.uint8, device="cuda")
    sc.rt.intersect_scene(rays, hits)
    shade = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)
    srays = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    src = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    sc.rt.spawn_shadows_pt(rays, hits, n, shade, srays, src, cnt)
    occ = torch.zeros(n, dtype=torch.uint8, device="cuda")
    sc.rt.sync()
    m = int(cnt.item())
    sc.rt.occluded_scene(srays[: m * 32], occ[:m])
    sc.rt.sync()
    oh, _ = osc.intersect(org, d)
    compare_hits(hits.cpu().numpy().view(spray.HIT_DTYPE), oh)
    so, sd, osrc = oracle.spawn_shadows_pt(org, d, oh, lights[0]["pos"], lights[0]["rad"],
                                           [0.4, 0.4, 0.4], 10.0)
    assert m == len(so) and m > 1000
    sr = srays[: m * 32].cpu().numpy().view(spray.RAY_DTYPE)
    assert np.array_equal(src[:m].cpu().numpy(), osrc)
    assert np.array_equal(sr["org"].view(np.uint32), so.view(np.uint32))
    assert np.array_equal(sr["dir"].view(np.uint32), sd.view(np.uint32))
    oocc, _ = osc.occluded(so, sd)
    assert np.array_equal(occ[:m].cpu().numpy(), oocc)
    assert 0.01 < oocc.mean() < 0.99


def test_scene_per_ray_surface(spray, oracle, scene64):
    """Scene::load / intersect / occluded per ray (scene.h:157-195)."""
    sc, osc, doms, _ = scene64
    v, f, c, n = oracle.load_domain_mesh(doms[21])
    blk = sc.load(21)
    assert blk == 21  # InfiniteCache: block = domain id
    rng = np.random.default_rng(7)
    b = doms[21]["world_bound"]
    org, d = random_rays(rng, 64, (b[:3] + b[3:]) / 2, 20.0)
    tri = oracle.prep_tris(v, f)
    t, u, vv, p = oracle.brute_intersect(tri, org, d)
    occ = oracle.brute_occluded(tri, org, d)
    for i in range(64):
        hit, rec = sc.intersect(blk, org[i], d[i])
        assert hit == (p[i] != INV)
        if hit:
            assert rec["primID"] == p[i] and rec["tfar"] == t[i]
        assert sc.occluded(blk, org[i], d[i]) == bool(occ[i])


def test_lru_scene_reloads(spray, oracle):
    """LRU cache of 2 blocks over the 2-domain example forces reloads."""
    sc = spray.Scene(WAVELETS64, SCENES, cache_size=4, device=0)
    assert sc.cache_capacity() == 4
    blocks = [sc.load(i) for i in [0, 1, 2, 3, 4, 0, 5]]
    assert blocks == [0, 1, 2, 3, 0, 1, 2]
    osc, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    v, f, _, _ = oracle.load_domain_mesh(doms[5])
    rng = np.random.default_rng(8)
    b = doms[5]["world_bound"]
    org, d = random_rays(rng, 500, (b[:3] + b[3:]) / 2, 20.0)
    recs = rtc_records(spray, org, d)
    sc.rt.intersect1M(2, recs)
    _, _, _, p = oracle.brute_intersect(oracle.prep_tris(v, f), org, d)
    assert np.array_equal(recs["primID"], p)
    sc.close()


def test_two_domain_example(spray, oracle):
    sc = spray.Scene(WAVELET2, SCENES, cache_size=-1, device=0)
    osc, doms, _ = oracle.load_scene(WAVELET2, SCENES)
    cam = oracle.camera_init([0, 0, 40], [0, 0, 0], [0, 1, 0], 60, 128, 128)
    org, d, _, _ = oracle.eye_rays_ooc(cam, 128, 1, (0, 0, 128, 128))
    hits = sc.rt.intersect_scene(spray.make_rays(org, d))
    oh, _ = osc.intersect(org, d)
    compare_hits(hits, oh)
    assert set(np.unique(oh["domain"])) == {-1, 0, 1}
    sc.close()


def test_fused_spawn_matches_oracle(spray, oracle, scene64):
    """intersect_scene_spawn_pt: same hits and exactly the oracle's shadow
    rays at their source positions; occluded_scene_masked over them."""
    import torch
    sc, osc, doms, lights = scene64
    _, org, d, _ = bench_tile(oracle, (320, 400, 384, 64), 8)
    n = len(org)
    rays = torch.from_numpy(spray.make_rays(org, d).view(np.uint8)).cuda()
    hits = torch.zeros(n * 48, dtype=torch.uint8, device="cuda")
    shade = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)
    srays = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    valid = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    cnt = torch.full((1,), 123, dtype=torch.int32, device="cuda")
    sc.rt.intersect_scene_spawn_pt(rays, hits, shade, srays, valid, cnt)
    occ = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    sc.rt.occluded_scene_masked(srays, valid, occ)
    sc.rt.sync()
    oh, _ = osc.intersect(org, d)
    compare_hits(hits.cpu().numpy().view(spray.HIT_DTYPE), oh)
    so, sd, osrc = oracle.spawn_shadows_pt(org, d, oh, lights[0]["pos"], lights[0]["rad"],
                                           [0.4, 0.4, 0.4], 10.0)
    v = valid.cpu().numpy()
    assert set(np.unique(v)) <= {0, 1}
    assert np.array_equal(np.nonzero(v)[0], osrc) and int(cnt.item()) == len(osrc)
    sr = srays.cpu().numpy().view(spray.RAY_DTYPE)[osrc]
    assert np.array_equal(sr["org"].view(np.uint32), so.view(np.uint32))
    assert np.array_equal(sr["dir"].view(np.uint32), sd.view(np.uint32))
    oocc, _ = osc.occluded(so, sd)
    o = occ.cpu().numpy()
    assert np.array_equal(o[osrc], oocc)
    assert (o[v == 0] == 9).all()  # only valid rays are written


def test_masked_occlusion_sparse_patterns(spray, oracle, scene64):
    """In-wave compaction with adversarial masks: all, none, every 63rd, one
    isolated ray, random 5%."""
    import torch
    sc, osc, _, _ = scene64
    _, org, d, _ = bench_tile(oracle, (400, 500, 256, 16), 8)
    n = len(org)
    rays = torch.from_numpy(spray.make_rays(org, d).view(np.uint8)).cuda()
    ref, _ = osc.occluded(org, d)
    rng = np.random.default_rng(11)
    for mask in [np.ones(n, np.uint8), np.zeros(n, np.uint8),
                 (np.arange(n) % 63 == 5).astype(np.uint8),
                 (np.arange(n) == n // 2).astype(np.uint8),
                 (rng.uniform(size=n) < 0.05).astype(np.uint8)]:
        occ = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
        sc.rt.occluded_scene_masked(rays, torch.from_numpy(mask).cuda(), occ)
        sc.rt.sync()
        o = occ.cpu().numpy()
        assert np.array_equal(o[mask == 1], ref[mask == 1])
        assert (o[mask == 0] == 9).all()


@pytest.mark.parametrize("cut", [0, 37, 4000])
def test_fused_shadow_trace_matches_two_launches(spray, oracle, scene64, cut):
    """intersect_scene_shadow_pt (closest hit + spawn + the shadows' any hit,
    one launch, per-wave LDS queues) equals spawn_pt + occluded_scene_masked
    and the oracle, including ragged batch sizes and partial queues."""
    import torch
    sc, osc, doms, lights = scene64
    _, org, d, _ = bench_tile(oracle, (320, 400, 384, 64), 8)
    n = len(org) - cut
    org, d = org[:n], d[:n]
    rays = torch.from_numpy(spray.make_rays(org, d).view(np.uint8)).cuda()
    shade = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)
    hits = torch.zeros(n * 48, dtype=torch.uint8, device="cuda")
    occ = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    sv = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    cnt = torch.full((1,), 123, dtype=torch.int32, device="cuda")
    sc.rt.intersect_scene_shadow_pt(rays, hits, shade, occ, sv, cnt)
    hits2 = torch.zeros_like(hits)
    srays = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    valid = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    cnt2 = torch.zeros(1, dtype=torch.int32, device="cuda")
    sc.rt.intersect_scene_spawn_pt(rays, hits2, shade, srays, valid, cnt2)
    occ2 = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    sc.rt.occluded_scene_masked(srays, valid, occ2)
    sc.rt.sync()
    assert hits.cpu().numpy().tobytes() == hits2.cpu().numpy().tobytes()
    v = sv.cpu().numpy()
    assert np.array_equal(v, valid.cpu().numpy()) and set(np.unique(v)) <= {0, 1}
    assert int(cnt.item()) == int(cnt2.item()) == int(v.sum()) > 1000
    o = occ.cpu().numpy()
    assert np.array_equal(o[v == 1], occ2.cpu().numpy()[v == 1])
    assert (o[v == 0] == 9).all()
    oh, _ = osc.intersect(org, d)
    so, sd, osrc = oracle.spawn_shadows_pt(org, d, oh, lights[0]["pos"], lights[0]["rad"],
                                           [0.4, 0.4, 0.4], 10.0)
    oocc, _ = osc.occluded(so, sd)
    assert np.array_equal(np.nonzero(v)[0], osrc) and np.array_equal(o[osrc], oocc)
    assert 0 < oocc.sum() < len(oocc)


def test_scene_more_than_64_domains(spray, oracle, tmp_path):
    """A 5x5x4 grid of 100 domains (the 256-domain variants of the scene
    kernels: four mask words, larger LDS tables): closest hit, any hit and the
    fused shadow launch equal the oracle."""
    import torch
    lines = ["light point 0 500 1000 1 1 1", ""]
    for i in range(5):
        for j in range(4):
            for k in range(5):
                lines += ["domain", "file wavelet.ply", "mtl diffuse 1 1 1",
                          "bound -10.000000 -10.000000 -10.000000 10.000000 9.324713 10.000000",
                          "face 5480", "vertex 2840",
                          "translate %f %f %f" % (20.0 * i, 19.324713 * j, 20.0 * k), ""]
    desc = tmp_path / "wavelets100.spray"
    desc.write_text("\n".join(lines))
    sc = spray.Scene(str(desc), SCENES, cache_size=-1, device=0)
    osc, doms, lights = oracle.load_scene(str(desc), SCENES)
    assert len(doms) == 100
    cam = oracle.camera_init([150.0, 120.0, 150.0], [40.0, 28.0, 40.0], [0, 1, 0], 60.0, 512, 512)
    org, d, _, _ = oracle.eye_rays_ooc(cam, 512, 2, (128, 128, 256, 128))
    n = len(org)
    rays = torch.from_numpy(spray.make_rays(org, d).view(np.uint8)).cuda()
    shade = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)
    hits = torch.zeros(n * 48, dtype=torch.uint8, device="cuda")
    occ = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    sv = torch.zeros(n, dtype=torch.uint8, device="cuda")
    sc.rt.intersect_scene_shadow_pt(rays, hits, shade, occ, sv, None)
    sc.rt.sync()
    oh, _ = osc.intersect(org, d)
    assert (oh["domain"] >= 64).sum() > 1000
    compare_hits(hits.cpu().numpy().view(spray.HIT_DTYPE), oh)
    so, sd, osrc = oracle.spawn_shadows_pt(org, d, oh, lights[0]["pos"], lights[0]["rad"],
                                           [0.4, 0.4, 0.4], 10.0)
    oocc, _ = osc.occluded(so, sd)
    v = sv.cpu().numpy()
    assert np.array_equal(np.nonzero(v)[0], osrc)
    assert np.array_equal(occ.cpu().numpy()[osrc], oocc) and 0 < oocc.sum() < len(oocc)
    g = sc.rt.occluded_scene(spray.make_rays(so, sd))
    assert np.array_equal(g, oocc)
    sc.close()
