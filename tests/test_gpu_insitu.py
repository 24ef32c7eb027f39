"""GPU parity of the in-situ (domain-sharded) path: device eye rays of a
stripe, routing masks, composite keys, and the engine's whole protocol
(spray_rt_insitu_trace: exchange, compositing, shading, film; configs[2]
PT, configs[4] AO-16, multi-bounce PT) -- over RCCL at one rank and over the
host transport with 2 and 8 processes sharing the box's one GPU -- against
the whole-scene oracle: every shaded sample bit-exact, totals exact, the
composited image within summation-order tolerance."""
import os
import tempfile

import numpy as np
import pytest
import torch

import insitu_helpers as H
from conftest import SCENES, WAVELETS64

pytestmark = pytest.mark.gpu


def _dev_rays(org, d):
    return H.rays_tensor(org, d).cuda()


@pytest.fixture(scope="module")
def spray():
    import spray_amd
    return spray_amd


def test_eye_rays_insitu_match_oracle(spray, oracle):
    cam = oracle.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0],
                             [0.0, 1.0, 0.0], 90.0, 1024, 1024)
    block = (0, 128, 1024, 128)
    for spp, stripe in [(8, (0, 170, 1024, 42)), (1, (0, 212, 1024, 44))]:
        org, d, pix, sam = oracle.eye_rays_insitu(cam, 1024, spp, block, stripe)
        rt = spray.RtContext(0)
        n = len(org)
        rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
        p = torch.empty(n, dtype=torch.int32, device="cuda")
        s = torch.empty(n, dtype=torch.int32, device="cuda")
        rt.eye_rays_insitu(cam, 1024, spp, block, stripe, rays, p, s)
        rt.sync()
        r = rays.cpu().numpy()
        assert r[:, 0:3].tobytes() == np.ascontiguousarray(org).tobytes()
        assert r[:, 4:7].tobytes() == np.ascontiguousarray(d).tobytes()
        assert (p.cpu().numpy() == pix).all() and (s.cpu().numpy() == sam).all()
        rt.close()


def test_route_and_keys_match_oracle(spray, oracle):
    """Rank 0 of a 2-way partition: routing masks and the keyed closest hit
    over its 32 resident domains equal the oracle's."""
    from spray_amd import insitu
    from test_insitu import scene_boxes
    boxes, bound = scene_boxes()
    owner = insitu.morton_partition(boxes, bound, 2)
    cam = H.bench_camera(oracle)
    org, d, _, _ = oracle.eye_rays_insitu(cam, H.IMG, H.SPP, H.TILE, H.TILE)
    rng = np.random.default_rng(5)
    from conftest import random_rays
    o2, d2 = random_rays(rng, 8000, np.array([30, 29, 30], np.float32), 70.0)
    org = np.concatenate([org, o2]).astype(np.float32)
    d = np.concatenate([d, d2]).astype(np.float32)
    ref = H.OracleLocal(oracle, owner, 0)
    rt = spray.RtContext(0)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, 0)
    rays = _dev_rays(org, d)
    n = len(org)
    m = torch.empty(n, dtype=torch.int64, device="cuda")
    rt.route(rays, m)
    hits = torch.empty((n, 12), dtype=torch.float32, device="cuda")
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    rt.intersect_scene_keyed(rays, hits, keys)
    torch.cuda.synchronize()
    cpu_rays = H.rays_tensor(org, d)
    assert (m.cpu() == ref.route(cpu_rays)).all()
    assert set(np.unique(m.cpu().numpy()).tolist()) >= {0, 1, 2, 3}
    rh, rk = ref.intersect_keyed(cpu_rays)
    assert (keys.cpu() == rk).all()
    assert hits.cpu().numpy().tobytes() == rh.numpy().tobytes()
    rt.close()


def _rendezvous_file():
    """A fresh rendezvous file for a gloo group: file:// init needs no TCP
    port (a probed free port can be taken by another process before the
    store binds it: EADDRINUSE)."""
    fd, p = tempfile.mkstemp(prefix="spray_rdv_")
    os.close(fd)
    os.unlink(p)
    return p


CASES = {  # name: (shader kind, bounces, samples, image size, spp)
    "pt1": ("pt", 1, 1, 128, 2),
    "ao16": ("ao", 1, 16, 64, 2),
    "pt3": ("pt", 3, 2, 96, 2),
    # footprint edge cases of the camera frame (footprint.cpp): the eye
    # inside domain 0's box (box_rows kind 2: E and U take the whole image)
    # and a point light inside the scene bound (S becomes U)
    "pt1-eyein": ("pt", 1, 1, 96, 2),
    "pt1-lightin": ("pt", 1, 1, 96, 2),
}
LIGHTS = {"pt3": [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0), (1, 0, 0, 0, 0.3, 0.3, 0.3)],
          "pt1-eyein": [(0, -300.0, 500.0, -200.0, 1.0, 1.0, 1.0)],
          "pt1-lightin": [(0, 69.0, 66.5, 69.0, 1.0, 1.0, 1.0)]}  # scene bound hi 70 67.3 70
CAMERAS = {"pt1-eyein": dict(pos=[9.0, 8.5, -9.0], lookat=[30.0, 28.649426, 30.0],
                             up=[0.0, 1.0, 0.0], fov=90.0)}  # domain 0's box: +-10


def _engine_rank(rank, world, case, transport, dist=None, one_owner=False, replicated=False,
                 mode=0, scene=None, owner=None):
    """One rank's engine frame of CASES[case]: returns (records, totals, image).
    one_owner: the last rank owns every domain (the others hold rays only).
    replicated: spray_rt_insitu_trace_frame with every eye ray on every rank
    (True) or spray_rt_insitu_trace_camera ("camera": the rays generated in
    the lanes); mode: the partition (GROUP_CLOSE / ROUND_ROBIN / VIEW);
    scene / owner: another scene file (meshes from SCENES) and its owners."""
    import spray_amd
    from spray_amd import insitu
    from oracle import pyoracle as po
    from test_insitu import scene_boxes
    kind, bounces, samples, img, spp = CASES[case]
    c = CAMERAS.get(case, H.BENCH_CAMERA)
    cam = spray_amd.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    scene = scene or WAVELETS64
    if owner is None:
        boxes, bound = scene_boxes()
        owner = insitu.partition(boxes, bound, world, mode, cam)
    owner = np.asarray(owner, np.int32)
    if one_owner:
        owner = np.full_like(owner, world - 1)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, scene, SCENES, owner, rank)
    rt.set_bsdfs(spray_amd.engine.host_scene_bsdfs(scene))
    rt.set_stream(torch.cuda.current_stream())
    block = (0, 0, img, img)
    stripe = block if replicated else insitu.horizontal_stripe(world, rank, block)
    n = stripe[2] * stripe[3] * spp
    rays = torch.empty((max(n, 1), 8), dtype=torch.float32, device="cuda")[:n]
    pix = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    sam = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    rt.eye_rays_insitu(cam, img, spp, block, stripe, rays, pix, sam)
    lights = LIGHTS.get(case, [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)])
    sh = spray_amd.frame.make_shader(kind, bounces, samples, lights=lights)
    eng = insitu.InsituEngine(rt, world, rank, dist=dist, transport=transport)
    recs = insitu.InsituRecords(img * img * spp * bounces + 16)
    image = torch.zeros(img * img * 4, dtype=torch.float32, device="cuda")
    if replicated == "camera":
        def trace(sh, rays, pix, sam, spp, image, recs=None):
            return eng.trace_camera(sh, cam, img, img, spp, image, recs)
    else:
        trace = eng.trace_frame if replicated else eng.trace
    eng.set_timing(True)
    tot = trace(sh, rays, pix, sam, spp, image, recs)
    # a second trace reuses the engine's buffers: same totals, image doubles
    tot2 = trace(sh, rays, pix, sam, spp, image)
    ph = eng.phase_times()
    assert ph and all(v >= 0 for v in ph.values()), ph
    assert tot2 == tot
    image.mul_(0.5)
    st = eng.stats()
    st["clog"] = eng.collective_log()  # both frames' collectives, in issue order
    out = (recs.numpy(), tot, image.cpu().numpy(), st)
    eng.close()
    rt.close()
    return out


def _reference(oracle, case):
    kind, bounces, samples, img, spp = CASES[case]
    c = CAMERAS.get(case, H.BENCH_CAMERA)
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    _, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    sh = H.insitu_shader(oracle, kind, bounces, samples, LIGHTS.get(case))
    return H.reference_frame(oracle, sh, oracle.scene_bsdfs(doms), cam, img, img, spp,
                             (0, 0, img, img))


def same_collectives(results):
    """Every rank issued the same collectives in the same order, on the same
    streams (RCCL's rule for one communicator)."""
    logs = [r[3]["clog"] for r in results]
    assert logs[0], "no collective logged"
    for k, lg in enumerate(logs[1:], 1):
        assert lg == logs[0], "rank %d issued %s, rank 0 %s" % (k, lg[:12], logs[0][:12])
    return logs[0]


def _check(oracle, case, results):
    if len(results) > 1:
        same_collectives(results)
    ref, ref_img, ref_tot = _reference(oracle, case)
    merged = []
    for recs, tot, _, _ in results:
        assert tot == ref_tot
        d = H.records_dict(recs)
        merged += [(b, s) + v for (b, s), v in d.items()]
    H.compare_records(H.records_dict(merged), ref)
    total = np.sum([r[2] for r in results], axis=0)
    assert (ref_img > 0).sum() > 500
    np.testing.assert_allclose(total, ref_img, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", ["pt1", "ao16", "pt3"])
def test_engine_one_rank_rccl(oracle, case):
    """The product transport (RCCL communicator of one rank): every
    all-reduce / reduce through RCCL, the self exchange through
    ncclSend / ncclRecv (SPRAY_INSITU_NCCL_SELF=1)."""
    os.environ["SPRAY_INSITU_NCCL_SELF"] = "1"
    try:
        res = _engine_rank(0, 1, case, "rccl")
    finally:
        del os.environ["SPRAY_INSITU_NCCL_SELF"]
    _check(oracle, case, [res])
    assert res[3]["collectives"] > 0 and res[3]["traces"] == 2


def test_engine_one_rank_host(oracle):
    _check(oracle, "pt1", [_engine_rank(0, 1, "pt1", "host")])


@pytest.mark.parametrize("case", ["pt1", "ao16", "pt3"])
def test_engine_one_rank_all_local(oracle, case):
    """One rank owns every domain: the frame takes the exchange-free path
    (insitu.cpp trace_local: the fused closest hit + shading + shadow any
    hit for a point-light PT bounce, the device frame layer's passes
    otherwise) -- the same records, totals and image as the protocol, and no
    exchange at all."""
    res = _engine_rank(0, 1, case, "rccl")
    _check(oracle, case, [res])
    st = res[3]
    assert st["exchanges"] == 0 and st["host_count_reads"] == 0 and st["traces"] == 2


def test_engine_one_rank_protocol_forced(oracle, monkeypatch):
    """SPRAY_INSITU_LOCAL=0 keeps the whole protocol at one rank."""
    monkeypatch.setenv("SPRAY_INSITU_LOCAL", "0")
    res = _engine_rank(0, 1, "pt1", "rccl")
    _check(oracle, "pt1", [res])
    assert res[3]["exchanges"] > 0


def _gpu_rank_main(rank, world, port, out, case, one_owner=False, replicated=False, mode=0,
                   scene=None, owner=None):
    import pickle
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        res = _engine_rank(rank, world, case, "host", dist, one_owner, replicated, mode, scene,
                           owner)
        with open(os.path.join(out, "r%d.pkl" % rank), "wb") as fh:
            pickle.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, "pt1"), (8, "pt1"), (8, "ao16"), (8, "pt3")])
def test_engine_ranks_on_gpu(oracle, world, case):
    """world processes sharing the box's one GPU, each an engine rank with
    its 64/world domains (configs[2]: 8 per rank at world 8), exchanging
    through the host transport over "gloo": every kernel and every step of
    the engine's protocol runs; RCCL itself is covered by the one-rank test
    (one GPU cannot hold an RCCL group of several ranks)."""
    import pickle
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main, args=(world, _rendezvous_file(), out, case),
                                    nprocs=world)
        res = []
        for r in range(world):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    _check(oracle, case, res)
    assert sum(len(r[0]["samid"]) > 50 for r in res) >= max(2, world // 2)
    assert all(r[3]["bytes_sent"] > 0 for r in res if len(r[0]["samid"]))


def test_engine_two_ranks_one_owner(oracle):
    """world 2, every domain on rank 1: rank 0 holds rays and no domain, rank
    1 owns everything -- both must run the same collectives (the exchange;
    no rank-local all-local shortcut at world > 1) and rank 0's
    rays must reach rank 1."""
    import pickle
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main,
                                    args=(2, _rendezvous_file(), out, "pt1", True), nprocs=2)
        res = []
        for r in range(2):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    _check(oracle, "pt1", res)
    assert len(res[0][0]["samid"]) == 0 and len(res[1][0]["samid"]) > 50
    assert res[0][3]["bytes_sent"] > 0


@pytest.mark.parametrize("world,mode,case", [(2, 0, "pt1"), (8, 0, "pt1"), (8, 1, "pt1"),
                                             (3, 1, "pt1"), (2, 0, "ao16"), (3, 1, "ao16"),
                                             (8, 0, "ao16"), (8, 1, "ao16"), (8, 1, "pt1-u64")])
def test_engine_replicated_frame_ranks(oracle, world, mode, case, monkeypatch):
    """spray_rt_insitu_trace_frame with world processes sharing the GPU over
    the host transport: every eye ray on every rank, the keys' MIN and the
    occlusion bytes' SUM all-reduced (the host transport's
    allreduce_min_u64 / allreduce_sum_u8; PT: the film's per-run sums
    reduced to rank 0; AO: the winners' normals and colours SUM-all-reduced,
    occlusion as 2- / 4-bit count fields, the film on rank 0) -- every
    shaded sample bit-exact against the whole-scene
    oracle, totals exact, the image within summation-order tolerance; both
    partitions.  PT's winner keys are split (a MIN of the t bits, then of
    the list positions at that t); "pt1-u64" keeps the 64-bit key MIN."""
    import pickle
    if case == "pt1-u64":
        monkeypatch.setenv("SPRAY_INSITU_SPLIT_KEYS", "0")
        case = "pt1"
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main,
                                    args=(world, _rendezvous_file(), out, case, False, True, mode),
                                    nprocs=world)
        res = []
        for r in range(world):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    _check(oracle, case, res)
    assert sum(len(r[0]["samid"]) > 50 for r in res) >= max(2, world // 2)
    for r in res:  # all-reduces and one host read per frame, no exchange
        assert r[3]["exchanges"] == 0 and r[3]["host_count_reads"] == 2
    # the whole film on rank 0, the other ranks' images untouched
    assert all(not r[2].any() for r in res[1:]) and res[0][2].any()


VIEW = 2  # insitu.PARTITION_VIEW


@pytest.mark.parametrize("world,mode,case", [(2, VIEW, "pt1"), (3, 0, "pt1"), (8, 0, "pt1"),
                                             (8, 1, "pt1"), (8, VIEW, "pt1"), (8, VIEW, "ao16"),
                                             (3, 1, "ao16"), (8, 0, "pt1-u64"),
                                             (3, VIEW, "pt1-eyein"), (2, 0, "pt1-eyein"),
                                             (3, VIEW, "pt1-lightin"), (2, 0, "pt1-lightin")])
def test_engine_camera_frame_ranks(oracle, world, mode, case, monkeypatch):
    """spray_rt_insitu_trace_camera with world processes sharing the GPU over
    the host transport: the eye rays generated in the lanes, each rank's
    closest hit / shadow / film passes over its domains' screen footprints
    only, the t / list-position MINs and occlusion SUM over U -- every shaded
    sample bit-exact against the whole-scene oracle, totals exact, the image
    (rank 0's) within summation order; GROUP_CLOSE, ROUND_ROBIN and the
    view-aligned partition.  No exchange and no host read."""
    import pickle
    if case == "pt1-u64":
        monkeypatch.setenv("SPRAY_INSITU_SPLIT_KEYS", "0")
        case = "pt1"
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main,
                                    args=(world, _rendezvous_file(), out, case, False, "camera", mode),
                                    nprocs=world)
        res = []
        for r in range(world):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    _check(oracle, case, res)
    assert sum(len(r[0]["samid"]) > 50 for r in res) >= max(2, world // 2)
    for r in res:
        assert r[3]["exchanges"] == 0 and r[3]["host_count_reads"] == 0
    assert all(not r[2].any() for r in res[1:]) and res[0][2].any()


TIE_DOMAINS = [  # (bound lo, bound hi, translate): wavelet.ply copies
    ((-10, -10, -10), (10, 9.324713, 10), (0, 0, 0)),
    ((-15, -15, -15), (15, 14.324713, 15), (0, 0, 0)),  # the same mesh, a wider box
    ((-10, -10, -10), (10, 9.324713, 10), (20, 0, 0)),
    ((-10, -10, -10), (10, 9.324713, 10), (20, 0, 0)),  # the same mesh, the same box
]


@pytest.mark.parametrize("split", [True, False])
def test_engine_camera_frame_cross_rank_ties(oracle, split, monkeypatch, tmp_path):
    """Exact t ties between ranks: domains 0 / 1 hold the same mesh in a
    tight and a wider box, domains 2 / 3 the same mesh in the same box, and
    each pair is split over the two ranks.  The sequential walk keeps the
    earlier list entry -- domain 1 (its wider box is entered first) and
    domain 2 (equal entry, smaller id) -- so the list positions decide the
    winner (the camera frame computes them for a rank's winners only, after
    testing the rank's boxes directly); the 64-bit key MIN as well."""
    import pickle
    lines = ["light point 0 500 1000 1 1 1", ""]
    for lo, hi, tr in TIE_DOMAINS:
        lines += ["domain", "file wavelet.ply", "mtl diffuse 1 1 1",
                  "bound %f %f %f %f %f %f" % (lo + hi), "face 5480", "vertex 2840",
                  "translate %f %f %f" % tr, ""]
    scene = str(tmp_path / "ties.spray")
    with open(scene, "w") as fh:
        fh.write("\n".join(lines))
    if not split:
        monkeypatch.setenv("SPRAY_INSITU_SPLIT_KEYS", "0")
    owner = [0, 1, 1, 0]
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main,
                                    args=(2, _rendezvous_file(), out, "pt1", False, "camera", 0,
                                          scene, owner),
                                    nprocs=2)
        res = []
        for r in range(2):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    kind, bounces, samples, img, spp = CASES["pt1"]
    c = H.BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    _, doms, _ = oracle.load_scene(scene, SCENES)
    sh = H.insitu_shader(oracle, kind, bounces, samples)
    ref, _, ref_tot = H.reference_frame(oracle, sh, oracle.scene_bsdfs(doms), cam, img, img, spp,
                                        (0, 0, img, img), desc=scene)
    same_collectives(res)
    merged = []
    for recs, tot, _, _ in res:
        assert tot == ref_tot
        d = H.records_dict(recs)
        merged += [(b, s) + v for (b, s), v in d.items()]
    got = H.records_dict(merged)
    H.compare_records(got, ref)
    # both kinds of tie occurred, and went to the earlier list entry
    dom = np.array([np.frombuffer(v[0], np.int32)[11] for v in ref.values()])
    assert (dom == 1).sum() > 100 and (dom == 2).sum() > 100
    assert not ((dom == 0) | (dom == 3)).any()


@pytest.mark.parametrize("case", ["pt1", "ao16", "pt1-u64"])
def test_engine_camera_steps_one_rank_rccl(oracle, case, monkeypatch):
    """The camera frame's replicated steps at world 1 through a one-rank RCCL
    communicator (SPRAY_INSITU_REPLICATED=1): the calls of the multi-GPU run
    -- out-of-place t-bits MIN, list-position MIN on the side stream,
    occlusion SUM, U-pixel film reduce (PT); key MIN, normals SUM, count
    fields SUM (AO).  Without it world 1 takes the all-local frame."""
    base = case.split("-")[0]
    _check(oracle, base, [_engine_rank(0, 1, base, "rccl", replicated="camera")])
    monkeypatch.setenv("SPRAY_INSITU_REPLICATED", "1")
    if case.endswith("-u64"):
        monkeypatch.setenv("SPRAY_INSITU_SPLIT_KEYS", "0")
    res = _engine_rank(0, 1, base, "rccl", replicated="camera")
    _check(oracle, base, [res])
    assert res[3]["collectives"] >= 6 and res[3]["exchanges"] == 0, res[3]


@pytest.mark.parametrize("case", ["pt1", "ao16"])
def test_engine_replicated_frame_one_rank_rccl(oracle, case):
    """World 1 through RCCL: trace_frame takes the all-local frame."""
    res = _engine_rank(0, 1, case, "rccl", replicated=True)
    _check(oracle, case, [res])


@pytest.mark.parametrize("case", ["pt1", "ao16", "pt1-u64"])
def test_engine_replicated_steps_one_rank_rccl(oracle, case, monkeypatch):
    """The replicated frame's steps at world 1 (SPRAY_INSITU_REPLICATED=1):
    every collective of the N > 1 frame -- t-bits MIN, list-position MIN on
    the side stream, occlusion SUM, run-sum reduce (PT); key MIN, published
    normals SUM, count-field SUM (AO) -- through a one-rank RCCL
    communicator, the same calls the driver's multi-GPU run makes."""
    monkeypatch.setenv("SPRAY_INSITU_REPLICATED", "1")
    if case.endswith("-u64"):
        monkeypatch.setenv("SPRAY_INSITU_SPLIT_KEYS", "0")
    base = case.split("-")[0]
    res = _engine_rank(0, 1, base, "rccl", replicated=True)
    _check(oracle, base, [res])
    assert res[3]["collectives"] >= 6 and res[3]["exchanges"] == 0, res[3]


@pytest.mark.parametrize("steps", ["local", "replicated"])
@pytest.mark.parametrize("kind", ["pt", "ao"])
def test_engine_frame_bit_reproducible(kind, steps, monkeypatch):
    """Two frames into zeroed images are bit-identical.  The film adds each
    pixel's samples in a wave-level segmented scan and commits a run with one
    atomic per wave it spans; a run of <= 8 samples spans at most two waves,
    and two addends onto zero commute exactly (a + b == b + a), so the image
    does not depend on the waves' timing.  The replicated steps (one rank
    through RCCL) sum each pixel run the same way into the compact film,
    reduce it and add one run per pixel."""
    import spray_amd
    from spray_amd import insitu
    from test_insitu import scene_boxes
    if steps == "replicated":
        monkeypatch.setenv("SPRAY_INSITU_REPLICATED", "1")
    img, spp = 256, 8
    boxes, bound = scene_boxes()
    owner = insitu.morton_partition(boxes, bound, 1, 0)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, 0)
    rt.set_bsdfs(spray_amd.engine.host_scene_bsdfs(WAVELETS64))
    rt.set_stream(torch.cuda.current_stream())
    c = H.BENCH_CAMERA
    cam = spray_amd.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    block = (0, 0, img, img)
    n = img * img * spp
    rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    pix = torch.empty(n, dtype=torch.int32, device="cuda")
    sam = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.eye_rays_insitu(cam, img, spp, block, block, rays, pix, sam)
    sh = spray_amd.frame.make_shader(kind, 1, 16 if kind == "ao" else 1,
                                     lights=[(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)])
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    out = []
    for _ in range(3):
        image = torch.zeros(img * img * 4, dtype=torch.float32, device="cuda")
        eng.trace_frame(sh, rays, pix, sam, spp, image)
        torch.cuda.synchronize()
        out.append(image.cpu().numpy().view(np.uint32))
    eng.close()
    rt.close()
    assert (out[0].view(np.float32) > 0).sum() > 1000
    for o in out[1:]:
        np.testing.assert_array_equal(o, out[0])


@pytest.mark.parametrize("kind", ["pt", "ao"])
@pytest.mark.parametrize("what", ["away", "none"])
def test_engine_replicated_steps_empty(kind, what, monkeypatch):
    """Edge cases of the replicated steps (world 1 through RCCL): a camera
    looking away from the scene (C' empty: no ray enters the scene box) and
    a frame with no rays at all -- the image stays zero, the totals count
    the radiance rays and no shadow / AO ray, and nothing faults."""
    import spray_amd
    from spray_amd import insitu
    from test_insitu import scene_boxes
    monkeypatch.setenv("SPRAY_INSITU_REPLICATED", "1")
    img, spp = 64, 2
    boxes, bound = scene_boxes()
    owner = insitu.morton_partition(boxes, bound, 1, 0)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, 0)
    rt.set_bsdfs(spray_amd.engine.host_scene_bsdfs(WAVELETS64))
    rt.set_stream(torch.cuda.current_stream())
    c = H.BENCH_CAMERA
    # the camera turned around: looking from its position away from the scene
    pos = np.array(c["pos"], np.float64)
    away = (2 * pos - np.array(c["lookat"], np.float64)).tolist()
    cam = spray_amd.camera_init(c["pos"], away, c["up"], c["fov"], img, img)
    block = (0, 0, img, img)
    n = img * img * spp if what == "away" else 0
    rays = torch.empty((max(n, 1), 8), dtype=torch.float32, device="cuda")[:n]
    pix = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    sam = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    if n:
        rt.eye_rays_insitu(cam, img, spp, block, block, rays, pix, sam)
    sh = spray_amd.frame.make_shader(kind, 1, 16 if kind == "ao" else 1,
                                     lights=[(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)])
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    image = torch.zeros(img * img * 4, dtype=torch.float32, device="cuda")
    tot = eng.trace_frame(sh, rays, pix, sam, spp, image)
    torch.cuda.synchronize()
    assert tot == (n, 0), tot
    assert float(image.abs().sum()) == 0.0
    eng.close()
    rt.close()


def test_engine_replicated_frame_unsupported_shading(oracle):
    """Several bounces are not a replicated frame: UNSUPPORTED, and nothing
    traced."""
    import spray_amd
    with pytest.raises(spray_amd.SprayRtError, match="-6|replicated"):
        _engine_rank(0, 1, "pt3", "rccl", replicated=True)


def test_transport_layout1_rejected(spray):
    """spray_rt_transport layout 2 put struct_size in front of `user`
    (include/spray_rt.h, SPRAY_RT_TRANSPORT_ABI): a caller built against
    layout 1 (`user` first) must get SPRAY_RT_ERR_ARG, not callbacks shifted
    by one slot -- its `user` pointer (or NULL) read as struct_size fails
    the range check before any callback is read."""
    import ctypes as C
    from spray_amd import insitu
    from spray_amd._native import lib

    class Layout1(C.Structure):
        _fields_ = [("user", C.c_void_p), ("alltoallv", insitu._A2A),
                    ("allreduce_u64", insitu._AR), ("reduce_f32", insitu._RED),
                    ("allreduce_min_u64", insitu._AR), ("allreduce_sum_u8", insitu._AR)]

    keep = insitu._LocalCollectives()
    rt = spray.RtContext(0)
    anchor = C.c_int(7)
    for user in (C.addressof(anchor), None, 8):
        s = Layout1(user, *keep._cbs)
        h = C.c_void_p()
        rc = lib().spray_rt_insitu_create(rt.h, 2, 0, None, C.byref(s), C.byref(h))
        assert rc == -1 and not h.value, (user, rc)
    # the current layout is accepted, a shorter version-2 struct too (the
    # callbacks past its size are NULL: replicated frames unsupported)
    for size in (C.sizeof(insitu.Transport), insitu.Transport.allreduce_min_u64.offset):
        s = insitu.Transport(size, None, *keep._cbs)
        h = C.c_void_p()
        assert lib().spray_rt_insitu_create(rt.h, 1, 0, None, C.byref(s), C.byref(h)) == 0
        assert lib().spray_rt_insitu_destroy(h.value) == 0
    rt.close()


def test_domain_mask_exact_on_box_boundaries(spray, oracle):
    """The top-level walk (fast slab on padded internal boxes, exact
    intersectAabb on the leaves) yields exactly the brute-force domain list:
    with owner[d] = d the routing mask IS the domain mask.  Rays aimed at box
    corners, edge midpoints and face centres (shared by neighbouring
    domains), from outside, from inside, and axis-parallel."""
    from spray_amd import insitu
    from test_insitu import scene_boxes
    boxes, bound = scene_boxes()
    rng = np.random.default_rng(17)
    pts = []
    for b in boxes:
        lo, hi = b[:3], b[3:]
        c = (lo + hi) / 2
        for k in range(8):  # corners
            pts.append(np.where([(k >> a) & 1 for a in range(3)], hi, lo))
        for a in range(3):  # face centres
            for v in (lo[a], hi[a]):
                p = c.copy()
                p[a] = v
                pts.append(p)
    pts = np.array(pts, np.float32)
    n = len(pts)
    org = np.concatenate([
        rng.uniform(-40, 110, size=(n, 3)),                   # outside / anywhere
        pts + rng.normal(scale=3.0, size=(n, 3)),              # near the target
        np.repeat(((bound[:3] + bound[3:]) / 2)[None], n, 0),  # from the centre
    ]).astype(np.float32)
    tgt = np.concatenate([pts, pts, pts])
    d = (tgt - org).astype(np.float32)
    nrm = np.linalg.norm(d, axis=1)
    keep = nrm > 0
    org, d = org[keep], d[keep] / nrm[keep, None]
    # axis-parallel rays grazing box faces
    m = 2000
    ax = rng.integers(0, 3, m)
    o2 = pts[rng.integers(0, n, m)].copy()
    d2 = np.zeros((m, 3), np.float32)
    d2[np.arange(m), ax] = rng.choice([-1.0, 1.0], m)
    o2[np.arange(m), ax] += -d2[np.arange(m), ax] * 150.0
    org = np.concatenate([org, o2]).astype(np.float32)
    d = np.concatenate([d, d2]).astype(np.float32)
    rt = spray.RtContext(0)
    rt.domain_bounds(boxes)
    rt.set_owners(np.arange(len(boxes), dtype=np.int32))
    mk = torch.empty(len(org), dtype=torch.int64, device="cuda")
    rt.route(H.rays_tensor(org, d).cuda(), mk)
    rt.sync()
    mask = mk.cpu().numpy().view(np.uint64)
    ids, _, cnt, _ = oracle.domain_query(org, d, boxes, len(boxes))
    ref = np.zeros(len(org), np.uint64)
    for i in range(len(org)):
        for k in range(cnt[i]):
            ref[i] |= np.uint64(1) << np.uint64(ids[i, k])
    assert (mask == ref).all(), np.nonzero(mask != ref)[0][:10]
    assert (cnt >= 4).sum() > 100
    rt.close()


# ---- image-parallel frames (spray_rt_insitu_trace_image) ----
IMG_CASES = {"pt1": ("pt", 1, 1, 128, 8, [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)]),
             "ao16": ("ao", 1, 16, 64, 4, [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)]),
             "pt3": ("pt", 3, 2, 96, 2, LIGHTS["pt3"])}


def _image_frame(rank, world, case, transport, dist=None, bands=1, how="image"):
    """One frame of IMG_CASES[case] into a zeroed image, every domain resident:
    spray_rt_insitu_trace_image (how "image") or, at one rank, the whole
    image's eye rays through spray_rt_insitu_trace (how "rays").  Returns (records, totals, image, stats)."""
    import spray_amd
    from spray_amd import insitu
    kind, bounces, samples, img, spp, lights = IMG_CASES[case]
    c = H.BENCH_CAMERA
    cam = spray_amd.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    rt = spray_amd.RtContext(0)
    nd = len(spray_amd.engine.host_parse_scene(WAVELETS64, SCENES)[0])
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, np.full(nd, rank, np.int32), rank)
    rt.set_bsdfs(spray_amd.engine.host_scene_bsdfs(WAVELETS64))
    rt.set_stream(torch.cuda.current_stream())
    sh = spray_amd.frame.make_shader(kind, bounces, samples, lights=lights)
    eng = insitu.InsituEngine(rt, world, rank, dist=dist, transport=transport)
    recs = insitu.InsituRecords(img * img * spp * bounces + 16)
    image = torch.zeros(img * img * 4, dtype=torch.float32, device="cuda")
    if how == "image":
        tot = eng.trace_image(sh, cam, img, img, spp, image, bands, recs)
    else:  # the whole image's stored eye rays through the one-rank all-local frame
        n = img * img * spp
        rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
        pix = torch.empty(n, dtype=torch.int32, device="cuda")
        sam = torch.empty(n, dtype=torch.int32, device="cuda")
        rt.eye_rays_insitu(cam, img, spp, (0, 0, img, img), (0, 0, img, img), rays, pix, sam)
        tot = eng.trace(sh, rays, pix, sam, spp, image, recs)
    torch.cuda.synchronize()
    st = eng.stats()
    st["clog"] = eng.collective_log()
    out = (recs.numpy(), tot, image.cpu().numpy(), st)
    eng.close()
    rt.close()
    return out


def _image_rank_main(rank, world, port, out, case, bands):
    import pickle
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        res = _image_frame(rank, world, case, "host", dist, bands)
        with open(os.path.join(out, "r%d.pkl" % rank), "wb") as fh:
            pickle.dump(res, fh)
    finally:
        dist.destroy_process_group()


def _image_reference(oracle, case):
    kind, bounces, samples, img, spp, lights = IMG_CASES[case]
    c = H.BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    _, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    sh = H.insitu_shader(oracle, kind, bounces, samples, lights)
    return H.reference_frame(oracle, sh, oracle.scene_bsdfs(doms), cam, img, img, spp,
                             (0, 0, img, img))


@pytest.mark.parametrize("world,bands,case", [(1, 1, "pt1"), (1, 2, "ao16"), (2, 1, "pt1"),
                                              (2, 4, "pt1"), (3, 1, "ao16"), (3, 1, "pt3"),
                                              (4, 16, "ao16"), (8, 8, "pt1"), (8, 1, "ao16")])
def test_engine_image_frame_ranks(oracle, world, bands, case):
    """The image-parallel strong split (ooc mode): world
    processes sharing the GPU over the host transport (world 1: RCCL), every
    domain resident on each, rank r tracing its row bands -- every shaded
    sample's record bit-exact against the whole-scene oracle and shaded on
    exactly one rank, totals exact, the same collectives on every rank, and
    rank 0's gathered image BIT-EQUAL to the one-rank frame's (the
    pixels are disjoint and the (pixel, sample) seeds do not see the split),
    the other ranks holding their own rows only."""
    import pickle
    if world == 1:
        res = [_image_frame(0, 1, case, "rccl", None, bands)]
    else:
        with tempfile.TemporaryDirectory() as out:
            torch.multiprocessing.spawn(_image_rank_main,
                                        args=(world, _rendezvous_file(), out, case, bands),
                                        nprocs=world)
            res = []
            for r in range(world):
                with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                    res.append(pickle.load(fh))
        log = same_collectives(res)
        assert [op for op, _, _ in log] == ["alltoallv_u8", "allreduce_sum_u64"], log
    ref, ref_img, ref_tot = _image_reference(oracle, case)
    merged = []
    for recs, tot, _, st in res:
        assert tot == ref_tot
        assert st["exchanges"] == 0 and st["host_count_reads"] == 0
        merged += [(b, s) + v for (b, s), v in H.records_dict(recs).items()]
    assert len(merged) == len({(m[0], m[1]) for m in merged})  # shaded once
    H.compare_records(H.records_dict(merged), ref)
    np.testing.assert_allclose(res[0][2], ref_img, rtol=1e-5, atol=1e-6)
    one = _image_frame(0, 1, case, "rccl", how="rays")[2]
    assert (one > 0).sum() > 500
    np.testing.assert_array_equal(res[0][2].view(np.uint32), one.view(np.uint32))
    img = IMG_CASES[case][3]
    for r in range(1, world):  # a rank's image: its own bands' rows only
        rows = np.zeros(img, bool)
        bt = world * bands
        for b in range(r, bt, world):
            rows[b * img // bt:(b + 1) * img // bt] = True
        im = res[r][2].reshape(img, img, 4)
        np.testing.assert_array_equal(im[rows].view(np.uint32),
                                      one.reshape(img, img, 4)[rows].view(np.uint32))
        assert not im[~rows].any()


@pytest.mark.parametrize("case", ["pt1", "ao16"])
def test_engine_image_frame_cull_matches_whole_bands(monkeypatch, case):
    """The image frame launches U's eye rays only (pixels outside every box's
    footprint are counted, not traced): image bits, totals and records equal
    to the frame that traces its bands whole (SPRAY_IMAGE_CULL=0)."""
    culled = _image_frame(0, 1, case, "rccl", bands=2)
    monkeypatch.setenv("SPRAY_IMAGE_CULL", "0")
    whole = _image_frame(0, 1, case, "rccl", bands=2)
    assert culled[1] == whole[1]
    np.testing.assert_array_equal(culled[2].view(np.uint32), whole[2].view(np.uint32))
    assert H.records_dict(culled[0]) == H.records_dict(whole[0])


def test_engine_image_frame_facing_away(spray):
    """A camera that sees no box: no eye ray launched, every one counted."""
    from spray_amd import insitu
    rt = spray.RtContext(0)
    nd = len(spray.engine.host_parse_scene(WAVELETS64, SCENES)[0])
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, np.zeros(nd, np.int32), 0)
    rt.set_bsdfs(spray.engine.host_scene_bsdfs(WAVELETS64))
    rt.set_stream(torch.cuda.current_stream())
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    c = H.BENCH_CAMERA
    away = [2 * p - q for p, q in zip(c["pos"], c["lookat"])]
    cam = spray.camera_init(c["pos"], away, c["up"], 60.0, 64, 48)
    sh = spray.frame.make_shader("pt", 1, 1, lights=[(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)])
    image = torch.zeros(64 * 48 * 4, dtype=torch.float32, device="cuda")
    tot = eng.trace_image(sh, cam, 64, 48, 4, image)
    torch.cuda.synchronize()
    assert tuple(tot) == (64 * 48 * 4, 0)
    assert not image.any()
    eng.close()
    rt.close()


def test_engine_image_frame_needs_every_domain(spray):
    """A rank missing a domain cannot trace an image-parallel frame."""
    from spray_amd import insitu
    from test_insitu import scene_boxes
    boxes, bound = scene_boxes()
    rt = spray.RtContext(0)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, insitu.morton_partition(boxes, bound, 2), 0)
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    c = H.BENCH_CAMERA
    cam = spray.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], 64, 64)
    sh = spray.frame.make_shader("pt", 1, 1, lights=[(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)])
    image = torch.zeros(64 * 64 * 4, dtype=torch.float32, device="cuda")
    with pytest.raises(spray.SprayRtError, match="-3|resident"):
        eng.trace_image(sh, cam, 64, 64, 2, image)
    eng.close()
    rt.close()
