"""GPU parity of the in-situ (domain-sharded) path: device eye rays of a
stripe, routing masks, composite keys, and the whole protocol through the
HIP engine (spray_amd.insitu.GpuLocal) at world_size 1 and 2 (two processes
sharing the box's one GPU over "gloo"), against the whole-scene oracle."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

import insitu_helpers as H
from conftest import SCENES, WAVELETS64

pytestmark = pytest.mark.gpu


def _dev_rays(org, d):
    return H.rays_tensor(org, d).cuda()


def _full_ctx(spray, owner=None):
    from spray_amd import insitu
    rt = spray.RtContext(0)
    if owner is None:
        owner = np.zeros(64, np.int32)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, 0)
    return rt


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
    loc = insitu.GpuLocal(rt, torch.device("cuda"))
    rays = _dev_rays(org, d)
    m = loc.route(rays)
    hits, keys = loc.intersect_keyed(rays)
    torch.cuda.synchronize()
    cpu_rays = H.rays_tensor(org, d)
    assert (m.cpu() == ref.route(cpu_rays)).all()
    assert set(np.unique(m.cpu().numpy()).tolist()) >= {0, 1, 2, 3}
    rh, rk = ref.intersect_keyed(cpu_rays)
    assert (keys.cpu() == rk).all()
    assert hits.cpu().numpy().tobytes() == rh.numpy().tobytes()
    rt.close()


def test_insitu_world1_matches_whole_scene(spray, oracle):
    from spray_amd import insitu
    rt = _full_ctx(spray)
    cam = H.bench_camera(oracle)
    org, d, _, sam = oracle.eye_rays_insitu(cam, H.IMG, H.SPP, H.TILE, H.TILE)
    tr = insitu.InsituTracer(insitu.GpuLocal(rt, torch.device("cuda")), insitu.Comm())
    n = len(org)
    res = tr.trace_tile(_dev_rays(org, d), torch.from_numpy(sam).cuda(), H.SHADE)
    hit_ref, occ_ref, nsh = H.full_reference(oracle, cam, H.TILE, H.SPP)
    got = np.zeros(n, oracle.HIT_DTYPE)
    got[res["samid"].cpu().numpy()] = res["hits"].cpu().numpy().view(oracle.HIT_DTYPE).reshape(-1)
    hit = hit_ref["domain"] >= 0
    assert len(res["samid"]) == hit.sum()
    assert got[hit].tobytes() == hit_ref[hit].tobytes()
    assert res["n_shadow"] == nsh and res["n_rays"] == n
    ss = res["shadow_samid"].cpu().numpy()
    assert len(ss) == nsh and (res["shadow_occ"].cpu().numpy() == occ_ref[ss]).all()
    rt.close()


def test_insitu_over_rccl_one_rank(spray, oracle):
    """The protocol's collectives through RCCL ("nccl", world_size 1, every
    all-to-all / all-reduce issued): same result as the whole scene."""
    import torch.distributed as dist
    from spray_amd import insitu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        rt = _full_ctx(spray)
        cam = H.bench_camera(oracle)
        org, d, _, sam = oracle.eye_rays_insitu(cam, H.IMG, H.SPP, H.TILE, H.TILE)
        tr = insitu.InsituTracer(insitu.GpuLocal(rt, torch.device("cuda")),
                                 insitu.Comm(dist, always=True))
        res = tr.trace_tile(_dev_rays(org, d), torch.from_numpy(sam).cuda(), H.SHADE)
        hit_ref, occ_ref, nsh = H.full_reference(oracle, cam, H.TILE, H.SPP)
        hit = hit_ref["domain"] >= 0
        got = np.zeros(len(org), oracle.HIT_DTYPE)
        got[res["samid"].cpu().numpy()] = (res["hits"].cpu().numpy()
                                           .view(oracle.HIT_DTYPE).reshape(-1))
        assert len(res["samid"]) == hit.sum()
        assert got[hit].tobytes() == hit_ref[hit].tobytes()
        ss = res["shadow_samid"].cpu().numpy()
        assert res["n_shadow"] == nsh and (res["shadow_occ"].cpu().numpy() == occ_ref[ss]).all()
        rt.close()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_rank_main(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    import spray_amd
    from spray_amd import insitu
    from oracle import pyoracle as po
    import insitu_helpers as Hh
    from test_insitu import scene_boxes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        boxes, bound = scene_boxes()
        owner = insitu.morton_partition(boxes, bound, world)
        rt = spray_amd.RtContext(0)
        insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, rank)
        cam = Hh.bench_camera(po)
        stripe = insitu.horizontal_stripe(world, rank, Hh.TILE)
        n = stripe[2] * stripe[3] * Hh.SPP
        rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
        sam = torch.empty(n, dtype=torch.int32, device="cuda")
        rt.eye_rays_insitu(cam, Hh.IMG, Hh.SPP, Hh.TILE, stripe, rays, None, sam)
        rt.sync()
        tr = insitu.InsituTracer(insitu.GpuLocal(rt, torch.device("cuda")), insitu.Comm(dist))
        res = tr.trace_tile(rays, sam, Hh.SHADE)
        np.savez(os.path.join(out, "r%d.npz" % rank), samid=res["samid"].cpu().numpy(),
                 hits=res["hits"].cpu().numpy(),
                 shadow_samid=res["shadow_samid"].cpu().numpy(),
                 shadow_occ=res["shadow_occ"].cpu().numpy(), n_shadow=res["n_shadow"],
                 n_rays=n)
        rt.close()
    finally:
        dist.destroy_process_group()


def test_insitu_two_ranks_on_gpu(oracle):
    """Two processes, 32 domains each, exchanging rays: the HIP route /
    keyed / spawn / any-hit kernels under the real protocol."""
    world = 2
    with tempfile.TemporaryDirectory() as out:
        torch.multiprocessing.spawn(_gpu_rank_main, args=(world, _free_port(), out),
                                    nprocs=world)
        res = [np.load(os.path.join(out, "r%d.npz" % r)) for r in range(world)]
    hit_ref, occ_ref, nsh = H.full_reference(oracle, H.bench_camera(oracle), H.TILE, H.SPP)
    n = len(hit_ref)
    assert sum(int(r["n_rays"]) for r in res) == n
    got = np.zeros(n, oracle.HIT_DTYPE)
    seen = np.zeros(n, np.int32)
    for r in res:
        got[r["samid"]] = r["hits"].view(oracle.HIT_DTYPE).reshape(-1)
        seen[r["samid"]] += 1
        assert int(r["n_shadow"]) == nsh
        assert (r["shadow_occ"] == occ_ref[r["shadow_samid"]]).all()
        assert len(r["samid"]) > 100
    hit = hit_ref["domain"] >= 0
    assert (seen[hit] == 1).all() and (seen[~hit] == 0).all()
    assert got[hit].tobytes() == hit_ref[hit].tobytes()


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
    loc = insitu.GpuLocal(rt, torch.device("cuda"))
    mask = loc.route(H.rays_tensor(org, d).cuda()).cpu().numpy().view(np.uint64)
    ids, _, cnt, _ = oracle.domain_query(org, d, boxes, len(boxes))
    ref = np.zeros(len(org), np.uint64)
    for i in range(len(org)):
        for k in range(cnt[i]):
            ref[i] |= np.uint64(1) << np.uint64(ids[i, k])
    assert (mask == ref).all(), np.nonzero(mask != ref)[0][:10]
    assert (cnt >= 4).sum() > 100
    rt.close()
