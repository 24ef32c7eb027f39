"""In-situ (domain-sharded) protocol on the CPU: partition, stripes, and the
exchange + compositing of spray_amd.insitu with world_size 2 over "gloo",
each rank's local work done by the oracle (tests/insitu_helpers.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

from conftest import SCENES, WAVELETS64
from spray_amd import insitu
from spray_amd.engine import host_parse_scene


def scene_boxes():
    boxes, _ = host_parse_scene(WAVELETS64, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    return boxes, bound


def test_morton_code_reference_values():
    # Morton::compute (src/render/morton.h:32-41)
    assert insitu.morton_code(0, 0, 0) == 0
    assert insitu.morton_code(1, 1, 1) == (1 << 30) - 1
    assert insitu.morton_code(1.0 / 1024, 0, 0) == 4
    assert insitu.morton_code(0, 1.0 / 1024, 0) == 2
    assert insitu.morton_code(0, 0, 1.0 / 1024) == 1
    assert insitu.morton_code(-3, 7, 0.5) == insitu.morton_code(0, 1, 0.5)


def test_partition_octants_of_the_grid():
    """64 domains on a 4x4x4 grid over 8 ranks: Morton order deals one 2x2x2
    octant to each rank."""
    boxes, bound = scene_boxes()
    owner = insitu.morton_partition(boxes, bound, 8)
    assert np.bincount(owner, minlength=8).tolist() == [8] * 8
    c = (boxes[:, :3] + boxes[:, 3:]) / 2
    cell = np.floor((c - bound[:3]) / ((bound[3:] - bound[:3]) / 4)).astype(int)
    octant = (cell[:, 0] // 2) * 4 + (cell[:, 1] // 2) * 2 + (cell[:, 2] // 2)
    for r in range(8):
        assert len(set(octant[owner == r])) == 1
    assert len(set(octant[owner == 0]) | set(octant[owner == 7])) == 2


def test_partition_shares_and_wrap():
    boxes, bound = scene_boxes()
    # shares = 64 // 3 = 21: the 64th domain wraps to rank 0
    assert np.bincount(insitu.morton_partition(boxes, bound, 3)).tolist() == [22, 21, 21]
    assert np.bincount(insitu.morton_partition(boxes, bound, 1)).tolist() == [64]
    # fewer domains than ranks: shares = 0, everything stays on rank 0
    assert insitu.morton_partition(boxes[:2], bound, 4).tolist() == [0, 0]


def test_horizontal_stripe():
    t = (0, 128, 1024, 128)
    assert insitu.horizontal_stripe(1, 0, t) == t
    assert [insitu.horizontal_stripe(3, r, t) for r in range(3)] == [
        (0, 128, 1024, 42), (0, 170, 1024, 42), (0, 212, 1024, 44)]
    # more ranks than rows: h = 1, the tail ranks get nothing
    t = (0, 0, 8, 2)
    assert [insitu.horizontal_stripe(4, r, t)[3] for r in range(4)] == [1, 1, 0, 0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from oracle import pyoracle as po
    import insitu_helpers as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        boxes, bound = scene_boxes()
        owner = insitu.morton_partition(boxes, bound, world)
        local = H.OracleLocal(po, owner, rank)
        cam = H.bench_camera(po)
        stripe = insitu.horizontal_stripe(world, rank, H.TILE)
        org, d, pix, sam = po.eye_rays_insitu(cam, H.IMG, H.SPP, H.TILE, stripe)
        tr = insitu.InsituTracer(local, insitu.Comm(dist))
        res = tr.trace_tile(H.rays_tensor(org, d), torch.from_numpy(sam), H.SHADE)
        np.savez(os.path.join(out, "r%d.npz" % rank), samid=res["samid"].numpy(),
                 hits=res["hits"].numpy(), shadow_samid=res["shadow_samid"].numpy(),
                 shadow_occ=res["shadow_occ"].numpy(), n_shadow=res["n_shadow"],
                 n_total=res["n_rays"], n_rays=len(org))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_insitu_protocol_gloo(oracle, world):
    """Sharded domains + ray exchange + key/occlusion compositing reproduce
    the whole-scene result bit-exactly (hits by sample id, occlusion of every
    spawned shadow ray, number of shadow rays)."""
    import insitu_helpers as H
    with tempfile.TemporaryDirectory() as out:
        port = _free_port()
        if world == 1:
            _rank_main(0, 1, port, out)
        else:
            torch.multiprocessing.spawn(_rank_main, args=(world, port, out), nprocs=world)
        res = [np.load(os.path.join(out, "r%d.npz" % r)) for r in range(world)]
    hit_ref, occ_ref, nsh_ref = H.full_reference(oracle, H.bench_camera(oracle), H.TILE, H.SPP)
    n = len(hit_ref)
    assert sum(int(r["n_rays"]) for r in res) == n
    got = np.zeros(n, oracle.HIT_DTYPE)
    seen = np.zeros(n, np.int32)
    for r in res:
        got[r["samid"]] = r["hits"].view(oracle.HIT_DTYPE).reshape(-1)
        seen[r["samid"]] += 1
    hit = hit_ref["domain"] >= 0
    assert hit.sum() > 3000 and (~hit).sum() > 3000
    if world > 1:  # the winners are spread over the ranks
        assert all(len(r["samid"]) > 100 for r in res)
    assert (seen[hit] == 1).all() and (seen[~hit] == 0).all()  # one winner per hit
    assert got[hit].tobytes() == hit_ref[hit].tobytes()
    for r in res:
        assert int(r["n_shadow"]) == nsh_ref and int(r["n_total"]) == n
        assert (r["shadow_occ"] == occ_ref[r["shadow_samid"]]).all()
        # a rank spawns shadow rays exactly for the samples it won
        assert set(r["shadow_samid"].tolist()) <= set(r["samid"].tolist())
    sh = np.concatenate([r["shadow_samid"] for r in res])
    assert len(sh) == nsh_ref and len(set(sh.tolist())) == nsh_ref
    assert 0 < occ_ref.sum() < nsh_ref
