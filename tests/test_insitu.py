"""In-situ (domain-sharded) frames on the CPU: the partition and stripes of
the product (spray_rt_insitu_partition, spray_amd.insitu), and the protocol
restated over "gloo" (oracle/insitu_ref.py, each rank's local work done by
the oracle) with world sizes 1, 2, 3 and 8 -- configs[2] (PT, one bounce),
configs[4] (AO-16) and multi-bounce PT -- against the whole-scene oracle:
every shaded sample's winning hit and shadow bits bit-exact, the ray totals
exact, the image within float-summation-order tolerance.  The engine's own
protocol runs the same cases on the GPU (tests/test_gpu_insitu.py)."""
import os
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


def _expand_bits(v):
    v = np.uint32(v)
    with np.errstate(over="ignore"):
        v = (v * np.uint32(0x00010001)) & np.uint32(0xFF0000FF)
        v = (v * np.uint32(0x00000101)) & np.uint32(0x0F00F00F)
        v = (v * np.uint32(0x00000011)) & np.uint32(0xC30C30C3)
        v = (v * np.uint32(0x00000005)) & np.uint32(0x49249249)
    return v


def morton_code(x, y, z):
    """Morton::compute (src/render/morton.h:32-41), float32 clamping."""
    f = np.float32
    c = [_expand_bits(int(f(min(max(f(a) * f(1024.0), f(0.0)), f(1023.0))))) for a in (x, y, z)]
    with np.errstate(over="ignore"):
        return int((c[0] * np.uint32(4) + c[1] * np.uint32(2) + c[2]) & np.uint32(0xFFFFFFFF))


def partition_restated(boxes, sb, nranks, mode=0):
    """InsituPartition::partition (data_partition.h:59-155) in numpy; mode 0
    GROUP_CLOSE_DOMAINS (contiguous shares, :118-137), 1 round robin over the
    sorted codes (:139-155)."""
    f = np.float32
    scale = (f(1.0) / (sb[3:] - sb[:3])).astype(f)
    off = (f(0.0) - (sb[:3] * scale).astype(f)).astype(f)
    codes = sorted((morton_code(*(((b[:3] + b[3:]) * f(0.5)).astype(f) * scale + off).astype(f)), i)
                   for i, b in enumerate(boxes))
    owner = np.zeros(len(boxes), np.int32)
    if mode == 1:
        for k, (_, dom) in enumerate(codes):
            owner[dom] = k % nranks
        return owner
    shares, rank, s = len(boxes) // nranks, 0, 0
    for _, dom in codes:
        owner[dom] = rank
        s += 1
        if s == shares:
            s, rank = 0, (rank + 1) % nranks
    return owner


def test_morton_code_reference_values():
    assert morton_code(0, 0, 0) == 0
    assert morton_code(1, 1, 1) == (1 << 30) - 1
    assert morton_code(1.0 / 1024, 0, 0) == 4
    assert morton_code(0, 1.0 / 1024, 0) == 2
    assert morton_code(0, 0, 1.0 / 1024) == 1


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8, 64, 100])
def test_engine_partition_matches_restatement(nranks):
    boxes, bound = scene_boxes()
    rng = np.random.default_rng(nranks)
    jitter = boxes + rng.uniform(-3, 3, size=(len(boxes), 1)).astype(np.float32)
    for b in (boxes, jitter.astype(np.float32)):
        sb = np.concatenate([b[:, :3].min(0), b[:, 3:].max(0)])
        for mode in (0, 1):
            assert np.array_equal(insitu.morton_partition(b, sb, nranks, mode),
                                  partition_restated(b, sb, nranks, mode))


def test_round_robin_scatters_close_domains():
    """ROUND_ROBIN over 8 ranks: every rank holds one domain of every 2x2x2
    octant (the GROUP_CLOSE octants dealt out one per rank)."""
    boxes, bound = scene_boxes()
    owner = insitu.morton_partition(boxes, bound, 8, insitu.PARTITION_ROUND_ROBIN)
    close = insitu.morton_partition(boxes, bound, 8)
    assert np.bincount(owner, minlength=8).tolist() == [8] * 8
    for r in range(8):
        assert sorted(close[owner == r].tolist()) == list(range(8))


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


def test_partition_shares_and_wrap():
    boxes, bound = scene_boxes()
    assert np.bincount(insitu.morton_partition(boxes, bound, 3)).tolist() == [22, 21, 21]
    assert np.bincount(insitu.morton_partition(boxes, bound, 1)).tolist() == [64]
    assert insitu.morton_partition(boxes[:2], bound, 4).tolist() == [0, 0]


def test_horizontal_stripe():
    t = (0, 128, 1024, 128)
    assert insitu.horizontal_stripe(1, 0, t) == t
    assert [insitu.horizontal_stripe(3, r, t) for r in range(3)] == [
        (0, 128, 1024, 42), (0, 170, 1024, 42), (0, 212, 1024, 44)]
    t = (0, 0, 8, 2)
    assert [insitu.horizontal_stripe(4, r, t)[3] for r in range(4)] == [1, 1, 0, 0]


def _rendezvous_file():
    """A fresh rendezvous file for a gloo group: file:// init needs no TCP
    port (a probed free port can be taken by another process before the
    store binds it: EADDRINUSE)."""
    fd, p = tempfile.mkstemp(prefix="spray_rdv_")
    os.close(fd)
    os.unlink(p)
    return p


CASES = {  # name: (shader kind, bounces, samples, image size, spp)
    "pt1": ("pt", 1, 1, 96, 2),
    "ao16": ("ao", 1, 16, 48, 2),
    "pt3": ("pt", 3, 2, 64, 2),
}
LIGHTS = {"pt3": [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0), (1, 0, 0, 0, 0.3, 0.3, 0.3)]}


def _rank_main(rank, world, port, out, case, mode=0, replicated=False):
    import pickle
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from oracle import insitu_ref, pyoracle as po
    import insitu_helpers as H
    if world > 1:
        dist.init_process_group("gloo", init_method="file://" + port, rank=rank,
                                world_size=world)
    try:
        kind, bounces, samples, img, spp = CASES[case]
        boxes, bound = scene_boxes()
        owner = insitu.morton_partition(boxes, bound, world, mode)
        local = H.OracleLocal(po, owner, rank)
        c = H.BENCH_CAMERA
        cam = po.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
        block = (0, 0, img, img)
        # replicated frames: every rank holds every eye ray of the frame
        stripe = block if replicated else insitu.horizontal_stripe(world, rank, block)
        org, d, pix, sam = po.eye_rays_insitu(cam, img, spp, block, stripe)
        sh = H.insitu_shader(po, kind, bounces, samples, LIGHTS.get(case))
        bs = po.scene_bsdfs(local.domains)
        image = np.zeros(img * img * 4, np.float32)
        comm = insitu_ref.Comm(dist if world > 1 else None)
        fn = insitu_ref.trace_frame_replicated if replicated else insitu_ref.trace_frame
        recs, tot = fn(po, local, comm, sh, bs, org, d, pix, sam, spp, image)
        with open(os.path.join(out, "r%d.pkl" % rank), "wb") as fh:
            pickle.dump({"recs": recs, "tot": tot, "image": image,
                         "n": len(org) if (rank == 0 or not replicated) else 0}, fh)
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world,case,mode", [(1, "pt1", 0), (2, "pt1", 0), (3, "pt1", 0),
                                             (2, "pt3", 0), (8, "pt1", 0), (8, "ao16", 0),
                                             (8, "pt3", 0), (8, "pt1", 1), (3, "pt3", 1)])
def test_insitu_protocol_gloo(oracle, world, case, mode, replicated=False):
    import pickle
    import insitu_helpers as H
    with tempfile.TemporaryDirectory() as out:
        port = _rendezvous_file()
        if world == 1:
            _rank_main(0, 1, port, out, case, mode, replicated)
        else:
            torch.multiprocessing.spawn(_rank_main,
                                        args=(world, port, out, case, mode, replicated),
                                        nprocs=world)
        res = []
        for r in range(world):
            with open(os.path.join(out, "r%d.pkl" % r), "rb") as fh:
                res.append(pickle.load(fh))
    kind, bounces, samples, img, spp = CASES[case]
    c = H.BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], img, img)
    _, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    sh = H.insitu_shader(oracle, kind, bounces, samples, LIGHTS.get(case))
    ref, ref_img, ref_tot = H.reference_frame(oracle, sh, oracle.scene_bsdfs(doms), cam, img,
                                              img, spp, (0, 0, img, img))
    assert sum(r["n"] for r in res) == img * img * spp
    got = H.records_dict([x for r in res for x in r["recs"]])
    H.compare_records(got, ref)
    assert len(ref) > 1000
    if bounces > 1:
        assert any(k[0] > 0 for k in ref)
    for r in res:
        assert r["tot"] == ref_tot
    if world > 1:  # the shading is spread over the ranks (hidden octants shade nothing)
        assert sum(len(r["recs"]) > 50 for r in res) >= max(2, world // 2)
    total = np.sum([r["image"] for r in res], axis=0)
    assert (ref_img > 0).sum() > 500
    np.testing.assert_allclose(total, ref_img, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world,mode,case", [(1, 0, "pt1"), (2, 0, "pt1"), (3, 1, "pt1"),
                                             (8, 0, "pt1"), (8, 1, "pt1"), (1, 0, "ao16"),
                                             (2, 0, "ao16"), (3, 1, "ao16"), (8, 0, "ao16")])
def test_replicated_frame_gloo(oracle, world, mode, case):
    """The replicated-ray frame (insitu.cpp trace_replicated /
    trace_replicated_ao, restated in oracle/insitu_ref.py): every rank holds
    all eye rays, one MIN all-reduce of the keys and SUM all-reduces of the
    occlusion bytes (AO: of the winners' normals and colours too) -- the same
    shaded samples, bits and totals as the whole-scene oracle, for the
    GROUP_CLOSE and ROUND_ROBIN partitions."""
    test_insitu_protocol_gloo(oracle, world, case, mode, replicated=True)
