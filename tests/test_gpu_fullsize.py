"""Parity of the bench's timed non-headline lines at their benchmarked size
(VERDICT r2, item 1): every result of the whole 1024x1024x8spp frame
against the oracle, not a small tile.

* configs[3] "ooc": spray_rt_ooc_intersect / _occluded over the whole frame
  at 4 slots with the default batching -- every 48-B record, every shadow
  ray and occlusion byte; the load schedule (loads per frame) asserted.
* configs[4] "ao" on one GPU: all ~36.6 M AO-16 rays of the frame -- the
  compacted spawn's rays bit for bit, their any hit, and the fused pairs
  path (rays generated in the any-hit lanes, the bench's form) -- against
  oracle.spawn_shadows_ao + occluded.
* configs[2] "insitu" at N = 1 through RCCL: the 1024x1024x8spp in-situ
  frame -- per-sample records bit-exact, totals exact, image within
  summation-order tolerance.

The oracle frame (8.4 M primary rays in the reference's 8 blocking tiles,
PT shadows) is computed once per module.  References: src/ooc/
ooc_pcontext.h:128-157, src/ooc/ooc_shader_ao.h:131-144, src/insitu/
insitu_multithread_tracer.inl:313-442.
"""
import os

import numpy as np
import pytest
import torch

from conftest import BENCH_CAMERA, SCENES, WAVELETS64

pytestmark = pytest.mark.gpu

W = H = 1024
SPP = 8
TILE_H = 128
PER = W * TILE_H * SPP
N = W * H * SPP
SHADE = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)


@pytest.fixture(scope="module")
def spray():
    import spray_amd
    return spray_amd


@pytest.fixture(scope="module")
def oframe(oracle):
    """The oracle's bench frame: per tile eye rays, hits, PT shadow spawn and
    occlusion; concatenated over the 8 tiles (source indices frame-global)."""
    c = BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    sc, _, _ = oracle.load_scene(WAVELETS64, SCENES)
    out = {"org": [], "dir": [], "pix": [], "hits": [], "so": [], "sd": [], "src": [], "occ": []}
    for k, y in enumerate(range(0, H, TILE_H)):
        org, d, pix, _ = oracle.eye_rays_ooc(cam, W, SPP, (0, y, W, TILE_H))
        hits, _ = sc.intersect(org, d)
        so, sd, src = oracle.spawn_shadows_pt(org, d, hits, SHADE[0:3], SHADE[3:6], SHADE[6:9],
                                              SHADE[9])
        occ, _ = sc.occluded(so, sd)
        for key, v in (("org", org), ("dir", d), ("pix", pix), ("hits", hits), ("so", so),
                       ("sd", sd), ("src", src.astype(np.int64) + k * PER), ("occ", occ)):
            out[key].append(v)
    out = {k: np.concatenate(v) for k, v in out.items()}
    out["scene"] = sc
    assert len(out["hits"]) == N and len(out["src"]) > 2_000_000
    return out


def device_rays(spray, rt):
    c = BENCH_CAMERA
    cam = spray.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    rays = torch.empty(N * 32, dtype=torch.uint8, device="cuda")
    pix = torch.empty(N, dtype=torch.int32, device="cuda")
    for k, y in enumerate(range(0, H, TILE_H)):
        rt.eye_rays_ooc(cam, W, SPP, (0, y, W, TILE_H), rays[k * PER * 32:(k + 1) * PER * 32],
                        pix[k * PER:(k + 1) * PER])
    return rays, pix


def test_ooc_full_frame_4_slots(spray, oracle, oframe):
    """configs[3] exactly as bench.py's "ooc" line runs it: closest hit with
    the domains streamed through a 4-slot LRU, compacted PT spawn, any hit of
    the shadow rays -- the whole frame, bit for bit against the oracle."""
    rt, oc = spray.ooc_scene(WAVELETS64, SCENES, 4)
    rt.set_stream(torch.cuda.current_stream())  # as bench.py: counts read through torch
    rays, _ = device_rays(spray, rt)
    hits = torch.empty(N * 48, dtype=torch.uint8, device="cuda")
    shadow = torch.empty(N * 32, dtype=torch.uint8, device="cuda")
    src = torch.empty(N, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    occ = torch.full((N,), 9, dtype=torch.uint8, device="cuda")
    frames = []
    for _ in range(2):  # the second frame starts from the first's cache state (the bench's)
        s0 = oc.stats()
        oc.intersect(rays, hits)
        rt.spawn_shadows_pt(rays, hits, N, SHADE, shadow, src, cnt)
        ns = int(cnt.item())
        oc.occluded(shadow[:ns * 32], None, occ[:ns])
        rt.sync()
        s1 = oc.stats()
        frames.append({k: s1[k] - s0[k] for k in s1})
        assert hits.cpu().numpy().tobytes() == oframe["hits"].tobytes()
        assert ns == len(oframe["src"])
        assert np.array_equal(src[:ns].cpu().numpy().astype(np.int64), oframe["src"])
        s = shadow[:ns * 32].cpu().numpy().view(np.float32).reshape(-1, 8)
        assert s[:, 0:3].tobytes() == np.ascontiguousarray(oframe["so"]).tobytes()
        assert s[:, 4:7].tobytes() == np.ascontiguousarray(oframe["sd"]).tobytes()
        assert np.array_equal(occ[:ns].cpu().numpy(), oframe["occ"])
        assert (occ[ns:].cpu().numpy() == 9).all()
    # the load schedule: every domain with live (ray, domain) pairs is loaded
    # (64 - 4 at least), each pass streaming through the 4 slots; the bench
    # line's 65 loads per frame
    for f in frames:
        assert 60 <= f["loads"] <= 70, f
        assert f["drains"] > 0 and f["bytes"] > 0
    oc.close()
    rt.close()


def test_ao16_full_frame_vs_oracle(spray, oracle, oframe):
    """configs[4] on one GPU: the frame's ~36.6 M AO-16 rays.  The compacted
    spawn equals oracle.spawn_shadows_ao ray for ray (same (source, sample)
    order), its any hit (persistent per-lane form) equals the oracle's, and
    the bench's fused path -- (source, sample) pairs, rays generated in the
    any-hit lanes, sample-major trace order -- has the same sources and the
    same occlusion bits once sorted back to (source, sample) order."""
    ns = 16
    sc = oframe["scene"]
    scene = spray.Scene(WAVELETS64, SCENES)
    rt = scene.rt
    rays, pix = device_rays(spray, rt)
    h = torch.empty(N * 48, dtype=torch.uint8, device="cuda")
    rt.set_coherence(rt.RAYS_COHERENT)
    rt.intersect_scene(rays, h)
    rt.sync()
    assert h.cpu().numpy().tobytes() == oframe["hits"].tobytes()
    # oracle AO rays per tile (frame-global sources)
    o_src, o_occ, o_org, o_dir = [], [], [], []
    for k in range(8):
        sl = slice(k * PER, (k + 1) * PER)
        so, sd, src = oracle.spawn_shadows_ao(oframe["org"][sl], oframe["dir"][sl],
                                              oframe["pix"][sl], oframe["hits"][sl], ns)
        oo, _ = sc.occluded(so, sd)
        o_src.append(src.astype(np.int64) + k * PER)
        o_occ.append(oo)
        o_org.append(so)
        o_dir.append(sd)
    o_src = np.concatenate(o_src)
    o_occ = np.concatenate(o_occ)
    m = len(o_src)
    assert 30_000_000 < m < 40_000_000 and 0 < o_occ.sum() < m

    # the compacted spawn: rays in (source, sample) order, as the oracle's
    cap = 40_000_000
    out = torch.empty((cap, 8), dtype=torch.float32, device="cuda")
    osrc = torch.empty(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pix, N, ns, out, osrc, cnt)
    rt.sync()
    assert int(cnt.item()) == m
    assert np.array_equal(osrc[:m].cpu().numpy().astype(np.int64), o_src)
    for k, ref in ((slice(0, 3), o_org), (slice(4, 7), o_dir)):
        got = out[:m, k].cpu().numpy()
        assert got.tobytes() == np.ascontiguousarray(np.concatenate(ref)).tobytes()
    del o_org, o_dir
    rt.set_coherence(rt.RAYS_INCOHERENT)  # the persistent per-lane any hit (>= 16 Mi rays)
    occ = torch.full((cap,), 9, dtype=torch.uint8, device="cuda")
    rt.occluded_scene_order(out, cap, None, cnt, occ)
    rt.sync()
    assert np.array_equal(occ[:m].cpu().numpy(), o_occ)
    del out, occ

    # the bench's fused path
    fpair = torch.empty(N * ns, dtype=torch.int32, device="cuda")
    fcnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    focc = torch.full((N * ns,), 9, dtype=torch.uint8, device="cuda")
    lv = torch.empty((W * H * ns, 4), dtype=torch.float32, device="cuda")
    rec = torch.empty((N, 16), dtype=torch.float32, device="cuda")
    rt.occluded_ao(rays, h, pix, N, ns, fpair, lv, rec, fcnt, focc)
    rt.sync()
    assert int(fcnt.item()) == m
    fp = fpair[:m].cpu().numpy().view(np.uint32).astype(np.int64)
    key = (fp >> 5) * 32 + (fp & 31)
    o = np.argsort(key, kind="stable")
    assert len(np.unique(key)) == m
    assert np.array_equal(fp[o] >> 5, o_src)
    assert np.array_equal(focc[:m].cpu().numpy()[o], o_occ)
    assert (focc[m:m + 4096].cpu().numpy() == 9).all()
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    scene.close()


def _oracle_insitu_frame(oracle, shader_rows, kind="pt", samples=1):
    """The whole-scene oracle of the in-situ frame (one blocking tile = the
    frame, (pixid, sample) seeds), one PT bounce (or AO with `samples` rays
    per hit), vectorised: per sample its hit, shadow-slot bits; the image;
    (radiance, shadow) totals."""
    c = BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    org, d, pix, sam = oracle.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), (0, 0, W, H))
    sc, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    sh = oracle.shader(kind, 1, samples, (0.4, 0.4, 0.4), 10.0, shader_rows)
    bs = oracle.scene_bsdfs(doms)
    n = len(org)
    hits, _ = sc.intersect(org, d)
    ns = oracle.shadow_slots(sh)
    org = np.ascontiguousarray(org)
    d = np.ascontiguousarray(d)
    w = np.ones((n, 3), np.float32)
    valid = np.ones(n, np.uint8)
    so, sd, sw, sv, bad = oracle.shade(sh, bs, 0, org, d, hits, w, valid, pix, sam)
    occ = np.zeros(n * ns, np.uint8)
    sel = np.flatnonzero(sv)
    occ[sel], _ = sc.occluded(np.ascontiguousarray(so[sel]), np.ascontiguousarray(sd[sel]))
    del so, sd
    image = np.zeros(W * H * 4, np.float32)
    oracle.film(image, pix, SPP, ns, sw, sv, occ, 1.0 / SPP)
    del sw
    vb = np.zeros(n, np.uint64)
    ob = np.zeros(n, np.uint64)
    svm, ocm = sv.reshape(n, ns), (sv & occ).reshape(n, ns)
    for k in range(ns):  # slot k = bit k, one column at a time (ns up to 16 here)
        vb |= svm[:, k].astype(np.uint64) << np.uint64(k)
        ob |= ocm[:, k].astype(np.uint64) << np.uint64(k)
    shaded = hits["domain"] >= 0
    order = np.argsort(sam[shaded], kind="stable")
    return {"samid": sam[shaded][order], "hits": hits[shaded][order], "svalid": vb[shaded][order],
            "occluded": ob[shaded][order], "image": image, "totals": (n, len(sel)), "bad": bad}


def test_insitu_full_frame_rccl_one_rank(spray, oracle):
    """bench.py's "insitu" line: the 1024x1024x8spp frame through the
    engine's in-situ tracer over a one-rank RCCL communicator -- every shaded
    sample's record bit-exact, the totals exact, the image within summation
    order (the film adds with hardware fp32 atomics)."""
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    boxes, lights = host_parse_scene(WAVELETS64, SCENES)  # lights: (type, pos, radiance) rows
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    owner = insitu.morton_partition(boxes, bound, 1)
    rt = spray.RtContext(0)
    insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, 0)
    rt.set_bsdfs(host_scene_bsdfs(WAVELETS64))
    rt.set_stream(torch.cuda.current_stream())
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    c = BENCH_CAMERA
    cam = spray.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    rays = torch.empty((N, 8), dtype=torch.float32, device="cuda")
    pix = torch.empty(N, dtype=torch.int32, device="cuda")
    sam = torch.empty(N, dtype=torch.int32, device="cuda")
    rt.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), (0, 0, W, H), rays, pix, sam)
    sh = spray.frame.make_shader("pt", 1, 1, ks=SHADE[6:9], shininess=SHADE[9], lights=lights)
    image = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    recs = insitu.InsituRecords(N + 16)
    tot = eng.trace(sh, rays, pix, sam, SPP, image, recs)
    eng.composite(image)
    torch.cuda.synchronize()
    got = recs.numpy()
    ref = _oracle_insitu_frame(oracle, [tuple(float(x) for x in l) for l in lights])
    assert ref["bad"] == 0
    assert tot == ref["totals"]
    assert (got["bounce"] == 0).all()
    assert np.array_equal(got["samid"], ref["samid"])
    assert got["hits"].tobytes() == ref["hits"].tobytes()
    assert np.array_equal(got["svalid"], ref["svalid"])
    assert np.array_equal(got["occluded"], ref["occluded"])
    img = image.cpu().numpy()
    assert (ref["image"] > 0).sum() > 100_000
    np.testing.assert_allclose(img, ref["image"], rtol=1e-5, atol=1e-6)
    eng.close()
    rt.close()


def _rep_rank_main(rank, world, port, out, mode, kind="pt"):
    """One rank of the full-size camera frame (spray_rt_insitu_trace_camera,
    bench.py's N > 1 form; 8 processes sharing the GPU, gloo + the engine's
    host transport; kind "pt" or "ao" = AO-16; mode: the partition, 2 =
    view-aligned): records to out/r<rank>.npz."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        boxes, lights = host_parse_scene(WAVELETS64, SCENES)
        bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
        c = BENCH_CAMERA
        cam = spray_amd.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
        owner = insitu.partition(boxes, bound, world, mode, cam)
        rt = spray_amd.RtContext(0)
        insitu.setup_rank_context(rt, WAVELETS64, SCENES, owner, rank)
        rt.set_bsdfs(host_scene_bsdfs(WAVELETS64))
        rt.set_stream(torch.cuda.current_stream())
        eng = insitu.InsituEngine(rt, world, rank, dist=dist, transport="host")
        sh = spray_amd.frame.make_shader(kind, 1, 16 if kind == "ao" else 1, ks=SHADE[6:9],
                                         shininess=SHADE[9], lights=lights)
        image = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        recs = insitu.InsituRecords(N // 2)
        eng.collective_log()  # the issue log of this frame only
        tot = eng.trace_camera(sh, cam, W, H, SPP, image, recs)
        torch.cuda.synchronize()
        g = recs.numpy()
        ops = list(insitu.InsituEngine.COLL_OPS.values())
        clog = np.array([(ops.index(op), n, s == "side") for op, n, s in eng.collective_log()],
                        np.int64).reshape(-1, 3)
        np.savez(os.path.join(out, "r%d.npz" % rank), samid=g["samid"], bounce=g["bounce"], clog=clog,
                 hits=g["hits"], svalid=g["svalid"], occluded=g["occluded"],
                 tot=np.array(tot, np.int64), image=image.cpu().numpy() if rank == 0 else
                 np.zeros(0, np.float32))
        eng.close()
        rt.close()
    finally:
        dist.destroy_process_group()


def _run_replicated(world, mode, kind):
    import tempfile
    with tempfile.TemporaryDirectory() as out:
        # file:// rendezvous in the run's own directory: no TCP port to collide
        port = os.path.join(out, "rdv")
        torch.multiprocessing.spawn(_rep_rank_main, args=(world, port, out, mode, kind),
                                    nprocs=world)
        return [dict(np.load(os.path.join(out, "r%d.npz" % r))) for r in range(world)]


def _check_replicated(parts, ref):
    # RCCL's rule: every rank enqueues the same collectives in the same order,
    # the side stream's included
    assert len(parts[0]["clog"]) >= 3
    for p in parts[1:]:
        assert np.array_equal(p["clog"], parts[0]["clog"])
    for p in parts:
        assert tuple(p["tot"]) == ref["totals"]
    assert sum(len(p["samid"]) > 10_000 for p in parts) >= 4  # the shading is spread
    sam = np.concatenate([p["samid"] for p in parts])
    order = np.argsort(sam, kind="stable")
    hits = np.concatenate([p["hits"] for p in parts])[order]
    assert np.array_equal(sam[order], ref["samid"])  # each sample shaded exactly once
    assert hits.tobytes() == ref["hits"].tobytes()
    assert np.array_equal(np.concatenate([p["svalid"] for p in parts])[order], ref["svalid"])
    assert np.array_equal(np.concatenate([p["occluded"] for p in parts])[order], ref["occluded"])
    np.testing.assert_allclose(parts[0]["image"], ref["image"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", [0, 2])
def test_replicated_full_frame_eight_ranks(spray, oracle, mode):
    """configs[2] at N = 8, the bench's camera frame at full size
    (1024x1024x8spp, the eye rays generated in the lanes, 8 domains per rank,
    GROUP_CLOSE and the view-aligned partition), 8 engine processes sharing
    the GPU over the host transport: every shaded sample's record bit-exact
    against the whole-scene oracle, shaded exactly once across the ranks,
    totals exact, rank 0's image within summation order."""
    from spray_amd.engine import host_parse_scene
    parts = _run_replicated(8, mode, "pt")
    _, lights = host_parse_scene(WAVELETS64, SCENES)
    _check_replicated(parts, _oracle_insitu_frame(
        oracle, [tuple(float(x) for x in l) for l in lights]))


@pytest.fixture(scope="module")
def ao_insitu_ref(oracle):
    from spray_amd.engine import host_parse_scene
    _, lights = host_parse_scene(WAVELETS64, SCENES)
    ref = _oracle_insitu_frame(oracle, [tuple(float(x) for x in l) for l in lights], "ao", 16)
    assert ref["bad"] == 0 and 30_000_000 < ref["totals"][1] < 40_000_000
    return ref


@pytest.mark.parametrize("mode", [0, 2])
def test_replicated_ao16_full_frame_eight_ranks(spray, oracle, ao_insitu_ref, mode):
    """configs[4] at N = 8, the bench's N > 1 "ao" line at its size: the
    camera AO-16 frame (1024x1024x8spp, ~36.6 M AO rays, 8 domains per rank,
    GROUP_CLOSE and view-aligned), 8 engine processes sharing the GPU over the
    host transport -- every shaded sample's winning record and all 16
    AO-slot spawn / occlusion bits bit-exact against the whole-scene oracle
    (ooc::ShaderAo, src/ooc/ooc_shader_ao.h:131-144), each sample shaded
    exactly once across the ranks, totals exact, rank 0's film within
    summation order."""
    _check_replicated(_run_replicated(8, mode, "ao"), ao_insitu_ref)
