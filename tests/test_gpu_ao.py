"""GPU ambient-occlusion rays (ooc::ShaderAo, 16 per hit) against the oracle:
same (source, sample) sequence, origins and directions bit for bit (both
sides round the hemisphere sample's sin / cos once from double, DESIGN.md
section 4), and any hit of the device's rays bit-identical to the oracle's,
in compaction order, through the trace-order permutation, written in trace
order (traced), and through the persistent any-hit form."""
import numpy as np
import pytest
import torch

from conftest import BENCH_CAMERA, SCENES, WAVELETS64

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ns", [16, 5, 40])
def test_ao16_spawn_and_occlusion(oracle, ns):
    import spray_amd
    c = BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], 1024, 1024)
    tile = (384, 448, 128, 32)
    org, d, pix, _ = oracle.eye_rays_ooc(cam, 1024, 2, tile)
    sc, _, _ = oracle.load_scene(WAVELETS64, SCENES)
    hits, _ = sc.intersect(org, d)
    so, sd, src = oracle.spawn_shadows_ao(org, d, pix, hits, ns)
    assert len(so) > ns * 1000

    scene = spray_amd.Scene(WAVELETS64, SCENES)
    rt = scene.rt
    n = len(org)
    rays = torch.zeros((n, 8), dtype=torch.float32)
    rays[:, 0:3] = torch.from_numpy(org)
    rays[:, 3] = 0.001
    rays[:, 4:7] = torch.from_numpy(d)
    rays[:, 7] = float("inf")
    rays = rays.cuda()
    h = torch.empty((n, 12), dtype=torch.float32, device="cuda")
    rt.intersect_scene(rays, h)
    pixid = torch.from_numpy(pix).cuda()
    out = torch.empty((n * ns, 8), dtype=torch.float32, device="cuda")
    osrc = torch.empty(n * ns, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pixid, n, ns, out, osrc, cnt)
    rt.sync()
    m = int(cnt.item())
    assert h.cpu().numpy().view(oracle.HIT_DTYPE).reshape(-1).tobytes() == hits.tobytes()
    assert m == len(so)
    assert (osrc[:m].cpu().numpy() == src).all()
    g = out[:m].cpu().numpy()
    assert g[:, 0:3].tobytes() == np.ascontiguousarray(so).tobytes()
    assert g[:, 4:7].tobytes() == np.ascontiguousarray(sd).tobytes()
    assert (g[:, 3] == np.float32(0.001)).all() and np.isinf(g[:, 7]).all()
    ref, _ = sc.occluded(np.ascontiguousarray(g[:, 0:3]), np.ascontiguousarray(g[:, 4:7]))
    # every traversal form (packet, per lane, per-wave choice) gives the same bits
    modes = (rt.RAYS_ADAPTIVE, rt.RAYS_COHERENT, rt.RAYS_INCOHERENT) if ns == 16 else ()
    for mode in modes:
        rt.set_coherence(mode)
        occ = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
        rt.occluded_scene(out[:m].contiguous(), occ)
        rt.sync()
        o = occ.cpu().numpy()
        assert (o == ref).all() and 0 < o.sum() < m

    # the sample-major trace order: same rays, a permutation of [0, m) that
    # keeps each 8-ray block's range, and the same occlusion bits
    out2 = torch.empty_like(out)
    osrc2 = torch.empty_like(osrc)
    cnt2 = torch.zeros(1, dtype=torch.int32, device="cuda")
    order = torch.full((n * ns,), -1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pixid, n, ns, out2, osrc2, cnt2, order=order)
    rt.sync()
    assert int(cnt2.item()) == m
    assert out2[:m].cpu().numpy().tobytes() == out[:m].cpu().numpy().tobytes()
    ordh = order[:m].cpu().numpy().astype(np.int64)
    assert np.array_equal(np.sort(ordh), np.arange(m))
    assert np.array_equal(src[ordh] // 8, src // 8)
    if ns <= 32:
        # blocks whose rays spawn all ns samples: (sample, ray) ascending
        first = np.searchsorted(src, src)
        rank = np.arange(m) - first
        per = np.bincount(src, minlength=n)
        full = np.array([(per[b * 8:b * 8 + 8] % ns == 0).all() for b in range(n // 8 + 1)])
        sel = full[src[ordh] // 8]
        key = (src[ordh] // 8) * 4096 + rank[ordh] * 8 + src[ordh] % 8
        k = key[sel]
        assert sel.sum() > m // 2 and (np.diff(k) > 0).all()
    for mode in (rt.RAYS_ADAPTIVE, rt.RAYS_INCOHERENT):
        rt.set_coherence(mode)
        occ = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
        rt.occluded_scene_order(out2, m, order, cnt2, occ)
        rt.sync()
        assert (occ.cpu().numpy() == ref).all()

    # traced: the same rays written in that order -- out3[k] = out[order[k]]
    out3 = torch.empty_like(out)
    osrc3 = torch.empty_like(osrc)
    cnt3 = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pixid, n, ns, out3, osrc3, cnt3, traced=True)
    rt.sync()
    assert int(cnt3.item()) == m
    assert out3[:m].cpu().numpy().tobytes() == out[:m].cpu().numpy()[ordh].tobytes()
    assert (osrc3[:m].cpu().numpy() == src[ordh]).all()
    rt.set_coherence(rt.RAYS_INCOHERENT)
    occ = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
    rt.occluded_scene_order(out3, m, None, cnt3, occ)
    rt.sync()
    assert (occ.cpu().numpy() == ref[ordh]).all()
    if ns <= 32:
        # fused: the rays generated in the any-hit lanes (never stored) -- the
        # traced order's (source, sample) pairs and occlusion bits
        fpair = torch.full((n * ns,), -1, dtype=torch.int32, device="cuda")
        fcnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        focc = torch.full((n * ns,), 9, dtype=torch.uint8, device="cuda")
        lv = torch.full((1024 * 1024 * ns, 4), float("nan"), dtype=torch.float32, device="cuda")
        rec = torch.empty((n, 16), dtype=torch.float32, device="cuda")
        rt.occluded_ao(rays, h, pixid, n, ns, fpair, lv, rec, fcnt, focc)
        rt.sync()
        assert int(fcnt.item()) == m
        fp = fpair[:m].cpu().numpy().view(np.uint32)
        fs = (fp >> 5).astype(np.int64)
        assert (fs == src[ordh]).all()
        assert (focc[:m].cpu().numpy() == ref[ordh]).all()
        sam = (fp & 31).astype(np.int64)
        # per source: its samples once each, in the order the spawn made them
        key = fs.astype(np.int64) * 64 + sam
        assert len(np.unique(key)) == m and (sam < ns).all()
        kk = np.sort(key)
        assert np.array_equal(kk // 64, src)
    if ns == 16:
        # a batch of >= 16 Mi rays capacity runs the persistent any-hit form
        # (kPersistAhRays); the device count bounds it to the m written rays
        cap = 16 << 20
        big = torch.empty((cap, 8), dtype=torch.float32, device="cuda")
        big[:m] = out3[:m]
        occb = torch.full((cap,), 9, dtype=torch.uint8, device="cuda")
        rt.occluded_scene_order(big, cap, None, cnt3, occb)
        rt.sync()
        ob = occb.cpu().numpy()
        assert (ob[:m] == ref[ordh]).all() and (ob[m:] == 9).all()
        del big, occb
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    scene.close()


def test_ao16_fused_full_frame():
    """configs[4] at its benchmarked size: the whole 1024x1024x8spp frame's
    36.6 M AO-16 rays through the fused spawn + any hit (persistent form)
    give the traced spawn + any hit's pairs and occlusion bits (the traced
    path is pinned to the oracle above)."""
    import spray_amd
    c = BENCH_CAMERA
    scene = spray_amd.Scene(WAVELETS64, SCENES)
    rt = scene.rt
    cam = spray_amd.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], 1024, 1024)
    n, ns, per = 1024 * 1024 * 8, 16, 1024 * 128 * 8
    rays = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    pix = torch.empty(n, dtype=torch.int32, device="cuda")
    for k in range(8):
        rt.eye_rays_ooc(cam, 1024, 8, (0, 128 * k, 1024, 128), rays[k * per * 32:(k + 1) * per * 32],
                        pix[k * per:(k + 1) * per])
    h = torch.empty(n * 48, dtype=torch.uint8, device="cuda")
    rt.intersect_scene(rays, h)
    cap = 40_000_000  # the frame spawns ~36.6 M AO rays; writes stay below *d_count
    out = torch.empty((cap, 8), dtype=torch.float32, device="cuda")
    osrc = torch.empty(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pix, n, ns, out, osrc, cnt, traced=True)
    rt.sync()
    m = int(cnt.item())
    assert 30_000_000 < m <= out.shape[0]
    rt.set_coherence(rt.RAYS_INCOHERENT)
    occ = torch.empty(m, dtype=torch.uint8, device="cuda")
    rt.occluded_scene_order(out, m, None, cnt, occ)
    rt.sync()
    ref_occ = occ.cpu().numpy()
    ref_src = osrc[:m].cpu().numpy()
    del out, occ
    fpair = torch.empty(n * ns, dtype=torch.int32, device="cuda")
    fcnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    focc = torch.empty(n * ns, dtype=torch.uint8, device="cuda")
    lv = torch.empty((1024 * 1024 * ns, 4), dtype=torch.float32, device="cuda")
    rec = torch.empty((n, 16), dtype=torch.float32, device="cuda")
    rt.occluded_ao(rays, h, pix, n, ns, fpair, lv, rec, fcnt, focc)
    rt.sync()
    assert int(fcnt.item()) == m
    assert np.array_equal((fpair[:m].cpu().numpy().view(np.uint32) >> 5).astype(np.int32),
                          ref_src)
    fo = focc[:m].cpu().numpy()
    assert np.array_equal(fo, ref_occ) and 0 < fo.sum() < m
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    scene.close()


def test_ao_pairs_misaligned_pixel_runs(oracle):
    """The fused pairs form over a subset of a frame's rays whose pixel runs
    do not align with the 8-lane groups (the replicated AO frame's C: rays
    dropped, a pixel's first ray a miss while its next one hits): the
    (pixel, sample) table must hold every sample any pair reads (filled with
    NaN beforehand), so pairs and occlusion equal the written-ray path's."""
    import spray_amd
    c = BENCH_CAMERA
    # the whole image at 128 x 128: silhouettes (pixels with hits and misses)
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], 128, 128)
    # pixel-major, the spp samples of a pixel adjacent (the in-situ order)
    org, d, pix, _ = oracle.eye_rays_insitu(cam, 128, 4, (0, 0, 128, 128), (0, 0, 128, 128))
    rng = np.random.default_rng(3)
    keep = np.flatnonzero(rng.random(len(org)) > 0.3)[1:]
    org, d, pix = org[keep], d[keep], pix[keep]
    scene = spray_amd.Scene(WAVELETS64, SCENES)
    rt = scene.rt
    n, ns = len(org), 16
    rays = torch.zeros((n, 8), dtype=torch.float32)
    rays[:, 0:3] = torch.from_numpy(np.ascontiguousarray(org))
    rays[:, 3] = 0.001
    rays[:, 4:7] = torch.from_numpy(np.ascontiguousarray(d))
    rays[:, 7] = float("inf")
    rays = rays.cuda()
    h = torch.empty((n, 12), dtype=torch.float32, device="cuda")
    rt.intersect_scene(rays, h)
    pixid = torch.from_numpy(np.ascontiguousarray(pix)).cuda()
    hit = h.cpu().numpy().view(oracle.HIT_DTYPE).reshape(-1)["domain"] >= 0
    # pixels whose first kept ray misses and whose next one hits
    first = np.r_[True, pix[1:] != pix[:-1]]
    assert ((~hit[:-1]) & first[:-1] & hit[1:] & (pix[1:] == pix[:-1])).sum() > 5
    out = torch.empty((n * ns, 8), dtype=torch.float32, device="cuda")
    osrc = torch.empty(n * ns, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(rays, h, pixid, n, ns, out, osrc, cnt, traced=True)
    rt.sync()
    m = int(cnt.item())
    rt.set_coherence(rt.RAYS_INCOHERENT)
    occ = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
    rt.occluded_scene_order(out, m, None, cnt, occ)
    rt.sync()
    fpair = torch.full((n * ns,), -1, dtype=torch.int32, device="cuda")
    fcnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    focc = torch.full((n * ns,), 9, dtype=torch.uint8, device="cuda")
    lv = torch.full((128 * 128 * ns, 4), float("nan"), dtype=torch.float32, device="cuda")
    rec = torch.empty((n, 16), dtype=torch.float32, device="cuda")
    rt.occluded_ao(rays, h, pixid, n, ns, fpair, lv, rec, fcnt, focc)
    rt.sync()
    assert int(fcnt.item()) == m
    fp = fpair[:m].cpu().numpy().view(np.uint32)
    assert ((fp >> 5).astype(np.int32) == osrc[:m].cpu().numpy()).all()
    # every table entry a pair reads was written
    lvh = lv.cpu().numpy().reshape(-1, 4)
    used = pix[(fp >> 5).astype(np.int64)].astype(np.int64) * ns + (fp & 31)
    assert np.isfinite(lvh[used, :3]).all()
    assert (focc[:m].cpu().numpy() == occ.cpu().numpy()).all()
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    scene.close()
