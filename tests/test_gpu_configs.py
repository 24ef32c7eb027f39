"""Every BASELINE.json config the device path serves, at its full size,
against the oracle (the timed kernel was never parity-checked at
its benchmarked size):

* configs[0] -- one wavelet.ply domain, 512x512, 1 spp film frame
  (tests/golden/scenes/wavelet1.spray): the device frame layer's image equals
  the oracle's bit for bit.
* configs[1] -- the bench step itself: spray_rt_intersect_scene_shadow_pt
  over the whole 1024x1024x8 spp frame (8,388,608 primary rays in the
  reference's 8 blocking tiles with tile-local seeds, ~2.26 M shadow rays
  queued and traced inside the launch): every hit record, every spawn flag
  and every occlusion byte equal the oracle's.
* the reference's published renders (docs/assets/img) through the device
  frame layer (tests/image_pin.py) -- bit-equal to the oracle's render and
  within the pin thresholds of the published images.
* the committed golden vectors (tests/golden/vectors_*.npz) through the C ABI.
"""
import os

import numpy as np
import pytest
import torch

import image_pin
from conftest import BENCH_CAMERA, SCENES, WAVELET1, WAVELETS64

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SHADE = np.array([0, 500, 1000, 1, 1, 1, 0.4, 0.4, 0.4, 10.0], np.float32)


@pytest.fixture(scope="module")
def spray():
    import spray_amd
    return spray_amd


def device_frame(spray, desc, cam, w, h, spp, kind, bounces, samples):
    sc = spray.Scene(desc, SCENES, cache_size=-1, device=0)
    boxes, lights = spray.engine.host_parse_scene(desc, SCENES)
    sc.rt.set_bsdfs(spray.engine.host_scene_bsdfs(desc))
    c = spray.camera_init(cam[:3], cam[3:], [0, 1, 0], 90.0, w, h)
    sh = spray.frame.make_shader(kind, bounces, samples, lights=lights)
    img, cnt = spray.frame.render_frame(sc.rt, sh, c, w, h, spp)
    torch.cuda.synchronize()
    out = img.cpu().numpy()
    sc.close()
    return out, cnt


def oracle_frame(oracle, desc, cam, w, h, spp, kind, bounces, samples):
    osc, doms, lights = oracle.load_scene(desc, SCENES)
    c = oracle.camera_init(cam[:3], cam[3:], [0, 1, 0], 90.0, w, h)
    sh = oracle.shader(kind, bounces, samples, (0.4, 0.4, 0.4), 10.0,
                       oracle.scene_lights(lights))
    bs = oracle.scene_bsdfs(doms)
    img = np.zeros(w * h * 4, np.float32)
    nrad = nsh = 0
    for t in oracle.tile_list(w, h, spp):
        a, b, _ = oracle.render_tile(osc, sh, bs, c, w, spp, t, img)
        nrad, nsh = nrad + a, nsh + b
    return img, (nrad, nsh)


def test_config0_single_domain_frame(spray, oracle):
    """configs[0]: wavelet.ply alone, 512x512 x 1 spp, PT with the scene's
    point light, the wavelet.sh camera."""
    cam = [-5.0, 10.0, 15.0, 0.0, 0.0, 0.0]
    img, cnt = device_frame(spray, WAVELET1, cam, 512, 512, 1, "pt", 1, 1)
    ref, rcnt = oracle_frame(oracle, WAVELET1, cam, 512, 512, 1, "pt", 1, 1)
    assert (ref > 0).sum() > 50000
    assert img.tobytes() == ref.tobytes()
    assert tuple(cnt) == rcnt and rcnt[0] == 512 * 512


@pytest.mark.parametrize("name", ["wavelets64", "wavelet"])
def test_device_render_matches_published(spray, oracle, name):
    desc, cam, spp, kind, bounces, samples = image_pin.SETTINGS[name]
    desc = os.path.join(SCENES, desc)
    s = image_pin.SIZE
    img, cnt = device_frame(spray, desc, cam, s, s, spp, kind, bounces, samples)
    ref, rcnt = oracle_frame(oracle, desc, cam, s, s, spp, kind, bounces, samples)
    assert img.tobytes() == ref.tobytes() and tuple(cnt) == rcnt
    corr, mask, flip = image_pin.compare(img, name)
    cmin, mmin = image_pin.THRESHOLDS[name]
    assert corr >= cmin and mask >= mmin and flip < 0.9, (corr, mask, flip)


def test_config1_full_frame_fused_launch(spray, oracle):
    """The benchmarked launch on the benchmarked frame, bit for bit."""
    sc = spray.Scene(WAVELETS64, SCENES, cache_size=-1, device=0)
    rt = sc.rt
    W = H = 1024
    spp = 8
    c = BENCH_CAMERA
    cam = spray.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    ocam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    n = W * H * spp
    per = W * 128 * spp
    rays = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    for k, y in enumerate(range(0, H, 128)):
        rt.eye_rays_ooc(cam, W, spp, (0, y, W, 128), rays[k * per * 32:(k + 1) * per * 32])
    hits = torch.empty(n * 48, dtype=torch.uint8, device="cuda")
    occ = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    sv = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.set_coherence(rt.RAYS_COHERENT)  # the bench's setting
    rt.intersect_scene_shadow_pt(rays, hits, SHADE, occ, sv, cnt)
    rt.sync()
    osc, _, _ = oracle.load_scene(WAVELETS64, SCENES)
    h_all = hits.cpu().numpy()
    o_all, v_all = occ.cpu().numpy(), sv.cpu().numpy()
    nshadow = 0
    for k, y in enumerate(range(0, H, 128)):
        org, d, _, _ = oracle.eye_rays_ooc(ocam, W, spp, (0, y, W, 128))
        r = rays[k * per * 32:(k + 1) * per * 32].cpu().numpy().view(spray.RAY_DTYPE)
        assert r["org"].tobytes() == org.tobytes() and r["dir"].tobytes() == d.tobytes()
        oh, _ = osc.intersect(org, d)
        assert h_all[k * per * 48:(k + 1) * per * 48].tobytes() == oh.tobytes(), k
        so, sd, src = oracle.spawn_shadows_pt(org, d, oh, [0, 500, 1000], [1, 1, 1],
                                              [0.4, 0.4, 0.4], 10.0)
        v = v_all[k * per:(k + 1) * per]
        assert np.array_equal(np.flatnonzero(v), src), k
        oo, _ = osc.occluded(so, sd)
        o = o_all[k * per:(k + 1) * per]
        assert np.array_equal(o[src], oo), k
        assert (o[v == 0] == 9).all()
        nshadow += len(src)
    assert int(cnt.item()) == nshadow > 2_000_000
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    sc.close()


def test_golden_vectors_on_device(spray, oracle):
    """tests/golden/vectors_*.npz (inputs + expected outputs) through the
    stream and scene entry points."""
    g = np.load(os.path.join(GOLDEN, "vectors_wavelet.npz"))
    v, f, col = oracle.load_ply(os.path.join(SCENES, "wavelet.ply"))
    rt = spray.RtContext(0)
    rt.upload_domain(0, v, f)
    r = np.zeros(len(g["org"]), spray.RTC_ISECT_DTYPE)
    r["org"], r["dir"], r["tnear"], r["tfar"] = g["org"], g["dir"], 0.001, np.inf
    r["geomID"] = r["primID"] = r["instID"] = 0xFFFFFFFF
    r2 = r.copy()
    rt.intersect1M(0, r)
    assert np.array_equal(r["primID"], g["prim"])
    assert r["tfar"].tobytes() == g["t"].tobytes()
    hit = g["prim"] != 0xFFFFFFFF
    assert r["u"][hit].tobytes() == g["u"][hit].tobytes()
    assert r["v"][hit].tobytes() == g["v"][hit].tobytes()
    rt.occluded1M(0, r2)
    assert np.array_equal(r2["geomID"] != 0xFFFFFFFF, g["occluded"].astype(bool))
    rt.close()
    g = np.load(os.path.join(GOLDEN, "vectors_wavelets64.npz"))
    sc = spray.Scene(WAVELETS64, SCENES, cache_size=-1, device=0)
    hits = sc.rt.intersect_scene(spray.make_rays(g["org"], g["dir"]))
    assert hits.view(np.uint8).reshape(-1, 48).tobytes() == g["hits"].tobytes()
    for mode in (sc.rt.RAYS_COHERENT, sc.rt.RAYS_INCOHERENT):
        sc.rt.set_coherence(mode)
        occ = sc.rt.occluded_scene(spray.make_rays(g["shadow_org"], g["shadow_dir"]))
        assert np.array_equal(occ, g["occluded"])
    sc.close()
