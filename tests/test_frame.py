"""CPU tests of the frame layer (no GPU): the product's host logic of
src/render/tile.cc (tile list), display/image.h (PPM writer) and
io/scene_loader.cc (materials) against the oracle's restatements, and the
oracle's shading pass against its own independent spawn functions."""
import os

import numpy as np
import pytest

from conftest import BENCH_CAMERA, SCENES, WAVELETS64


@pytest.fixture(scope="module")
def spray():
    from spray_amd import build
    build.build()
    import spray_amd
    return spray_amd


@pytest.mark.parametrize("w,h,spp,nranks,ms", [
    (1024, 1024, 8, 1, 1 << 20), (1024, 1024, 8, 8, 1 << 20), (512, 512, 1, 1, 1 << 20),
    (640, 480, 4, 3, 100000), (97, 61, 3, 5, 777), (33, 17, 2, 40, 1000),
    (1024, 1024, 8, 1, 8 << 20)])
@pytest.mark.parametrize("schedule", ["image", "blocking"])
def test_tile_list_matches_reference_rules(spray, oracle, w, h, spp, nranks, ms, schedule):
    for rank in range(nranks):
        got = spray.frame.tile_list(w, h, spp, nranks, rank, ms, schedule)
        ref = oracle.tile_list(w, h, spp, nranks, rank, ms, schedule)
        assert got == ref
    # the tiles of all ranks partition the image
    cover = np.zeros((h, w), np.int32)
    for rank in range(nranks):
        for x, y, tw, th in spray.frame.tile_list(w, h, spp, nranks, rank, ms, schedule):
            cover[y:y + th, x:x + tw] += 1
    assert (cover == 1).all()


def test_ooc_schedule_of_the_bench_frame(spray):
    """1024x1024x8spp, 1M samples per rank: 8 tiles of 1024x128 on one
    rank (the bench's ray layout); 8 ranks: one 128-column stripe each."""
    assert spray.frame.tile_list(1024, 1024, 8) == [(0, y, 1024, 128) for y in range(0, 1024, 128)]
    assert spray.frame.tile_list(1024, 1024, 8, 8, 3) == [(384, 0, 128, 1024)]


def test_tile_list_rejects_bad_arguments(spray):
    with pytest.raises(spray.SprayRtError):
        spray.frame.tile_list(0, 10, 1)
    with pytest.raises(spray.SprayRtError):
        spray.frame.tile_list(10, 10, 1, nranks=2, rank=2)
    with pytest.raises(spray.SprayRtError):  # more tiles per side than pixels
        spray.frame.tile_list(4, 4, 64, max_samples_per_rank=1, schedule="blocking")
    with pytest.raises(spray.SprayRtError):  # zero-height tiles
        spray.frame.tile_list(4, 4, 64, max_samples_per_rank=1)


def test_write_ppm_format(spray, tmp_path):
    w, h = 5, 3
    rng = np.random.default_rng(2)
    img = rng.uniform(-0.2, 1.3, size=(h * w * 4)).astype(np.float32)
    img[0] = np.float32(1.0 / 1023.0)
    p = tmp_path / "a.ppm"
    spray.frame.write_ppm(p, img, w, h)
    lines = p.read_text().splitlines()
    assert lines[:3] == ["P3", "%d %d" % (w, h), "1023"]
    px = img.reshape(h, w, 4)
    rows = []
    for y in range(h - 1, -1, -1):  # bottom row first
        for x in range(w):
            v = [int(np.clip(px[y, x, k] * np.float32(1023.0), 0, 1023)) for k in range(3)]
            rows.append("%d %d %d" % tuple(v))
    assert lines[3:] == rows


def test_scene_materials(spray, oracle, tmp_path):
    doms, _ = oracle.parse_spray(WAVELETS64, SCENES)
    ref = oracle.scene_bsdfs(doms)
    got = spray.engine.host_scene_bsdfs(WAVELETS64)
    assert len(got) == 64
    assert [tuple(np.float32(x) for x in g) for g in got] == \
        [tuple(np.float32(x) for x in r) for r in ref]
    # every material kind, and the reference's fatal cases
    txt = open(WAVELETS64).read().split("# domain")
    mats = ["mtl mirror 0.9 0.8 0.7", "mtl glass 1.0 1.5", "mtl transmission 1.0 1.33",
            "mtl diffuse 0.5 0.5 0.5"]
    body = txt[0]
    for k, mat in enumerate(mats):
        body += "# domain" + txt[1 + k].replace("mtl diffuse 1 1 1", mat)
    p = tmp_path / "m.spray"
    p.write_text(body)
    got = spray.engine.host_scene_bsdfs(str(p))
    doms, _ = oracle.parse_spray(str(p), SCENES)
    ref = oracle.scene_bsdfs(doms)
    assert [g[0] for g in got] == [1, 2, 3, 0]
    assert [tuple(np.float32(x) for x in g) for g in got] == \
        [tuple(np.float32(x) for x in r) for r in ref]
    bad = tmp_path / "bad.spray"
    bad.write_text(body.replace("mtl glass 1.0 1.5", "mtl plastic 1 1"))
    with pytest.raises(spray.SprayRtError):
        spray.engine.host_scene_bsdfs(str(bad))


def _small_scene(oracle):
    sc, doms, lights = oracle.load_scene(WAVELETS64, SCENES)
    cam = np.zeros(14, np.float32)
    c = BENCH_CAMERA
    oracle.lib().or_camera_init(oracle._p(np.float32(c["pos"])), oracle._p(np.float32(c["lookat"])),
                                oracle._p(np.float32(c["up"])), c["fov"], 64, 64,
                                oracle._p(cam))
    return sc, doms, lights, cam


def test_oracle_shade_agrees_with_spawn_functions(oracle):
    """bounce-0 PT shadows of one point light (Lin = 1) are the positional
    form of or_spawn_shadows_pt; AO shadows those of or_spawn_shadows_ao."""
    sc, doms, lights, cam = _small_scene(oracle)
    org, d, pix, sam = oracle.eye_rays_ooc(cam, 64, 2, (0, 0, 64, 64))
    hits, _ = sc.intersect(org, d)
    assert (hits["domain"] >= 0).sum() > 500
    L = lights[0]
    sh = oracle.shader("pt", 1, 1, lights=oracle.scene_lights(lights))
    o2, d2 = org.copy(), d.copy()
    w = np.ones((len(org), 3), np.float32)
    valid = np.ones(len(org), np.uint8)
    so, sd, sw, sv, bad = oracle.shade(sh, oracle.scene_bsdfs(doms), 0, o2, d2, hits, w,
                                       valid, pix, sam)
    assert bad == 0 and not valid.any()  # bounces = 1: no next rays
    ro, rd, src = oracle.spawn_shadows_pt(org, d, hits, L["pos"], L["rad"],
                                          [0.4, 0.4, 0.4], 10.0)
    sel = np.flatnonzero(sv)
    assert (sel == src).all()
    assert so[sel].tobytes() == ro.tobytes() and sd[sel].tobytes() == rd.tobytes()
    assert (sw[sel] > 0).any(axis=1).all()

    sh = oracle.shader("ao", 1, 3)
    o2, d2 = org.copy(), d.copy()
    valid[:] = 1
    w[:] = 1
    so, sd, sw, sv, bad = oracle.shade(sh, oracle.scene_bsdfs(doms), 0, o2, d2, hits, w,
                                       valid, pix, sam)
    ro, rd, src = oracle.spawn_shadows_ao(org, d, pix, hits, 3)
    sel = np.flatnonzero(sv)
    assert (sel // 3 == src).all()
    assert so[sel].tobytes() == ro.tobytes() and sd[sel].tobytes() == rd.tobytes()


def test_oracle_film_order_and_scale(oracle):
    img = np.zeros(4 * 4, np.float32)
    pix = np.array([1, 1, 3, 3], np.int32)  # two pixels x spp 2
    sw = np.array([[0.1, 0.2, 0.3], [1, 1, 1], [0.5, 0, 0], [0.25, 0.25, 0.25],
                   [2, 2, 2], [3, 3, 3], [0.7, 0.7, 0.7], [9, 9, 9]], np.float32)
    sv = np.array([1, 1, 1, 0, 1, 1, 1, 1], np.uint8)
    occ = np.array([0, 1, 0, 0, 0, 0, 1, 0], np.uint8)
    oracle.film(img, pix, 2, 2, sw, sv, occ, 0.5)
    px = img.reshape(4, 4)
    exp1 = np.float32(0)
    for j in (0, 2):
        exp1 = np.float32(np.float64(exp1) + 0.5 * np.float64(sw[j, 0]))
    assert px[1, 0] == exp1
    # pixel 3: slot 2 -> shadows 4, 5; slot 3 -> 6 (occluded), 7
    assert px[3, 0] == np.float32(0.5 * 2 + 0.5 * 3 + 0.5 * 9)
    assert px[0].sum() == 0 and px[2].sum() == 0


def test_oracle_pt_bounces_spawn_next_rays(oracle):
    """bounces = 3: each live slot either dies (miss, zero weight) or
    carries a next ray from its hit point along a cosine-weighted
    direction with weight Lin * kd * cos / (pi * pdf)."""
    sc, doms, lights, cam = _small_scene(oracle)
    img = np.zeros(64 * 64 * 4, np.float32)
    sh = oracle.shader("pt", 3, 1, lights=oracle.scene_lights(lights))
    nrad, nsh, bad = oracle.render_tile(sc, sh, oracle.scene_bsdfs(doms), cam, 64, 1,
                                        (0, 0, 64, 64), img)
    assert bad == 0
    assert nrad > 64 * 64 and nsh > 0
    assert np.isfinite(img).all() and (img >= 0).all() and img.max() > 0
