"""GPU parity of the frame layer (spray_rt_shade / spray_rt_film /
spray_rt_render_tile): whole ooc-mode tiles -- eye rays, closest hit,
ooc::ShaderPt / ooc::ShaderAo shading with bounces, any hit of the shadow
rays, film -- against the CPU oracle's render_tile on the same inputs.  The
image must be bit-identical (the film adds in a fixed order, trig/pow are
rounded once from double on both sides), and so must the ray counts."""
import numpy as np
import pytest
import torch

from conftest import BENCH_CAMERA, SCENES, WAVELETS64

pytestmark = pytest.mark.gpu

IMG = 96


@pytest.fixture(scope="module")
def spray():
    import spray_amd
    return spray_amd


@pytest.fixture(scope="module")
def scene64(spray, oracle):
    sc = spray.Scene(WAVELETS64, SCENES, cache_size=-1, device=0)
    osc, doms, lights = oracle.load_scene(WAVELETS64, SCENES)
    yield sc, osc, doms, lights
    sc.close()


def camera(oracle, w=IMG, h=IMG):
    c = BENCH_CAMERA
    return oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], w, h)


def render_both(spray, oracle, scene64, kind, bounces, samples, spp, tiles, lights=None,
                bsdfs=None, w=IMG, h=IMG):
    sc, osc, doms, slights = scene64
    rows = oracle.scene_lights(slights) if lights is None else lights
    bs = oracle.scene_bsdfs(doms) if bsdfs is None else bsdfs
    cam = camera(oracle, w, h)
    sh_o = oracle.shader(kind, bounces, samples, lights=rows)
    sh_g = spray.frame.make_shader(kind, bounces, samples, lights=rows)
    sc.rt.set_bsdfs(bs)
    ref = np.zeros(w * h * 4, np.float32)
    img = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
    nrad = nsh = bad = 0
    sc.rt.frame_stats(reset=True)
    for t in tiles:
        a, b, c = oracle.render_tile(osc, sh_o, bs, cam, w, spp, t, ref)
        nrad, nsh, bad = nrad + a, nsh + b, bad + c
        sc.rt.render_tile(sh_g, cam, w, spp, t, img)
    try:
        cnt = sc.rt.frame_stats(reset=True)
    except spray.SprayRtError as e:
        assert bad and "abort" in str(e)
        cnt = None
    torch.cuda.synchronize()
    return img.cpu().numpy(), ref, cnt, (nrad, nsh, bad)


@pytest.mark.parametrize("bounces", [1, 2, 3])
def test_pt_frame_matches_oracle(spray, oracle, scene64, bounces):
    tiles = [(0, 0, IMG, IMG // 2), (0, IMG // 2, IMG, IMG // 2)]
    img, ref, cnt, (nrad, nsh, bad) = render_both(spray, oracle, scene64, "pt", bounces, 1, 2,
                                                  tiles)
    assert bad == 0
    assert (ref > 0).sum() > 1000
    assert img.tobytes() == ref.tobytes()
    assert cnt == (nrad, nsh)
    if bounces > 1:
        assert nrad > IMG * IMG * 2


def test_pt_frame_area_and_point_lights(spray, oracle, scene64):
    lights = [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0), (1, 0, 0, 0, 0.3, 0.4, 0.5),
              (0, 80.0, -20.0, 10.0, 0.5, 0.2, 0.1)]
    img, ref, cnt, (nrad, nsh, bad) = render_both(spray, oracle, scene64, "pt", 2, 3, 1,
                                                  [(8, 16, 64, 48)], lights=lights)
    assert bad == 0 and nsh > 3 * 64 * 48 * 0.2
    assert img.tobytes() == ref.tobytes()
    assert cnt == (nrad, nsh)


@pytest.mark.parametrize("bounces", [1, 2])
def test_ao_frame_matches_oracle(spray, oracle, scene64, bounces):
    img, ref, cnt, (nrad, nsh, bad) = render_both(spray, oracle, scene64, "ao", bounces, 4, 2,
                                                  [(0, 0, IMG, IMG)])
    assert bad == 0 and (ref > 0).sum() > 1000
    assert img.tobytes() == ref.tobytes()
    assert cnt == (nrad, nsh)


def test_delta_materials(spray, oracle, scene64):
    """Mirror and transmission domains bend the next rays; glass with both
    reflection and transmission is a case the reference aborts on -- the
    engine skips it, counts it and reports SPRAY_RT_ERR_UNSUPPORTED."""
    sc, osc, doms, _ = scene64
    bs = oracle.scene_bsdfs(doms)
    for k in range(0, 64, 3):
        bs[k] = (1, 0.9, 0.9, 0.9)
    for k in range(1, 64, 3):
        bs[k] = (3, 1.0, 1.33, 0.0)
    img, ref, cnt, (nrad, nsh, bad) = render_both(spray, oracle, scene64, "pt", 3, 1, 1,
                                                  [(0, 0, IMG, IMG)], bsdfs=bs)
    assert bad == 0
    assert img.tobytes() == ref.tobytes()
    assert cnt == (nrad, nsh)
    bs[47] = (2, 1.0, 1.5, 0.0)  # two domains the 96x96 view sees most of
    bs[63] = (2, 1.0, 1.5, 0.0)
    img, ref, cnt, (nrad, nsh, bad) = render_both(spray, oracle, scene64, "pt", 2, 1, 1,
                                                  [(0, 0, IMG, IMG)], bsdfs=bs)
    assert bad > 0
    assert img.tobytes() == ref.tobytes()
    sc.rt.set_bsdfs(oracle.scene_bsdfs(doms))


def test_shade_and_film_entry_points(spray, oracle, scene64):
    """The low-level pair on given hits (the stream form a custom scheduler
    drives): shadows, weights, next rays and the film equal the oracle's."""
    sc, osc, doms, slights = scene64
    cam = camera(oracle)
    spp = 2
    org, d, pix, sam = oracle.eye_rays_ooc(cam, IMG, spp, (0, 0, IMG, IMG))
    hits, _ = osc.intersect(org, d)
    rows = oracle.scene_lights(slights) + [(1, 0, 0, 0, 0.2, 0.2, 0.2)]
    bs = oracle.scene_bsdfs(doms)
    sc.rt.set_bsdfs(bs)
    for kind, bounce in (("pt", 0), ("pt", 1), ("ao", 0)):
        sh_o = oracle.shader(kind, 3, 2, lights=rows)
        sh_g = spray.frame.make_shader(kind, 3, 2, lights=rows)
        ns = oracle.shadow_slots(sh_o)
        assert spray.frame.shadow_slots(sh_g) == ns
        n = len(org)
        rng = np.random.default_rng(bounce)
        w = rng.uniform(0.1, 1.0, size=(n, 3)).astype(np.float32)
        valid = (rng.uniform(size=n) < 0.8).astype(np.uint8)
        o2, d2, w2, v2 = org.copy(), d.copy(), w.copy(), valid.copy()
        so, sd, sw, sv, bad = oracle.shade(sh_o, bs, bounce, o2, d2, hits, w2, v2, pix, sam)
        rays = torch.from_numpy(spray.make_rays(org, d).view(np.float32).reshape(-1, 8)).cuda()
        ghits = torch.from_numpy(hits.view(np.float32).reshape(-1, 12)).cuda()
        gw = torch.zeros((n, 4), dtype=torch.float32)
        gw[:, :3] = torch.from_numpy(w)
        gw = gw.cuda()
        gv = torch.from_numpy(valid).cuda()
        gpix = torch.from_numpy(pix).cuda()
        gsam = torch.from_numpy(sam).cuda()
        gsh = torch.zeros((n * ns, 8), dtype=torch.float32, device="cuda")
        gsw = torch.zeros((n * ns, 4), dtype=torch.float32, device="cuda")
        gsv = torch.full((n * ns,), 7, dtype=torch.uint8, device="cuda")
        stats = torch.zeros(4, dtype=torch.int64, device="cuda")
        sc.rt.shade(sh_g, bounce, rays, ghits, gw, gv, gpix, gsam, gsh, gsw, gsv, stats)
        torch.cuda.synchronize()
        gsv_h = gsv.cpu().numpy()
        assert (gsv_h == sv).all()
        sel = np.flatnonzero(sv)
        gsh_h = gsh.cpu().numpy()
        assert gsh_h[sel, 0:3].tobytes() == so[sel].tobytes()
        assert gsh_h[sel, 4:7].tobytes() == sd[sel].tobytes()
        assert gsw.cpu().numpy()[sel, :3].tobytes() == sw[sel].tobytes()
        assert (gv.cpu().numpy() == v2).all()
        live = np.flatnonzero(v2)
        r_h = rays.cpu().numpy()
        assert r_h[live, 0:3].tobytes() == o2[live].tobytes()
        assert r_h[live, 4:7].tobytes() == d2[live].tobytes()
        assert gw.cpu().numpy()[live, :3].tobytes() == w2[live].tobytes()
        st = stats.cpu().numpy()
        assert tuple(st) == (bad, len(sel), len(live), int(valid.sum()))
        # film with a given occlusion pattern
        occ = (rng.uniform(size=n * ns) < 0.3).astype(np.uint8)
        ref = rng.uniform(0, 0.1, size=IMG * IMG * 4).astype(np.float32)
        img = torch.from_numpy(ref.copy()).cuda()
        oracle.film(ref, pix, spp, ns, sw, sv, occ, 1.0 / spp)
        sc.rt.film(img, gpix, n, spp, ns, gsw, gsv, torch.from_numpy(occ).cuda(), 1.0 / spp)
        torch.cuda.synchronize()
        assert img.cpu().numpy().tobytes() == ref.tobytes()


def test_render_frame_ranks_partition_and_ppm(spray, oracle, scene64, tmp_path):
    """render_frame over the ooc tile schedule of 3 ranks (one process): the
    ranks' images (vertical stripes) have disjoint support, their sum equals the oracle's
    per-rank renders, and the PPM of the composite is the reference format."""
    sc, osc, doms, slights = scene64
    w = h = 64
    cam = camera(oracle, w, h)
    rows = oracle.scene_lights(slights)
    bs = oracle.scene_bsdfs(doms)
    sc.rt.set_bsdfs(bs)
    sh_g = spray.frame.make_shader("pt", 2, 1, lights=rows)
    sh_o = oracle.shader("pt", 2, 1, lights=rows)
    total = np.zeros(w * h * 4, np.float32)
    ref = np.zeros(w * h * 4, np.float32)
    for rank in range(3):
        img, cnt = spray.frame.render_frame(sc.rt, sh_g, cam, w, h, 2, nranks=3, rank=rank,
                                            max_samples_per_rank=1500)
        assert cnt[0] >= len(spray.frame.tile_list(w, h, 2, 3, rank, 1500)) > 0
        torch.cuda.synchronize()
        part = img.cpu().numpy()
        one = np.zeros_like(ref)
        for t in oracle.tile_list(w, h, 2, 3, rank, 1500, "image"):
            if t[2] * t[3]:
                oracle.render_tile(osc, sh_o, bs, cam, w, 2, t, one)
        assert part.tobytes() == one.tobytes()
        assert not ((total != 0) & (part != 0)).any()
        total += part
        ref += one
    assert (total > 0).sum() > 500
    p = tmp_path / "f.ppm"
    spray.frame.write_ppm(p, total, w, h)
    assert p.read_text().startswith("P3\n64 64\n1023\n")


@pytest.mark.parametrize("kind", ["pt", "ao"])
def test_batched_tiles_equal_per_tile(spray, oracle, scene64, kind):
    """spray_rt_render_tiles (all tiles as one device batch) gives the image
    of render_tile per tile, bit for bit, and the same ray counts."""
    sc, osc, doms, slights = scene64
    w = h = 96
    cam = camera(oracle, w, h)
    rows = oracle.scene_lights(slights)
    sc.rt.set_bsdfs(oracle.scene_bsdfs(doms))
    sh_g = spray.frame.make_shader(kind, 2, 3, lights=rows)
    tiles = [t for t in spray.frame.tile_list(w, h, 2, 1, 0, 4000) if t[2] * t[3]]
    assert len(tiles) > 3
    one = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
    sc.rt.frame_stats(reset=True)
    for t in tiles:
        sc.rt.render_tile(sh_g, cam, w, 2, t, one)
    c1 = sc.rt.frame_stats(reset=True)
    many = torch.zeros_like(one)
    sc.rt.render_tiles(sh_g, cam, w, 2, tiles, many)
    c2 = sc.rt.frame_stats(reset=True)
    torch.cuda.synchronize()
    assert c1 == c2 and c1[0] > 0
    a, b = one.cpu().numpy(), many.cpu().numpy()
    assert (a > 0).sum() > 1000 and a.tobytes() == b.tobytes()


def test_fused_frame_cull_matches_whole_tiles(spray, oracle, scene64, monkeypatch):
    """The fused frame launches only the eye rays of pixels some domain box's
    footprint covers (the others counted as misses): image bits and ray
    counts equal to the frame that launches the whole tiles
    (SPRAY_FRAME_CULL=0), for a batch of tiles and for a camera that sees
    no box at all."""
    sc, osc, doms, slights = scene64
    w, h, spp = 96, 80, 4
    rows = oracle.scene_lights(slights)
    sc.rt.set_bsdfs(oracle.scene_bsdfs(doms))
    sh = spray.frame.make_shader("pt", 1, 1, lights=rows)
    c = BENCH_CAMERA
    away = [2 * p - q for p, q in zip(c["pos"], c["lookat"])]
    for cam in (camera(oracle, w, h), oracle.camera_init(c["pos"], away, c["up"], 60.0, w, h)):
        tiles = [t for t in spray.frame.tile_list(w, h, spp, 1, 0, 5000) if t[2] * t[3]]
        out = []
        for cull in ("1", "0"):
            monkeypatch.setenv("SPRAY_FRAME_CULL", cull)
            img = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
            sc.rt.frame_stats(reset=True)
            sc.rt.render_tiles(sh, cam, w, spp, tiles, img)
            cnt = sc.rt.frame_stats(reset=True)
            torch.cuda.synchronize()
            out.append((img.cpu().numpy(), cnt))
        assert out[0][1] == out[1][1] and out[0][1][0] == w * h * spp
        assert out[0][0].tobytes() == out[1][0].tobytes()
    assert out[0][1][1] == 0 and not out[0][0].any()  # the camera facing away
