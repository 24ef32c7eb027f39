"""The camera frame's footprints (spray_amd/csrc/footprint.cpp) are
conservative, checked on the CPU against the oracle: every eye ray whose
domain list holds a box lies in that box's pixel rectangle, and every hit
point whose point-light shadow ray's list holds a box lies in the box's
shadow region and its pixel in that region's rectangle -- on the bench
frame (wavelets64, 1024x1024x8spp, insitu seeds).  Also the view-aligned
partition's counts and the degenerate cases (eye inside a box, a box
behind the eye).  No GPU: the footprint primitives are host code of the
engine library."""
import numpy as np
import pytest

from conftest import BENCH_CAMERA, SCENES, WAVELETS64

W = H = 1024
SPP = 8
LIGHT = np.array([0.0, 500.0, 1000.0], np.float32)
SHADE = [0.0, 500.0, 1000.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4, 10.0]


@pytest.fixture(scope="module")
def frame(oracle):
    c = BENCH_CAMERA
    cam = oracle.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], W, H)
    org, d, pix, sam = oracle.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), (0, 0, W, H))
    sc, doms, _ = oracle.load_scene(WAVELETS64, SCENES)
    boxes = np.array([dm["world_bound"] for dm in doms], np.float32)
    return {"cam": cam, "org": np.ascontiguousarray(org), "dir": np.ascontiguousarray(d),
            "pix": pix, "sc": sc, "boxes": boxes}


def test_eye_footprints_hold_every_listed_ray(oracle, frame):
    from spray_amd import insitu
    ids, _, cnt, _ = oracle.domain_query(frame["org"], frame["dir"], frame["boxes"], 16)
    x = frame["pix"] % W
    y = frame["pix"] // W
    rows = np.repeat(np.arange(len(cnt)), cnt)
    dom = ids[ids >= 0]
    assert len(dom) == cnt.sum() > 1_000_000
    area = 0
    for b in range(len(frame["boxes"])):
        kind, r = insitu.box_rect(frame["cam"], W, H, frame["boxes"][b])
        sel = rows[dom == b]
        assert kind in (1, 2)  # every wavelet domain is in view
        if kind == 1:
            inside = (x[sel] >= r[0]) & (x[sel] <= r[1]) & (y[sel] >= r[2]) & (y[sel] <= r[3])
            assert inside.all(), (b, (~inside).sum())
            area += (r[1] - r[0] + 1) * (r[3] - r[2] + 1)
    # the rectangles are tight: together not far beyond the listed pixels
    listed = len(np.unique(frame["pix"][rows]))
    assert area < 4 * listed * 8  # 64 overlapping boxes


def test_shadow_regions_hold_every_crossing_hit(oracle, frame):
    from spray_amd import insitu
    hits, _ = frame["sc"].intersect(frame["org"], frame["dir"])
    so, sd, src = oracle.spawn_shadows_pt(frame["org"], frame["dir"], hits, SHADE[0:3],
                                          SHADE[3:6], SHADE[6:9], SHADE[9])
    so = np.ascontiguousarray(so)
    ids, _, cnt, _ = oracle.domain_query(so, np.ascontiguousarray(sd), frame["boxes"], 16)
    rows = np.repeat(np.arange(len(cnt)), cnt)
    dom = ids[ids >= 0]
    assert len(so) > 2_000_000 and len(dom) > 1_000_000
    boxes = frame["boxes"]
    scene = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    pix = frame["pix"][src]
    x, y = pix % W, pix // W
    for b in range(len(boxes)):
        kind, reg = insitu.shadow_region(boxes[b], scene, LIGHT)
        assert kind == 0  # the light is outside the scene
        sel = rows[dom == b]
        p = so[sel]
        assert ((p >= reg[:3]) & (p <= reg[3:])).all(), b
        k2, r = insitu.box_rect(frame["cam"], W, H, reg)
        if k2 == 1:
            inside = (x[sel] >= r[0]) & (x[sel] <= r[1]) & (y[sel] >= r[2]) & (y[sel] <= r[3])
            assert inside.all(), (b, (~inside).sum())
    # a light inside the scene: every hit point may be shadowed by any box
    k, _ = insitu.shadow_region(boxes[0], scene, scene[:3] + 1.0)
    assert k == 1


def test_footprint_degenerate_cases(frame):
    from spray_amd import insitu
    cam = frame["cam"]
    eye = cam[0:3]
    k, r = insitu.box_rect(cam, W, H, np.concatenate([eye - 1.0, eye + 1.0]))
    assert k == 2 and list(r) == [0, W - 1, 0, H - 1]  # the eye inside the box
    back = eye + (eye - np.array(BENCH_CAMERA["lookat"], np.float32)) * 2.0
    k, _ = insitu.box_rect(cam, W, H, np.concatenate([back - 1.0, back + 1.0]))
    assert k == 0  # wholly behind the eye


@pytest.mark.parametrize("world", [2, 3, 8])
def test_view_partition_counts(frame, world):
    from spray_amd import insitu
    o = insitu.view_partition(frame["boxes"], frame["cam"], world)
    c = np.bincount(o, minlength=world)
    assert c.sum() == 64 and c.max() - c.min() <= 1
    assert np.array_equal(o, insitu.view_partition(frame["boxes"], frame["cam"], world))
