"""The camera frame's footprints (spray_amd/csrc/footprint.cpp) are
conservative, checked on the CPU against the oracle: every eye ray whose
domain list holds a box lies in that box's pixel rows (the projected hull,
per image row), and every hit point whose point-light shadow ray's list
holds a box lies in one of the box's shadow slices and its pixel in that
slice's rows -- on the bench
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
    for b in range(len(frame["boxes"])):
        kind, x0, x1 = insitu.box_rows(frame["cam"], W, H, frame["boxes"][b])
        sel = rows[dom == b]
        assert kind == 1  # every wavelet domain is in view, in front of the eye
        inside = (x[sel] >= x0[y[sel]]) & (x[sel] <= x1[y[sel]])
        assert inside.all(), (b, (~inside).sum())
        # the hull rows are tight: the box's listed pixels fill most of them
        listed = len(np.unique(frame["pix"][sel]))
        assert np.maximum(x1 - x0 + 1, 0).sum() < 1.6 * listed + 4 * H, b


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
        sl = insitu.shadow_boxes(boxes[b], scene, LIGHT)
        assert sl is not None and 0 < len(sl) <= 16  # the light is outside the scene
        sel = rows[dom == b]
        p = so[sel]
        in_box = np.zeros(len(sel), bool)
        in_rows = np.zeros(len(sel), bool)
        for q in sl:
            in_box |= ((p >= q[:3]) & (p <= q[3:])).all(1)
            kind, x0, x1 = insitu.box_rows(frame["cam"], W, H, q)
            if kind == 2:
                in_rows[:] = True
            elif kind == 1:
                in_rows |= (x[sel] >= x0[y[sel]]) & (x[sel] <= x1[y[sel]])
        assert in_box.all(), (b, (~in_box).sum())
        assert in_rows.all(), (b, (~in_rows).sum())
    # a light inside the scene: every hit point may be shadowed by any box
    assert insitu.shadow_boxes(boxes[0], scene, scene[:3] + 1.0) is None


def test_footprint_degenerate_cases(frame):
    from spray_amd import insitu
    cam = frame["cam"]
    eye = cam[0:3]
    k, x0, x1 = insitu.box_rows(cam, W, H, np.concatenate([eye - 1.0, eye + 1.0]))
    assert k == 2 and (x0 == 0).all() and (x1 == W - 1).all()  # the eye inside the box
    back = eye + (eye - np.array(BENCH_CAMERA["lookat"], np.float32)) * 2.0
    k, x0, x1 = insitu.box_rows(cam, W, H, np.concatenate([back - 1.0, back + 1.0]))
    assert k == 0 and (x0 > x1).all()  # wholly behind the eye


@pytest.mark.parametrize("world", [2, 3, 8])
def test_view_partition_counts(frame, world):
    from spray_amd import insitu
    o = insitu.view_partition(frame["boxes"], frame["cam"], world)
    c = np.bincount(o, minlength=world)
    assert c.sum() == 64 and c.max() - c.min() <= 1
    assert np.array_equal(o, insitu.view_partition(frame["boxes"], frame["cam"], world))
