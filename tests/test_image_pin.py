"""The oracle pinned to the reference's own output: its film
renders of the two documented examples match the published images
(tests/image_pin.py).  The GPU counterpart,
tests/test_gpu_configs.py::test_device_render_matches_published, renders the
same frames on the device and checks them against the same images."""
import numpy as np
import pytest

import image_pin
from conftest import SCENES


def render_oracle(oracle, name):
    desc, cam, spp, kind, bounces, samples = image_pin.SETTINGS[name]
    sc, doms, lights = oracle.load_scene(SCENES + "/" + desc, SCENES)
    w = h = image_pin.SIZE
    c = oracle.camera_init(cam[:3], cam[3:], [0, 1, 0], 90.0, w, h)
    sh = oracle.shader(kind, bounces, samples, (0.4, 0.4, 0.4), 10.0, oracle.scene_lights(lights))
    bs = oracle.scene_bsdfs(doms)
    img = np.zeros(w * h * 4, np.float32)
    for t in oracle.tile_list(w, h, spp):
        oracle.render_tile(sc, sh, bs, c, w, spp, t, img)
    return img


@pytest.mark.parametrize("name", ["wavelets64", "wavelet"])
def test_oracle_matches_published_render(oracle, name):
    corr, mask, flip = image_pin.compare(render_oracle(oracle, name), name)
    cmin, mmin = image_pin.THRESHOLDS[name]
    assert corr >= cmin and mask >= mmin, (corr, mask)
    assert flip < 0.9, flip  # the comparison sees orientation errors
