"""Generates tests/golden/reference_images.npz from the only outputs the
reference itself holds: the film-mode renders shown in its docs.

    python tests/golden/make_image_fixtures.py   (needs /root/reference)

* docs/assets/img/wavelets64.jpg (230x230): examples/wavelets64/wavelets64.sh
  settings (512x512, 1 spp, PT, 1 bounce, --blinn 0.4 0.4 0.4 10, camera
  90.172180 84.141418 82.480225 -> 30 28.649426 30, fov 90), docs/example1.md:43.
* docs/assets/img/wavelet.jpg (256x256): examples/wavelet/wavelet.sh path
  tracing settings (512x512, 2 spp, 2 light samples, 2 bounces, camera
  -5 10 15 -> 0 0 0), docs/example2.md:87.

Only the Rec.601 luma of each image is kept (uint8, rounded) -- the expected
output the tests compare the oracle's and the engine's renders with
(tests/image_pin.py).  The script runs in the build container only; the
fixture travels with the tests.
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/docs/assets/img"


def luma(path):
    rgb = np.asarray(Image.open(path).convert("RGB"), np.float64)
    y = 0.299 * rgb[..., 0] + 0.587 * rgb[..., 1] + 0.114 * rgb[..., 2]
    return np.clip(np.rint(y), 0, 255).astype(np.uint8)


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "reference_images.npz"),
                        wavelets64=luma(os.path.join(SRC, "wavelets64.jpg")),
                        wavelet=luma(os.path.join(SRC, "wavelet.jpg")))
    print("ok")
