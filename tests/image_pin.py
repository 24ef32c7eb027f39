"""Comparison of a rendered HDR frame with the reference's published render
(tests/golden/reference_images.npz, made by golden/make_image_fixtures.py).

The frame is mapped the way the reference writes it (HdrImage::writePpm,
src/display/image.h:183-204: clamp(v * 1023, 0, 1023) truncated, bottom row
first), scaled to 8 bits, resized to the published size (Lanczos), and
compared on Rec.601 luma: Pearson correlation, and agreement of the coverage
masks (luma > 8).  The published images are lossy JPEGs of an unknown
resize, so this pins orientation, camera, geometry and shading to within
those; bit-level parity is checked against the oracle elsewhere.
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# (scene file, camera pos + lookat, spp, shader kind, bounces, light samples)
SETTINGS = {
    "wavelets64": ("wavelets64.spray", [90.172180, 84.141418, 82.480225, 30.0, 28.649426, 30.0],
                   1, "pt", 1, 1),
    "wavelet": ("wavelet2.spray", [-5.0, 10.0, 15.0, 0.0, 0.0, 0.0], 2, "pt", 2, 2),
}
SIZE = 512


def reference(name):
    return np.load(os.path.join(GOLDEN, "reference_images.npz"))[name].astype(np.float64)


def _luma(rgb):
    return 0.299 * rgb[..., 0] + 0.587 * rgb[..., 1] + 0.114 * rgb[..., 2]


def compare(image_rgba, name, w=SIZE, h=SIZE):
    """image_rgba: float32 [h*w*4] in the film's layout (row y = 0 first).
    Returns (correlation, mask agreement, correlation of the vertically
    flipped render -- the discrimination check)."""
    from PIL import Image
    ref = reference(name)
    a = np.asarray(image_rgba, np.float32).reshape(h, w, 4)[..., :3]
    v = np.clip(a * np.float32(1023.0), 0.0, 1023.0).astype(np.uint32)[::-1]
    rgb8 = (v.astype(np.float64) / 1023.0 * 255.0).astype(np.uint8)
    n = ref.shape[0]
    small = np.asarray(Image.fromarray(rgb8).resize((n, n), Image.LANCZOS), np.float64)
    y = _luma(small)
    corr = float(np.corrcoef(y.ravel(), ref.ravel())[0, 1])
    flip = float(np.corrcoef(y[::-1].ravel(), ref.ravel())[0, 1])
    mask = float(((y > 8) == (ref > 8)).mean())
    return corr, mask, flip


# pass marks: measured oracle values 0.9989 / 0.990 (wavelets64) and
# 0.985 / 0.987 (wavelet, 2 spp noise on both sides)
THRESHOLDS = {"wavelets64": (0.99, 0.985), "wavelet": (0.97, 0.975)}
