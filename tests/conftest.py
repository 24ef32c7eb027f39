import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
WAVELETS64 = os.path.join(SCENES, "wavelets64.spray")
WAVELET2 = os.path.join(SCENES, "wavelet2.spray")
WAVELET1 = os.path.join(SCENES, "wavelet1.spray")
# examples/wavelets64/wavelets64.sh:142 camera, config.cc:42 fov
BENCH_CAMERA = dict(pos=[90.172180, 84.141418, 82.480225],
                    lookat=[30.0, 28.649426, 30.0], up=[0.0, 1.0, 0.0], fov=90.0)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


def random_rays(rng, n, center, radius):
    """Rays from a sphere shell around `center` aimed at random points of the
    region: a mix of hits, misses and grazing rays."""
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    org = center + u * radius
    tgt = center + rng.uniform(-1, 1, size=(n, 3)) * radius * 0.6
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return org.astype(np.float32), d.astype(np.float32)


def edge_rays(rng, verts, faces, n):
    """Rays aimed exactly at triangle vertices and edge midpoints (shared
    edges / vertices: the tie and crack cases)."""
    f = faces[rng.integers(0, len(faces), n)]
    a, b = verts[f[:, 0]], verts[f[:, 1]]
    w = rng.integers(0, 3, n)[:, None]
    tgt = np.where(w == 0, a, np.where(w == 1, (a + b) * np.float32(0.5), b))
    lo, hi = verts.min(0), verts.max(0)
    c = (lo + hi) / 2
    r = float(np.linalg.norm(hi - lo))
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    org = c + u * r
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return org.astype(np.float32), d.astype(np.float32)


def axis_rays(verts, n):
    """Axis-aligned rays (direction components exactly zero)."""
    lo, hi = verts.min(0), verts.max(0)
    g = np.linspace(0.05, 0.95, int(np.sqrt(n)) + 1)
    org, d = [], []
    for i, x in enumerate(g):
        for y in g:
            for ax in range(3):
                o = lo + (hi - lo) * np.array([x, y, x * y])[[(ax + 1) % 3, (ax + 2) % 3, ax]]
                o = o.copy()
                o[ax] = lo[ax] - 5.0
                dd = np.zeros(3)
                dd[ax] = 1.0
                org.append(o)
                d.append(dd)
    return np.array(org, np.float32), np.array(d, np.float32)
