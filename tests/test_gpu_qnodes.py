"""The per-lane any hit over the 4-wide quantized nodes (rt_device.h,
occluded_tree_q4) against the oracle on geometry that stresses its grid
(ADVICE r1): flat domains away from the origin (a ground quad at y = -1, a
wall at x = 5), a small domain at large coordinates, and rays from origins
hundreds to thousands of domain extents away aimed at triangle vertices and
edge midpoints -- the rays whose boxes sit right at a face of the child box.
Every traversal form must give the oracle's occlusion bits."""
import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu


def _quad(axis, value, lo, hi):
    o = [a for a in range(3) if a != axis]
    v = np.zeros((4, 3), np.float32)
    for k, (s, t) in enumerate([(lo, lo), (hi, lo), (hi, hi), (lo, hi)]):
        v[k, axis] = value
        v[k, o[0]], v[k, o[1]] = s, t
    return v, np.array([[0, 1, 2], [0, 2, 3]], np.uint32)


def _far_rays(rng, v, f, n, dist):
    """Rays from `dist` away aimed at vertices / edge midpoints of (v, f)."""
    fi = f[rng.integers(0, len(f), n)]
    a, b = v[fi[:, 0]], v[fi[:, 1]]
    w = rng.integers(0, 3, n)[:, None]
    tgt = np.where(w == 0, a, np.where(w == 1, (a + b) * np.float32(0.5), b)).astype(np.float64)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    org = tgt + u * dist
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return org.astype(np.float32), d.astype(np.float32)


def test_quantized_any_hit_far_origins(oracle):
    import torch
    import spray_amd
    wv, wf, _ = oracle.load_ply(SCENES + "/wavelet.ply")
    small = (wv * np.float32(0.05)).astype(np.float32)  # extent ~1
    meshes = [
        (small, wf),                                              # at the origin
        ((small + np.float32([1.0e4, 0, 0])).astype(np.float32), wf),  # large coordinates
        _quad(1, -1.0, -50.0, 50.0),                              # ground quad y = -1
        _quad(0, 5.0, -2.0, 2.0),                                 # wall x = 5
    ]
    rt = spray_amd.RtContext(0)
    osc = oracle.Scene(len(meshes))
    boxes = []
    for i, (v, f) in enumerate(meshes):
        rt.upload_domain(i, v, f)  # the flat quads used to fail here
        box = np.concatenate([v.min(0), v.max(0)]).astype(np.float32)
        boxes.append(box)
        osc.set_domain(i, v, f, np.zeros(len(v), np.uint32), np.zeros_like(v), box)
    rt.domain_bounds(np.array(boxes))
    for i in range(len(meshes)):
        rt.map_domain(i, i)
    rng = np.random.default_rng(21)
    org, d = [], []
    for i, (v, f) in enumerate(meshes):
        ext = float(np.max(v.max(0) - v.min(0)))
        for k in (370.0, 2000.0, 9000.0):
            o, dd = _far_rays(rng, v, f, 3000 if i < 2 else 600, k * ext)
            org.append(o)
            d.append(dd)
    org, d = np.concatenate(org), np.concatenate(d)
    ref, _ = osc.occluded(org, d)
    assert 0.2 < ref.mean() < 0.95
    rays = torch.from_numpy(spray_amd.make_rays(org, d).view(np.uint8)).cuda()
    for mode in (rt.RAYS_INCOHERENT, rt.RAYS_ADAPTIVE, rt.RAYS_COHERENT):
        rt.set_coherence(mode)
        occ = torch.full((len(org),), 9, dtype=torch.uint8, device="cuda")
        rt.occluded_scene(rays, occ)
        rt.sync()
        got = occ.cpu().numpy()
        bad = np.nonzero(got != ref)[0]
        assert len(bad) == 0, (mode, len(bad), bad[:8])
    rt.close()


def test_quantized_any_hit_deep_stack(oracle):
    """A deep tree (the nested-sliver chain of test_host.py: depth 22, a
    4-wide stack bound of kQ4Stack = 40) traced by rays along the chain that
    sit inside every box but miss every triangle (s + t > 1 in each sliver's
    plane) -- the walk holds the most pending entries, through the LDS stack
    into the private overflow -- and by rays that hit; bit-exact occlusion
    against the oracle in every traversal form."""
    import torch
    import spray_amd
    n = 40000
    x = (np.arange(n, dtype=np.float64) ** 3 / n ** 2).astype(np.float32)
    v = np.zeros((3 * n, 3), np.float32)
    v[0::3, 0] = x
    v[1::3, 0] = x + 1e-3
    v[1::3, 1] = 1e-3
    v[2::3, 2] = 1e-3
    v[2::3, 0] = x
    f = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    rt = spray_amd.RtContext(0)
    osc = oracle.Scene(1)
    rt.upload_domain(0, v, f)
    box = np.concatenate([v.min(0), v.max(0)]).astype(np.float32)
    osc.set_domain(0, v, f, np.zeros(len(v), np.uint32), np.zeros_like(v), box)
    rt.domain_bounds(box[None])
    rt.map_domain(0, 0)
    rng = np.random.default_rng(8)
    m = 8192
    st = rng.uniform(0.02, 0.98, size=(m, 2))
    miss = np.arange(m) % 2 == 0  # half inside every box, past the triangles
    st[miss] = 1.0 - st[miss] * 0.45  # s + t > 1.1
    st[~miss] *= 0.45                 # s + t < 0.9
    org = np.zeros((m, 3), np.float32)
    org[:, 0] = np.where(np.arange(m) % 4 < 2, -1.0, float(x[-1]) + 1.0)
    org[:, 1:] = (st * 1e-3).astype(np.float32)
    d = np.zeros((m, 3), np.float32)
    d[:, 0] = np.where(org[:, 0] < 0, 1.0, -1.0)
    d[:, 1:] = rng.normal(scale=1e-9, size=(m, 2)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    ref, _ = osc.occluded(org, d)
    assert 0.3 < ref.mean() < 0.7
    rays = torch.from_numpy(spray_amd.make_rays(org, d).view(np.uint8)).cuda()
    for mode in (rt.RAYS_INCOHERENT, rt.RAYS_ADAPTIVE, rt.RAYS_COHERENT):
        rt.set_coherence(mode)
        occ = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
        rt.occluded_scene(rays, occ)
        rt.sync()
        got = occ.cpu().numpy()
        bad = np.nonzero(got != ref)[0]
        assert len(bad) == 0, (mode, len(bad), bad[:8])
    rt.close()
