"""Generates the committed golden fixtures from the CPU oracle.

    python tests/golden/make_golden.py

* workload_counts.json -- canonical BVH2 node / triangle / domain-visit counts
  of the bench workload (configs[1]: wavelets64, 1024x1024x8spp, 8 OOC
  blocking tiles of 1024x128, PT point-light shadow rays), the per-unit
  figures of the algorithmic-byte formula.
* vectors_*.npz -- small ray batches with expected hit records (inputs and
  outputs only), checked by tests/test_oracle.py on every CPU run and by
  tests/test_gpu_configs.py::test_golden_vectors_on_device through the C ABI.

The oracle is pinned by internal consistency (BVH == brute force bit for bit,
float64 checker within 1e-4), by the survey's known answers (primary hit
fraction 0.274, 1.38 domains per ray on the 48x48 pixel-centre probe) and by
the reference's published renders (tests/golden/reference_images.npz, made by
make_image_fixtures.py; tests/test_image_pin.py); no Embree output exists to
pin it further ("Oracle").
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402

SCENES = os.path.join(HERE, "scenes")
CAM = dict(pos=[90.172180, 84.141418, 82.480225], lookat=[30.0, 28.649426, 30.0],
           up=[0.0, 1.0, 0.0], fov=90.0)
SHADE = ([0.0, 500.0, 1000.0], [1.0, 1.0, 1.0], [0.4, 0.4, 0.4], 10.0)


def workload_counts():
    sc, doms, lights = po.load_scene(os.path.join(SCENES, "wavelets64.spray"), SCENES)
    cam = po.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], 1024, 1024)
    tot = {"primary": dict(nodes=0, tris=0, visits=0, rays=0),
           "shadow": dict(nodes=0, tris=0, visits=0, rays=0)}
    hits_n = 0
    for y in range(0, 1024, 128):
        org, d, _, _ = po.eye_rays_ooc(cam, 1024, 8, (0, y, 1024, 128))
        h, c = sc.intersect(org, d)
        for k in tot["primary"]:
            tot["primary"][k] += c[k]
        hits_n += int((h["domain"] >= 0).sum())
        so, sd, _ = po.spawn_shadows_pt(org, d, h, *SHADE)
        _, c2 = sc.occluded(so, sd)
        for k in tot["shadow"]:
            tot["shadow"][k] += c2[k]
    tot["primary_hits"] = hits_n
    tot["note"] = ("canonical BVH2 (binned SAH 32 bins x 3 axes, <=4 tris/leaf), "
                   "closest-child-first, tfar carried across the sorted domain list, "
                   "early exit for occlusion; oracle/oracle.c")
    return tot


def vectors():
    rng = np.random.default_rng(20261015)
    sc, doms, lights = po.load_scene(os.path.join(SCENES, "wavelets64.spray"), SCENES)
    cam = po.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], 1024, 1024)
    org, d, pix, sam = po.eye_rays_ooc(cam, 1024, 8, (0, 384, 1024, 128))
    sel = np.sort(rng.choice(len(org), 8192, replace=False))
    org, d, pix = org[sel], d[sel], pix[sel]
    h, _ = sc.intersect(org, d)
    so, sd, src = po.spawn_shadows_pt(org, d, h, *SHADE)
    occ, _ = sc.occluded(so, sd)
    np.savez_compressed(os.path.join(HERE, "vectors_wavelets64.npz"), org=org, dir=d,
                        pixid=pix, hits=h.view(np.uint8).reshape(len(h), 48),
                        shadow_org=so, shadow_dir=sd, shadow_src=src, occluded=occ)
    # single domain: rays around wavelet.ply incl. edge/vertex-aimed rays
    v, f, c = po.load_ply(os.path.join(SCENES, "wavelet.ply"))
    ctr = (v.min(0) + v.max(0)) / 2
    u = rng.normal(size=(4096, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o1 = (ctr + 25 * u).astype(np.float32)
    tgt = ctr + rng.uniform(-12, 12, size=(4096, 3))
    ff = f[rng.integers(0, len(f), 4096)]
    tgt[::2] = v[ff[::2, 0]]  # every other ray aimed exactly at a vertex
    d1 = (tgt - o1)
    d1 = (d1 / np.linalg.norm(d1, axis=1, keepdims=True)).astype(np.float32)
    tri = po.prep_tris(v, f)
    t, uu, vv, p = po.brute_intersect(tri, o1, d1)
    o = po.brute_occluded(tri, o1, d1)
    np.savez_compressed(os.path.join(HERE, "vectors_wavelet.npz"), org=o1, dir=d1, t=t,
                        u=uu, v=vv, prim=p, occluded=o)


if __name__ == "__main__":
    c = workload_counts()
    with open(os.path.join(HERE, "workload_counts.json"), "w") as fh:
        json.dump(c, fh, indent=1)
    print(json.dumps(c))
    vectors()
    print("ok")
