"""Per-pair cost of the out-of-core any-hit drains vs the in-core any hit on
the same shadow rays (the bench frame's PT shadows): run under
rocprofv3 --kernel-trace --stats.  SLOTS: cache slots of the OOC run."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import spray_amd  # noqa: E402

slots = int(os.environ.get("SLOTS", "64"))
sc = spray_amd.Scene(bench.SCENE, bench.SCENES, cache_size=-1)
rt = sc.rt
cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"],
                            bench.CAM["fov"], bench.W, bench.H)
n = bench.W * bench.H * bench.SPP
per = bench.W * bench.TILE_H * bench.SPP
prim = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
pix = torch.empty(n, dtype=torch.int32, device="cuda")
for k, t in enumerate(bench.tiles()):
    rt.eye_rays_ooc(cam, bench.W, bench.SPP, t, prim[k * per * 32:(k + 1) * per * 32],
                    pix[k * per:(k + 1) * per])
hits = torch.empty(n * 48, dtype=torch.uint8, device="cuda")
shadow = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
src = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
occ = torch.empty(n, dtype=torch.uint8, device="cuda")
rt.set_coherence(rt.RAYS_COHERENT)
rt.intersect_scene(prim, hits)
rt.spawn_shadows_pt(prim, hits, n, bench.SHADE, shadow, src, cnt)
rt.sync()
ns = int(cnt.item())
for _ in range(3):
    rt.occluded_scene(shadow[:ns * 32], occ[:ns])
rt.sync()
ref = occ[:ns].clone()
rt2, oc = spray_amd.engine.ooc_scene(bench.SCENE, bench.SCENES, slots)
rt2.set_coherence(rt2.RAYS_COHERENT)
occ2 = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(3):
    oc.occluded(shadow[:ns * 32], None, occ2[:ns])
rt2.sync()
print("shadow rays", ns, "same bits", bool(torch.equal(ref, occ2[:ns])), "occluded",
      int(ref.sum()))
