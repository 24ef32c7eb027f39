"""Bench frame: closest hit + PT spawn + any hit as two launches (bench
step) against the one-launch fused form (intersect_scene_shadow_pt)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import spray_amd  # noqa: E402


def main():
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES)
    rt = sc.rt
    rt.set_stream(torch.cuda.current_stream())
    rt.set_coherence(rt.RAYS_COHERENT)
    cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"],
                                bench.CAM["fov"], bench.W, bench.H)
    n = bench.W * bench.H * bench.SPP
    per = bench.W * bench.TILE_H * bench.SPP
    prim = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    for k, t in enumerate(bench.tiles()):
        rt.eye_rays_ooc(cam, bench.W, bench.SPP, t, prim[k * per * 32:(k + 1) * per * 32], None)
    hits = torch.empty(n * 48, dtype=torch.uint8, device="cuda")
    sh = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    valid = torch.empty(n, dtype=torch.uint8, device="cuda")
    occ = torch.empty(n, dtype=torch.uint8, device="cuda")
    occ2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    sv = torch.empty(n, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")

    def two():
        rt.intersect_scene_spawn_pt(prim, hits, bench.SHADE, sh, valid, cnt)
        rt.occluded_scene_masked(sh, valid, occ)

    def one():
        rt.intersect_scene_shadow_pt(prim, hits, bench.SHADE, occ2, sv, cnt)

    for name, f in (("two launches", two), ("fused", one), ("two launches", two), ("fused", one)):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        print("%-13s %.4f ms" % (name, (time.perf_counter() - t0) / 20 * 1e3), flush=True)
    v = valid.bool()
    print("same valid:", bool(torch.equal(valid, sv)), " same occ:",
          bool(torch.equal(occ[v], occ2[v])), " shadows:", int(v.sum()))


if __name__ == "__main__":
    main()
