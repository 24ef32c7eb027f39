"""Times the AO-16 any-hit launch of the bench frame under each traversal
form (spray_rt_set_coherence: packet, per lane, per-wave adaptive), in the
spawn's output order and in its sample-major trace order."""
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
    rt.intersect_scene(prim, hits)
    ao = torch.empty(n * 16 * 32, dtype=torch.uint8, device="cuda")
    src = torch.empty(n * 16, dtype=torch.int32, device="cuda")
    order = torch.empty(n * 16, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(prim, hits, pix, n, 16, ao, src, cnt, order=order)
    rt.sync()
    m = int(cnt.item())
    occ = torch.empty(m, dtype=torch.uint8, device="cuda")
    ref = None
    for ordered in (False, True):
        for name, mode in (("adaptive", 0), ("packet", 1), ("lane", 2)):
            rt.set_coherence(mode)

            def run():
                if ordered:
                    rt.occluded_scene_order(ao, m, order, cnt, occ)
                else:
                    rt.occluded_scene(ao[:m * 32], occ)
            run()
            rt.sync()
            t0 = time.perf_counter()
            for _ in range(5):
                run()
            rt.sync()
            ms = (time.perf_counter() - t0) / 5 * 1e3
            o = occ.clone()
            same = True if ref is None else bool(torch.equal(o, ref))
            ref = o if ref is None else ref
            print("%-8s %-9s %8.3f ms  %d rays  occluded %.3f  same=%s" % (
                "ordered" if ordered else "output", name, ms, m, float(o.float().mean()), same),
                flush=True)


if __name__ == "__main__":
    main()
