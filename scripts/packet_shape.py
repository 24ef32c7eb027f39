"""Effect of the packet footprint on the fused closest-hit launch: the bench
frame's primary rays in their bufid order (8 pixels of a row x 8 spp per
wave) against the same rays permuted so that a wave holds a 4x2 or 2x4 block
of pixels (x 8 spp).  Results are checked equal (up to the permutation)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import spray_amd  # noqa: E402


def block_perm(w, rows, spp, bw, bh):
    """ray index order of a tile (w x rows, spp) walked in bw x bh pixel blocks"""
    y, x = np.mgrid[0:rows, 0:w]
    key = ((y // bh) * (w // bw) + x // bw) * (bw * bh) + (y % bh) * bw + x % bw
    pix = np.argsort(key.reshape(-1), kind="stable")
    return (pix[:, None] * spp + np.arange(spp)[None, :]).reshape(-1)


def main():
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES)
    rt = sc.rt
    rt.set_coherence(rt.RAYS_COHERENT)
    cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"],
                                bench.CAM["fov"], bench.W, bench.H)
    n = bench.W * bench.H * bench.SPP
    per = bench.W * bench.TILE_H * bench.SPP
    prim = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    pix = torch.empty(n, dtype=torch.int32, device="cuda")
    for k, t in enumerate(bench.tiles()):
        rt.eye_rays_ooc(cam, bench.W, bench.SPP, t, prim[k * per:(k + 1) * per],
                        pix[k * per:(k + 1) * per])
    hits = torch.empty((n, 12), dtype=torch.float32, device="cuda")
    sh = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    valid = torch.empty(n, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    ref = None
    for bw, bh in ((8, 1), (4, 2), (2, 4), (8, 8), (16, 4)):
        p1 = block_perm(bench.W, bench.TILE_H, bench.SPP, bw, bh)
        perm = torch.from_numpy(np.concatenate([p1 + k * per for k in range(8)])).cuda()
        rays = prim[perm].contiguous()
        rt.intersect_scene_spawn_pt(rays, hits, bench.SHADE, sh, valid, cnt)
        rt.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            rt.intersect_scene_spawn_pt(rays, hits, bench.SHADE, sh, valid, cnt)
        rt.sync()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        back = torch.empty_like(hits)
        back[perm] = hits
        same = True if ref is None else bool(torch.equal(back.view(torch.int32),
                                                          ref.view(torch.int32)))
        ref = back if ref is None else ref
        print("block %2dx%d  CH+spawn %.4f ms  same=%s" % (bw, bh, ms, same), flush=True)


if __name__ == "__main__":
    main()
