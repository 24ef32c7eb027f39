"""Experiment: any hit of the frame's AO-16 rays in different lane orders --
output order, the spawn's sample-major order, and orders sorted on the
device by keys of origin (Morton code over the scene box) and direction
(octant / quantised angles).  Prints the launch time of each and checks the
occlusion bits are identical."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import spray_amd  # noqa: E402


def spread10(x):
    x = x & 0x3FF
    x = (x | (x << 16)) & 0x030000FF
    x = (x | (x << 8)) & 0x0300F00F
    x = (x | (x << 4)) & 0x030C30C3
    x = (x | (x << 2)) & 0x09249249
    return x


def morton(p, lo, hi, bits=10):
    q = ((p - lo) / (hi - lo) * (2 ** bits - 1)).clamp(0, 2 ** bits - 1).to(torch.int64)
    return spread10(q[:, 0]) | (spread10(q[:, 1]) << 1) | (spread10(q[:, 2]) << 2)


def main():
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES)
    rt = sc.rt
    rt.set_stream(torch.cuda.current_stream())  # torch's key/sort kernels and ours in order
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
    rt.set_coherence(rt.RAYS_COHERENT)
    rt.intersect_scene(prim, hits)
    ao = torch.empty((n * 16, 8), dtype=torch.float32, device="cuda")
    src = torch.empty(n * 16, dtype=torch.int32, device="cuda")
    order = torch.empty(n * 16, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(prim, hits, pix, n, 16, ao, src, cnt, order=order)
    rt.sync()
    m = int(cnt.item())
    r = ao[:m]
    o, d = r[:, 0:3], r[:, 4:7]
    lo, hi = o.min(0).values, o.max(0).values
    mo = morton(o, lo, hi)
    octant = ((d[:, 0] < 0).long() << 2) | ((d[:, 1] < 0).long() << 1) | (d[:, 2] < 0).long()
    # direction quantised on the cube map: face (6) x 4x4 cells
    ax = d.abs().argmax(1)
    face = ax * 2 + (d.gather(1, ax[:, None])[:, 0] < 0).long()
    dq = ((d + 1) * 2).clamp(0, 3.999).long()
    dcell = face * 64 + dq[:, 0] * 16 + dq[:, 1] * 4 + dq[:, 2]
    orders = {
        "output": torch.arange(m, device="cuda", dtype=torch.int32),
        "sample-major": order[:m].clone(),
        "morton(org)": torch.argsort(mo).to(torch.int32),
        "octant,morton": torch.argsort((octant << 30) | mo).to(torch.int32),
        "dircell,morton": torch.argsort((dcell << 30) | mo).to(torch.int32),
        "morton,octant": torch.argsort((mo << 3) | octant).to(torch.int32),
    }
    rank = torch.empty(m, dtype=torch.int64, device="cuda")
    rank[order[:m].long()] = torch.arange(m, device="cuda")  # position in sample-major order
    dq8 = ((d + 1) * 4).clamp(0, 7.999).long()
    dcell8 = face * 512 + dq8[:, 0] * 64 + dq8[:, 1] * 8 + dq8[:, 2]
    orders["dircell,sample-major"] = torch.argsort((dcell << 32) | rank).to(torch.int32)
    orders["dircell512,sample-major"] = torch.argsort((dcell8 << 32) | rank).to(torch.int32)
    orders["dircell512,morton"] = torch.argsort((dcell8 << 30) | mo).to(torch.int32)
    orders["octant,sample-major"] = torch.argsort((octant << 32) | rank).to(torch.int32)
    occ = torch.empty(m, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for name, od in orders.items():  # each a permutation of [0, m)
        assert od.numel() == m and int(od.min()) == 0 and int(od.max()) == m - 1, name
    ref = None
    for mode_name, mode in (("lane", rt.RAYS_INCOHERENT),):
        rt.set_coherence(mode)
        for name, od in orders.items():
            rt.occluded_scene_order(ao, m, od, cnt, occ)
            rt.sync()
            t0 = time.perf_counter()
            for _ in range(5):
                rt.occluded_scene_order(ao, m, od, cnt, occ)
            rt.sync()
            ms = (time.perf_counter() - t0) / 5 * 1e3
            same = True if ref is None else bool(torch.equal(occ, ref))
            ref = occ.clone() if ref is None else ref
            print("%-9s %-16s %7.3f ms  same=%s" % (mode_name, name, ms, same), flush=True)
    t0 = time.perf_counter()
    for _ in range(5):
        torch.argsort((octant << 30) | mo)
    rt.sync()
    print("torch argsort of %d int64 keys: %.3f ms" % (m, (time.perf_counter() - t0) / 5 * 1e3))


if __name__ == "__main__":
    main()
