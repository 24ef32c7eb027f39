"""The bench's "ooc" line alone (configs[3]: 4-slot HBM cache), for kernel
traces: python scripts/ooc_only.py [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("OOC_PKG_ROOT"):  # an A/B build of the package
    sys.path.insert(0, os.environ["OOC_PKG_ROOT"])


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import torch
    import spray_amd  # before bench (which puts the repo first on sys.path)
    import bench

    class A:
        steps = frames
        warmup = 3
    torch.cuda.set_device(0)
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES, cache_size=-1, device=0)
    rt = sc.rt
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rt.set_stream(stream)
    cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"],
                                bench.CAM["fov"], bench.W, bench.H)
    n = bench.W * bench.H * bench.SPP
    per = bench.W * bench.TILE_H * bench.SPP
    prim = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    pixid = torch.empty(n, dtype=torch.int32, device="cuda")
    for k, t in enumerate(bench.tiles()):
        rt.eye_rays_ooc(cam, bench.W, bench.SPP, t, prim[k * per * 32:(k + 1) * per * 32],
                        pixid[k * per:(k + 1) * per])
    t0 = time.time()
    out = bench.run_ooc(A, rt, prim, n)
    print(out, "%.1f s" % (time.time() - t0), flush=True)
    sc.close()


if __name__ == "__main__":
    main()
