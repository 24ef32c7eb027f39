"""Times spray_rt_spawn_shadows_ao (AO-16 over the bench frame's hits) under
the shipped library and the diagnostic builds in spray_amd/lib/diag
(SPRAY_AO_DIAG=1: stores only, 2: sampling only).

    python scripts/ao_spawn_diag.py build   # here
    python scripts/ao_spawn_diag.py run     # GPU box
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG = os.path.join(ROOT, "spray_amd", "lib", "diag")
VARIANTS = {"ao_stores_only": ["SPRAY_AO_DIAG=1"], "ao_sample_only": ["SPRAY_AO_DIAG=2"]}


def one():
    import torch
    import bench
    import spray_amd
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES)
    rt = sc.rt
    rt.set_stream(torch.cuda.current_stream())  # the events below time this stream
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
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rt.spawn_shadows_ao(prim, hits, pix, n, 16, ao, src, cnt)
    rt.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        rt.spawn_shadows_ao(prim, hits, pix, n, 16, ao, src, cnt)
    e1.record()
    rt.sync()
    torch.cuda.synchronize()
    print("spawn_ao %.3f ms  (%d rays)" % (e0.elapsed_time(e1) / 10, int(cnt.item())))


def main():
    if sys.argv[1] == "build":
        from spray_amd import build as b
        for name, defs in VARIANTS.items():
            print(b.build(defines=defs, out=os.path.join(DIAG, "libspray_rt_%s.so" % name)))
    elif sys.argv[1] == "one":
        one()
    else:
        for name in ["shipped"] + list(VARIANTS):
            env = dict(os.environ)
            if name != "shipped":
                env["SPRAY_RT_LIB"] = os.path.join(DIAG, "libspray_rt_%s.so" % name)
            r = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True,
                               text=True, timeout=300)
            print("%-16s %s" % (name, (r.stdout.strip() or r.stderr[-400:])), flush=True)


if __name__ == "__main__":
    main()
