import sys, os, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import bench
import spray_amd
torch.cuda.set_device(0)
sc = spray_amd.Scene(bench.SCENE, bench.SCENES, cache_size=-1, device=0)
rt = sc.rt
st = torch.cuda.Stream(); torch.cuda.set_stream(st); rt.set_stream(st)
cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"], bench.CAM["fov"], 1024, 1024)
W=1024; SPP=8
def rays_rows(y0, h):
    n = W*h*SPP
    r = torch.empty(n*32, dtype=torch.uint8, device="cuda"); p = torch.empty(n, dtype=torch.int32, device="cuda")
    rt.eye_rays_ooc(cam, W, SPP, (0, y0, W, h), r, p)
    return r, n
rt.set_coherence(rt.RAYS_COHERENT)
out = {"env": os.environ.get("SPRAY_STATIC_FIRST")}
for name, (y0, h) in {"miss_1M": (896, 128), "miss_64K": (1016, 8), "mid_1M": (384, 128), "full": (0, 1024)}.items():
    r, n = rays_rows(y0, h)
    hits = torch.empty(n*48, dtype=torch.uint8, device="cuda")
    occ = torch.empty(n, dtype=torch.uint8, device="cuda"); val = torch.empty(n, dtype=torch.uint8, device="cuda")
    nsh = torch.zeros(1, dtype=torch.int32, device="cuda")
    for m in ([n, 64] if name == "miss_1M" else [n]):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = []
        for k in range(12):
            ev[0].record(st); rt.intersect_scene_shadow_pt(r[:m*32], hits[:m*48], bench.SHADE, occ[:m], val[:m], nsh); ev[1].record(st)
            torch.cuda.synchronize(); ts.append(ev[0].elapsed_time(ev[1]))
        out["%s_M%d" % (name, m)] = round(float(np.median(ts[2:]))*1e3, 1)
print(json.dumps(out))
