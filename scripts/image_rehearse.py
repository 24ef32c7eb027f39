"""Per-rank device time of the image-parallel frame (spray_rt_insitu_trace_image,
bench.py's "image_parallel" key) at N ranks, each rank rehearsed ALONE on one
GPU with its exact share of the work, and the N-GPU frame projected from them.

    python scripts/image_rehearse.py --worlds 1 2 4 8 --bands 1 2 4 8 \
        --out gpurun_out/img/rehearse.json

The image-parallel frame has no data dependency between ranks until its end:
each rank traces its own row bands with every domain resident, then the rows
go to rank 0 in one gather and the totals in one 24-B all-reduce.  A replay
engine (spray_rt_insitu_create_replay) runs a rank's part exactly -- its eye
rays, launches and film -- with the gather and the all-reduce keeping the
rank's own data, so the per-rank device time is measured, not modelled.
Projection: the busiest rank's frame + the gather (every rank but 0 sends
the RGB of its rows' pixels in U -- those some domain box's footprint covers,
12 B each -- to rank 0 on its own xGMI link: alpha + the largest rank's bytes
/ link bandwidth, conservative / optimistic) + the totals all-reduce (alpha).
No multi-GPU box is available to this build: the link terms are modelled.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
SCENE = os.path.join(SCENES, "wavelets64.spray")
CAM = dict(pos=[90.172180, 84.141418, 82.480225], lookat=[30.0, 28.649426, 30.0],
           up=[0.0, 1.0, 0.0], fov=90.0)
W = H = 1024
SPP = 8
SHADE = [0.0, 500.0, 1000.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4, 10.0]
# point-to-point xGMI link (one per peer pair): alpha per call (ms) and GB/s;
# the small all-reduce: alpha only
LINK = {"cons": (0.030, 100.0), "opt": (0.015, 140.0)}
AR_ALPHA = {"cons": 0.030, "opt": 0.015}


def u_rows(cam, boxes):
    """Per image row the pixels of U (the union of the boxes' footprints)."""
    from spray_amd import insitu
    cover = np.zeros((H, W), bool)
    for b in boxes:
        k, x0, x1 = insitu.box_rows(cam, W, H, b[:6])
        if k == 2:
            cover[:] = True
        elif k == 1:
            for y in np.nonzero(x1 >= x0)[0]:
                cover[y, x0[y]:x1[y] + 1] = True
    return cover.sum(1)


def gather_bytes(urow, world, bands):
    """Bytes each rank sends to rank 0 (its bands' U pixels, 12 B each)."""
    bt = world * bands
    out = np.zeros(world)
    for b in range(bt):
        out[b % world] += urow[b * H // bt:(b + 1) * H // bt].sum() * 12
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--bands", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--kinds", nargs="+", default=["pt"])
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    torch.cuda.set_device(0)
    boxes, lights = host_parse_scene(SCENE, SCENES)
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, SCENE, SCENES, np.zeros(len(boxes), np.int32), 0)
    rt.set_bsdfs(host_scene_bsdfs(SCENE))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rt.set_stream(stream)
    image = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    urow = u_rows(cam, boxes)
    out = {"runs": [], "link": LINK, "frames": args.frames, "u_pixels": int(urow.sum())}
    for kind in args.kinds:
        sh = spray_amd.frame.make_shader(kind, 1, 16 if kind == "ao" else 1, ks=SHADE[6:9],
                                         shininess=SHADE[9], lights=lights)
        for world in args.worlds:
            for bands in (args.bands if world > 1 else [1]):
                if H % (world * bands) and bands > 1:
                    continue
                ranks = []
                for rank in range(world):
                    eng = insitu.InsituEngine(rt, world, rank, transport="replay")
                    eng.set_timing(True)
                    for _ in range(args.warmup):
                        image.zero_()
                        eng.trace_image(sh, cam, W, H, SPP, image, bands)
                    eng.phase_times()
                    t0 = time.perf_counter()
                    for _ in range(args.frames):
                        image.zero_()
                        tot = eng.trace_image(sh, cam, W, H, SPP, image, bands)
                    torch.cuda.synchronize()
                    wall = (time.perf_counter() - t0) / args.frames * 1e3
                    ph = eng.phase_times()
                    ranks.append({"rank": rank, "frame_ms": ph.get("frame", 0.0) / args.frames,
                                  "wall_ms": wall, "rays": tot[0] + tot[1]})
                    eng.close()
                busiest = max(r["frame_ms"] for r in ranks)
                gb = gather_bytes(urow, world, bands)
                proj = {}
                for k, (alpha, bw) in LINK.items():
                    comm = 0.0
                    if world > 1:
                        comm = alpha + gb[1:].max() / (bw * 1e9) * 1e3 + AR_ALPHA[k]
                    proj[k] = round(busiest + comm, 4)
                run = {"kind": kind, "world": world, "bands": bands, "ranks": ranks,
                       "gather_bytes": [int(x) for x in gb],
                       "busiest_ms": round(busiest, 4),
                       "mean_ms": round(float(np.mean([r["frame_ms"] for r in ranks])), 4),
                       "sum_ms": round(float(np.sum([r["frame_ms"] for r in ranks])), 4),
                       "projected_ms": proj}
                out["runs"].append(run)
                print("%s N=%d bands=%d busiest %.3f mean %.3f sum %.3f ms -> frame %.3f / %.3f ms"
                      % (kind, world, bands, busiest, run["mean_ms"], run["sum_ms"],
                         proj["cons"], proj["opt"]), flush=True)
    base = {r["kind"]: r["projected_ms"]["cons"] for r in out["runs"] if r["world"] == 1}
    for r in out["runs"]:
        if r["kind"] in base:
            r["speedup"] = {k: round(base[r["kind"]] / v, 3) for k, v in r["projected_ms"].items()}
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        json.dump(out, open(args.out, "w"), indent=1)
    rt.close()


if __name__ == "__main__":
    main()
