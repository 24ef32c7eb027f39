"""Per-rank kernel times of the replicated PT frame, one process, no
collectives: for each rank of an N-way partition its engine context (own
domains resident), then -- on the bench frame's eye rays (wavelets64,
1024x1024x8spp) -- the launches a replicated frame makes on that rank, each
timed alone with HIP events on the context's stream:

  route      owner-rank masks of every eye ray (launch_route)
  keyed      keyed closest hit of the rank's rays L (compacted) over its domains
  shadows    any hit of every hit's point-light shadow ray over its domains
             (the hits from a whole-scene context, positional with a mask)

    python scripts/insitu_rank_kernels.py --worlds 8 --modes close rr

The rehearsal (insitu_rep_rehearse.py) times whole phases with the ranks'
device work serialised; this isolates the kernels of one rank.
"""
import argparse
import json
import os
import sys

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


def timed(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    s = torch.cuda.current_stream()
    for k in range(reps):
        ev[2 * k].record(s)
        fn()
        ev[2 * k + 1].record(s)
    torch.cuda.synchronize()
    return float(np.median([ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(reps)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[8])
    ap.add_argument("--modes", nargs="+", default=["close", "rr"])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    boxes, _ = host_parse_scene(SCENE, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    n = W * H * SPP
    rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    pix = torch.empty(n, dtype=torch.int32, device="cuda")
    sam = torch.empty(n, dtype=torch.int32, device="cuda")
    # whole scene: the frame's hits and their shadow rays
    sc = spray_amd.Scene(SCENE, SCENES, cache_size=-1)
    full = sc.rt
    full.set_stream(stream)
    full.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), (0, 0, W, H), rays, pix, sam)
    full.set_coherence(full.RAYS_COHERENT)
    hits = torch.empty((n, 12), dtype=torch.float32, device="cuda")
    srays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    svalid = torch.empty(n, dtype=torch.uint8, device="cuda")
    nsh = torch.zeros(1, dtype=torch.int32, device="cuda")
    occ = torch.empty(n, dtype=torch.uint8, device="cuda")
    t_fused = timed(lambda: full.intersect_scene_shadow_pt(rays, hits, SHADE, occ, svalid, nsh))
    full.intersect_scene_spawn_pt(rays, hits, SHADE, srays, svalid, nsh)
    torch.cuda.synchronize()
    report = {"n_rays": n, "n_shadow": int(nsh.item()), "n1_fused_ms": round(t_fused, 4),
              "runs": []}
    print("N=1 fused launch %.3f ms, %d shadow rays" % (t_fused, int(nsh.item())), flush=True)
    # C' (rays entering the scene box) gathered: keyed closest hit over it
    # with every domain resident vs. each rank's domains only
    lo = torch.tensor(boxes[:, :3].min(0), dtype=torch.float32, device="cuda")
    hi = torch.tensor(boxes[:, 3:].max(0), dtype=torch.float32, device="cuda")
    o, dr = rays[:, 0:3], rays[:, 4:7]
    inv = 1.0 / dr
    neg = inv < 0
    tmn = ((torch.where(neg, hi, lo) - o) * inv).max(dim=1).values
    tmx = ((torch.where(neg, lo, hi) - o) * inv).min(dim=1).values
    cp = rays[((tmn <= tmx) & (tmn < float("inf")) & (tmx > 0.001)) | (dr == 0).any(dim=1)]
    cp = cp.contiguous()
    ncp = cp.shape[0]
    ch = torch.empty((ncp, 12), dtype=torch.float32, device="cuda")
    ck = torch.empty(ncp, dtype=torch.int64, device="cuda")
    t_full_keyed = timed(lambda: full.intersect_scene_keyed(cp, ch, ck))
    t_full_ch = timed(lambda: full.intersect_scene(cp, ch))
    full.set_coherence(full.RAYS_INCOHERENT)
    t_full_lane = timed(lambda: full.intersect_scene(cp, ch))
    full.set_coherence(full.RAYS_COHERENT)
    report["cprime"] = {"n": ncp, "full_keyed_ms": round(t_full_keyed, 4),
                        "full_ch_ms": round(t_full_ch, 4), "full_ch_lane_ms": round(t_full_lane, 4)}
    print("C' %d rays: all domains keyed %.3f ms, plain CH packets %.3f / per lane %.3f ms" % (
        ncp, t_full_keyed, t_full_ch, t_full_lane), flush=True)
    for world in args.worlds:
        for mode in args.modes:
            pm = insitu.PARTITION_ROUND_ROBIN if mode == "rr" else insitu.PARTITION_GROUP_CLOSE
            owner = insitu.morton_partition(boxes, bound, world, pm)
            ranks = []
            for r in range(world):
                rt = spray_amd.RtContext(0)
                insitu.setup_rank_context(rt, SCENE, SCENES, owner, r)
                rt.set_stream(stream)
                rt.set_coherence(rt.RAYS_COHERENT)
                m = torch.empty(n, dtype=torch.int64, device="cuda")
                t_route = timed(lambda: rt.route(rays, m))
                on = m != 0
                mine = ((m >> r) & 1).bool()
                lr = rays[mine].contiguous()
                nl = lr.shape[0]
                lh = torch.empty((max(nl, 1), 12), dtype=torch.float32, device="cuda")[:nl]
                lk = torch.empty(max(nl, 1), dtype=torch.int64, device="cuda")[:nl]
                t_keyed = timed(lambda: rt.intersect_scene_keyed(lr, lh, lk)) if nl else 0.0
                so = torch.empty(n, dtype=torch.uint8, device="cuda")
                t_sh = timed(lambda: rt.occluded_scene_masked(srays, svalid, so))
                t_ck = timed(lambda: rt.intersect_scene_keyed(cp, ch, ck))
                t_cc = timed(lambda: rt.intersect_scene(cp, ch))
                rt.set_coherence(rt.RAYS_INCOHERENT)  # the same launch walked per lane
                t_cl = timed(lambda: rt.intersect_scene(cp, ch))
                rt.set_coherence(rt.RAYS_COHERENT)
                ranks.append({"rank": r, "L": nl, "C": int(on.sum()), "route_ms": round(t_route, 4),
                              "keyed_ms": round(t_keyed, 4), "shadow_ms": round(t_sh, 4),
                              "cprime_keyed_ms": round(t_ck, 4), "cprime_ch_ms": round(t_cc, 4),
                              "cprime_ch_lane_ms": round(t_cl, 4)})
                print("N=%d %s rank %d: L %d route %.3f keyed(L) %.3f shadow %.3f keyed(C') %.3f "
                      "CH(C') packets %.3f per lane %.3f ms" % (
                          world, mode, r, nl, t_route, t_keyed, t_sh, t_ck, t_cc, t_cl), flush=True)
                rt.close()
            report["runs"].append({"world": world, "partition": mode, "ranks": ranks})
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(report, fh, indent=1)
    sc.close()


if __name__ == "__main__":
    main()
