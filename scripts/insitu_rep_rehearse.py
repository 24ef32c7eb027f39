"""Per-rank device time of the replicated-ray in-situ frame at N ranks,
rehearsed on ONE GPU (the input of scripts/insitu_rep_projection.py).

    python scripts/insitu_rep_rehearse.py --worlds 2 4 8 --modes close rr \
        --out gpurun_out/rep/rehearse.json

For each (N, partition) N processes share the GPU, each an engine rank with
its 64/N domains (gloo + the engine's host transport), and trace the bench
frame (1024x1024x8spp, PT) with spray_rt_insitu_trace_frame.  With
SPRAY_INSITU_SERIAL the ranks' device work runs one rank at a time (a file
lock released while a rank waits in a collective), so the per-phase HIP-event
times of a rank are its own kernels' times, not shared-GPU contention.  The
collectives' times (host-staged here) are NOT measurements of RCCL: the
projection models them.  Also measured: the one-rank RCCL all-reduce of the
frame's message sizes (the per-call floor of the real collectives).
"""
import argparse
import itertools
import json
import os
import socket
import sys
import tempfile
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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, mode, frames, out, kind="pt"):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    boxes, lights = host_parse_scene(SCENE, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    pm = insitu.PARTITION_ROUND_ROBIN if mode == "rr" else insitu.PARTITION_GROUP_CLOSE
    owner = insitu.morton_partition(boxes, bound, world, pm)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, SCENE, SCENES, owner, rank)
    rt.set_bsdfs(host_scene_bsdfs(SCENE))
    stream = torch.cuda.Stream()
    rt.set_stream(stream)
    eng = insitu.InsituEngine(rt, world, rank, dist=dist, transport="host")
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    # pt / ao: the replicated-ray frames (every eye ray on every rank);
    # ao_protocol: AO-16 through the stripe protocol (the rank's stripe)
    proto = kind == "ao_protocol"
    stripe = insitu.horizontal_stripe(world, rank, (0, 0, W, H)) if proto else (0, 0, W, H)
    n = stripe[2] * stripe[3] * SPP
    rays = torch.empty((max(n, 1), 8), dtype=torch.float32, device="cuda")[:n]
    pix = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    sam = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")[:n]
    rt.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), stripe, rays, pix, sam)
    ao = kind != "pt"
    sh = spray_amd.frame.make_shader("ao" if ao else "pt", 1, 16 if ao else 1, ks=SHADE[6:9],
                                     shininess=SHADE[9], lights=lights)
    trace = eng.trace if proto else eng.trace_frame
    image = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rt.sync()
    tot = trace(sh, rays, pix, sam, SPP, image)  # warm-up (buffers)
    eng.set_timing(True)
    eng.phase_times()
    s0 = eng.stats()
    for _ in range(frames):
        tot = trace(sh, rays, pix, sam, SPP, image)
    s1 = eng.stats()
    ph = {k: v / frames for k, v in eng.phase_times().items()}
    # no device work outside the lock until every rank's frames are done (the
    # sizes below would run beside a slower rank's last frame)
    dist.barrier()
    # the sizes of the frame's collectives: PT |C'| (rays entering the
    # scene's bounding box: k_rep_cull's slab test, the same float ops), AO
    # |C| (rays with a non-empty domain list), and the pixel runs along them
    if kind == "pt":
        lo = torch.tensor(boxes[:, :3].min(0), dtype=torch.float32, device="cuda")
        hi = torch.tensor(boxes[:, 3:].max(0), dtype=torch.float32, device="cuda")
        o, dr = rays[:, 0:3], rays[:, 4:7]
        inv = 1.0 / dr
        neg = inv < 0
        t0 = (torch.where(neg, hi, lo) - o) * inv
        t1 = (torch.where(neg, lo, hi) - o) * inv
        tmin = t0.max(dim=1).values
        tmax = t1.min(dim=1).values
        on = ((tmin <= tmax) & (tmin < float("inf")) & (tmax > 0.001)) | (dr == 0).any(dim=1)
    else:
        m = torch.empty(n, dtype=torch.int64, device="cuda")
        rt.route(rays, m)
        on = m != 0
    pc = pix[on]
    nc, nruns = int(on.sum()), int(1 + (pc[1:] != pc[:-1]).sum()) if pc.numel() else 0
    res = {"rank": rank, "pid": os.getpid(), "domains": int((owner == rank).sum()),
           "phases_ms": ph,
           "nc": nc, "pixel_runs": nruns,
           "totals": list(tot), "stats": eng.stats(),
           "per_frame": {k: (s1[k] - s0[k]) / frames for k in s1}}
    with open(os.path.join(out, "r%d.json" % rank), "w") as fh:
        json.dump(res, fh)
    eng.close()
    rt.close()
    dist.destroy_process_group()


def rccl_floor(sizes):
    """One-rank RCCL all-reduce time per message size (ms): the per-call
    floor of the frame's collectives (no link traffic at one rank)."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out = {}
    for name, (nbytes, dtype, op) in sizes.items():
        t = torch.zeros(max(nbytes // torch.tensor([], dtype=dtype).element_size(), 1),
                        dtype=dtype, device="cuda")
        for _ in range(5):
            dist.all_reduce(t, op=op)
        torch.cuda.synchronize()
        k = 50
        t0 = time.perf_counter()
        for _ in range(k):
            dist.all_reduce(t, op=op)
        torch.cuda.synchronize()
        out[name] = {"bytes": nbytes, "ms": (time.perf_counter() - t0) / k * 1e3}
    dist.destroy_process_group()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--modes", nargs="+", default=["close", "rr"])
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--kinds", nargs="+", default=["pt"],
                    help="pt: replicated PT frame (configs[2]); ao: replicated AO-16 frame "
                         "(configs[4]); ao_protocol: AO-16 through the stripe protocol")
    ap.add_argument("--out", default="gpurun_out/rep/rehearse.json")
    ap.add_argument("--rccl-floor", type=int, default=1)
    args = ap.parse_args()
    import torch
    import torch.multiprocessing as mp
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    lock = os.path.join(tempfile.gettempdir(), "spray_insitu_serial_%d.lock" % os.getpid())
    os.environ["SPRAY_INSITU_SERIAL"] = lock
    report = {"frame": "wavelets64 1024x1024x8spp: PT / AO-16 replicated-ray frames "
                       "(configs[2] / configs[4]), AO-16 stripe protocol", "runs": []}
    for kind, mode, world in itertools.product(args.kinds, args.modes, args.worlds):
        t0 = time.time()
        with tempfile.TemporaryDirectory() as out:
            mp.spawn(_rank, args=(world, _port(), mode, args.frames, out, kind), nprocs=world)
            ranks = [json.load(open(os.path.join(out, "r%d.json" % r))) for r in range(world)]
        report["runs"].append({"world": world, "partition": mode, "kind": kind, "ranks": ranks})
        print("%s world %d %s: %.1f s; per-rank device ms: %s" % (
            kind, world, mode, time.time() - t0,
            [round(sum(v for k, v in r["phases_ms"].items() if k != "collectives"), 3)
             for r in ranks]), flush=True)
        with open(args.out, "w") as fh:
            json.dump(report, fh, indent=1)
    os.environ.pop("SPRAY_INSITU_SERIAL", None)
    if args.rccl_floor:
        nc = 2600000  # ~ rays of the bench frame with a non-empty domain list
        report["rccl_one_rank_floor"] = rccl_floor({
            "keys_min_u64": (8 * nc, torch.int64, torch.distributed.ReduceOp.MIN),
            "ao_normals_u64": (16 * nc, torch.int64, torch.distributed.ReduceOp.SUM),
            "ao_fields_u8": (8 * nc, torch.uint8, torch.distributed.ReduceOp.SUM),
            "occ_sum_u8": (nc + 192, torch.uint8, torch.distributed.ReduceOp.SUM),
            "image_16MB": (W * H * 16, torch.float32, torch.distributed.ReduceOp.SUM),
            "small_8B": (8, torch.int64, torch.distributed.ReduceOp.SUM)})
        print("rccl floor:", report["rccl_one_rank_floor"], flush=True)
    with open(args.out, "w") as fh:
        json.dump(report, fh, indent=1)
    try:
        os.unlink(lock)
    except OSError:
        pass


if __name__ == "__main__":
    main()
