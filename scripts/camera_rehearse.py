"""Per-rank device time of the camera frame (spray_rt_insitu_trace_camera,
bench.py's N > 1 configs[2] line) at N ranks, each rank rehearsed ALONE on
one GPU with its exact share of the work, and the N-GPU frame projected from
them.

    python scripts/camera_rehearse.py --worlds 2 4 8 --modes close rr view \
        --out gpurun_out/cam/rehearse.json

1. Capture: a one-rank context with every domain resident traces the frame
   with the replicated steps (SPRAY_INSITU_REPLICATED=1, one-rank RCCL); its
   t-bits minima and list-position minima over U are the group results of
   ANY partition (U and the winners do not depend on it).
2. Per (N, partition, rank): a context holding the rank's domains and a
   replay engine (spray_rt_insitu_create_replay) whose collectives hand back
   the captured minima.  The rank's launches -- their sizes, the rays they
   walk, the shadow rays of the group's winners over its shadow footprint --
   are the N-rank frame's, run back to back on one stream (no idle gaps, its
   own data in the caches).  HIP-event phase times averaged over --frames.
3. Projection: the frame's three segments between the collectives that
   synchronise the group (t MIN; occlusion SUM; film reduce), each at its
   busiest rank, plus a link model of those collectives (alpha + bytes /
   bus bandwidth, conservative / optimistic; the list-position MIN runs on a
   side stream beside the shadow launch).  No multi-GPU box is available to
   this build: the link terms are modelled, the device terms measured.
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
MODES = {"close": 0, "rr": 1, "view": 2}
SEGMENTS = [("prepare", "keyed_shade"), ("list_pos", "shadow_trace", "winners"), ("film_totals",)]
# AO-16 (configs[4]): between the key MIN, the publish SUM and the occlusion SUM
SEGMENTS_AO = [("prepare", "keyed_closest_hit"), ("publish",), ("ao_spawn", "ao_own_trace"),
               ("film_totals",)]
AO_SAMPLES = 16
# ring all-reduce / reduce on N GPUs: alpha per call (ms) and bus bandwidth (GB/s)
LINK = {"cons": (0.030, 300.0), "opt": (0.015, 500.0)}


def balanced_partition(boxes, w, world, cam, mode):
    """Experimental equal-count partitions balancing weights w: hitlpt =
    largest weight first to the lightest rank with room; hitaxis = recursive
    equal-count splits of the projected box centres, each along the screen
    axis whose halves' weights differ least."""
    n = len(boxes)
    per = n // world
    if mode == "hitlpt":
        owner = np.zeros(n, np.int32)
        load = np.zeros(world)
        cnt = np.zeros(world, np.int64)
        for d in np.argsort(-w, kind="stable"):
            r = min((k for k in range(world) if cnt[k] < per), key=lambda k: (load[k], k))
            owner[d] = r
            load[r] += w[d]
            cnt[r] += 1
        return owner
    pos = np.asarray(cam["pos"], np.float64)
    f = np.asarray(cam["lookat"], np.float64) - pos
    f /= np.linalg.norm(f)
    rt = np.cross(f, np.asarray(cam["up"], np.float64))
    rt /= np.linalg.norm(rt)
    up = np.cross(rt, f)
    c = 0.5 * (boxes[:, :3] + boxes[:, 3:]).astype(np.float64) - pos
    z = c @ f
    xy = np.stack([(c @ rt) / z, (c @ up) / z], 1)
    owner = np.zeros(n, np.int32)

    def split(ids, r0, k):
        if k == 1:
            owner[ids] = r0
            return
        best = None
        for ax in (0, 1):
            o = ids[np.argsort(xy[ids, ax], kind="stable")]
            h = len(o) // 2
            diff = abs(w[o[:h]].sum() - w[o[h:]].sum())
            if best is None or diff < best[0]:
                best = (diff, o[:h], o[h:])
        split(best[1], r0, k // 2)
        split(best[2], r0 + k // 2, k // 2)

    split(np.arange(n), 0, world)
    return owner


def comm_ms(world, nu, npu, model):
    """t MIN (4 B / slot) + occlusion SUM (1 B / slot + 192) all-reduces and
    the film reduce (12 B / U pixel); ring all-reduce moves 2 (N-1)/N of the
    bytes per GPU, a reduce (N-1)/N"""
    if world == 1:
        return 0.0
    a, bw = LINK[model]
    f = (world - 1) / world
    ar = lambda b: a + 2 * f * b / (bw * 1e6)  # noqa: E731
    rd = lambda b: a + f * b / (bw * 1e6)  # noqa: E731
    return ar(4 * nu) + ar(nu + 192) + rd(12 * npu)


def comm_ao_ms(world, nu, model):
    """AO: key MIN (8 B / slot), published normals + colours SUM (16 B /
    slot), the first round's occlusion bits SUM (1 bit per (slot, sample)),
    occlusion count fields SUM (fb bits per (slot, sample)), the per-pixel
    film slices reduced to rank 0 (12 B per U pixel)"""
    if world == 1:
        return 0.0
    a, bw = LINK[model]
    f = (world - 1) / world
    fb = 2 if world <= 3 else (4 if world <= 15 else 8)
    ar = lambda b: a + 2 * f * b / (bw * 1e6)  # noqa: E731
    rd = lambda b: a + f * b / (bw * 1e6)  # noqa: E731
    return (ar(8 * nu) + ar(16 * nu) + ar(nu * AO_SAMPLES / 8) + ar(nu * AO_SAMPLES * fb / 8) +
            rd(12 * nu / SPP))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--modes", nargs="+", default=["close", "rr", "view"],
                    help="close / rr / view, or (AO, experimental) hitlpt / hitaxis / fplpt")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/cam/rehearse.json")
    ap.add_argument("--shader", choices=("pt", "ao"), default="pt",
                    help="pt: configs[2] (PT point-light shadows); ao: configs[4] (AO-16)")
    args = ap.parse_args()
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    boxes, lights = host_parse_scene(SCENE, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    ao = args.shader == "ao"
    segments = SEGMENTS_AO if ao else SEGMENTS
    if ao:
        sh = spray_amd.frame.make_shader("ao", 1, AO_SAMPLES, lights=lights)
    else:
        sh = spray_amd.frame.make_shader("pt", 1, 1, ks=SHADE[6:9], shininess=SHADE[9],
                                         lights=lights)
    image = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")

    # 1. the group results (every domain on one rank, replicated steps)
    os.environ["SPRAY_INSITU_REPLICATED"] = "1"
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, SCENE, SCENES, np.zeros(len(boxes), np.int32), 0)
    rt.set_bsdfs(host_scene_bsdfs(SCENE))
    rt.set_stream(stream)
    eng = insitu.InsituEngine(rt, 1, 0, transport="rccl")
    tot = eng.trace_camera(sh, cam, W, H, SPP, image)
    if ao:
        kmin, pub = eng.replay_capture_ao()
        nu = kmin.numel()
    else:
        tmin, lpmin = eng.replay_capture()
        nu = tmin.numel()
    print("capture: %d U slots (%d pixels), totals %s" % (nu, nu // SPP, tot), flush=True)
    eng.close()
    rt.close()
    os.environ.pop("SPRAY_INSITU_REPLICATED")
    report = {"frame": "wavelets64 1024x1024x8spp %s camera frame (%s)" % (
                  ("AO-16", "configs[4]") if ao else ("PT", "configs[2]")), "u_slots": nu,
              "u_pixels": nu // SPP, "totals": list(tot), "link": LINK, "runs": []}

    # per-domain AO / eye-ray work weights for the experimental balanced
    # partitions: the U slots each domain wins (the captured key minima)
    win = None
    if ao:
        km = kmin.cpu().numpy().astype(np.uint64)
        hit = km != np.uint64(0x7FFFFFFFFFFFFFFF)
        win = np.bincount((km[hit] & np.uint64(0xFFFF)).astype(np.int64),
                          minlength=len(boxes)).astype(np.float64)
    for mode in args.modes:
        for world in args.worlds:
            if mode in ("hitlpt", "hitaxis"):
                owner = balanced_partition(boxes, win, world, CAM, mode)
            elif mode == "fplpt":  # weights: the boxes' screen footprints (pixels)
                fpw = np.array([float(np.clip(x1 - x0 + 1, 0, None).sum()) if k == 1 else float(W * H)
                                for k, x0, x1 in (insitu.box_rows(cam, W, H, b) for b in boxes)])
                owner = balanced_partition(boxes, fpw, world, CAM, "hitlpt")
            else:
                owner = insitu.partition(boxes, bound, world, MODES[mode], cam)
            ranks = []
            t0 = time.time()
            bits = None
            if ao:
                # the first round's occlusion bits depend on the partition:
                # every rank once, OR-ed, then handed back by that SUM
                for r in range(world):
                    rt = spray_amd.RtContext(0)
                    insitu.setup_rank_context(rt, SCENE, SCENES, owner, r)
                    rt.set_bsdfs(host_scene_bsdfs(SCENE))
                    rt.set_stream(stream)
                    eng = insitu.InsituEngine(rt, world, r, transport="replay")
                    eng.replay_set_ao(kmin, pub)
                    eng.trace_camera(sh, cam, W, H, SPP, image)
                    own = eng.replay_bits_ao()
                    bits = own.clone() if bits is None else bits | own
                    eng.close()
                    rt.close()
            for r in range(world):
                rt = spray_amd.RtContext(0)
                insitu.setup_rank_context(rt, SCENE, SCENES, owner, r)
                rt.set_bsdfs(host_scene_bsdfs(SCENE))
                rt.set_stream(stream)
                eng = insitu.InsituEngine(rt, world, r, transport="replay")
                if ao:
                    eng.replay_set_ao(kmin, pub)
                    eng.replay_bits_ao(bits)
                else:
                    eng.replay_set(tmin, lpmin)
                for _ in range(3):
                    eng.trace_camera(sh, cam, W, H, SPP, image)
                eng.set_timing(True)
                eng.phase_times()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(stream)
                for _ in range(args.frames):
                    eng.trace_camera(sh, cam, W, H, SPP, image)
                ev[1].record(stream)
                torch.cuda.synchronize()
                ph = {k: v / args.frames for k, v in eng.phase_times().items()}
                eng.set_timing(False)
                # the same frames without the phase events: the rank's wall time
                ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev2[0].record(stream)
                for _ in range(args.frames):
                    eng.trace_camera(sh, cam, W, H, SPP, image)
                ev2[1].record(stream)
                torch.cuda.synchronize()
                seg = [sum(ph.get(k, 0.0) for k in s) for s in segments]
                ranks.append({"rank": r, "domains": int((owner == r).sum()),
                              "phases_ms": {k: round(v, 4) for k, v in ph.items()},
                              "segments_ms": [round(x, 4) for x in seg],
                              "frame_ms": round(ev2[0].elapsed_time(ev2[1]) / args.frames, 4)})
                eng.close()
                rt.close()
            busiest = [max(rk["segments_ms"][k] for rk in ranks) for k in range(len(segments))]
            dev = sum(busiest)
            cm = {m: (comm_ao_ms(world, nu, m) if ao else comm_ms(world, nu, nu // SPP, m))
                  for m in LINK}
            proj = {m: dev + cm[m] for m in LINK}
            run = {"world": world, "partition": mode, "ranks": ranks,
                   "busiest_segments_ms": [round(x, 4) for x in busiest],
                   "device_ms": round(dev, 4),
                   "comm_ms": {m: round(cm[m], 4) for m in LINK},
                   "frame_ms": {m: round(v, 4) for m, v in proj.items()}}
            report["runs"].append(run)
            print("N=%d %-5s (%.0f s): busiest segments %s = %.3f ms device; frame %.3f / %.3f ms"
                  " (cons / opt); per-rank frame ms %s" % (
                      world, mode, time.time() - t0, run["busiest_segments_ms"], dev,
                      proj["cons"], proj["opt"], [rk["frame_ms"] for rk in ranks]), flush=True)
            with open(args.out, "w") as fh:
                json.dump(report, fh, indent=1)


if __name__ == "__main__":
    main()
