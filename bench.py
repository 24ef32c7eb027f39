"""Headline benchmark: Mrays/s (primary + shadow) on the 64-domain wavelets
scene at 1024x1024, 8 spp (BASELINE.json, configs[1]).

One step = one frame of the hot path over rays already resident in HBM,
as ONE launch (spray_rt_intersect_scene_shadow_pt):
  1. closest hit of the 8,388,608 primary rays against every domain of their
     sorted domain lists (domain query + BVH2 traversal + updateIntersection
     epilogue),
  2. point-light shadow-ray spawn of ooc::ShaderPt in the epilogue of (1),
  3. any hit of the spawned shadow rays: each wave queues its shadow rays in
     LDS and traces them as 64-ray packets.
The same work as two launches (spawn_pt, then select + any hit) is timed
beside it ("unfused").
Primary rays are generated once before timing by the reference's camera /
sampler (ooc::Tracer::genMultiEyes over its 8 blocking tiles of 1024x128).

Multi-GPU (torchrun, one process per GPU): the headline becomes configs[2],
the same frame traced with the domains sharded 64/N per GPU (Morton
partition) and the rays moving to their domains' owners through the
engine's in-situ tracer over RCCL (spray_rt_insitu_*) -- strong scaling of
one frame; barrier + max over ranks around the K timed steps.  Every rank
also times the whole-frame fused step on its own ("replicas", weak scaling).
"ao" is configs[4]: AO-16 on the domain-sharded frame (N > 1) or the
resident frame (N = 1).  At N = 1 the line carries "insitu" (the in-situ
frame through a one-rank RCCL communicator) and "ooc": configs[3], the
frame with a 4-slot HBM cache of domain images streamed from pinned host
memory (spray_rt_ooc_*).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
SCENE = os.path.join(SCENES, "wavelets64.spray")
COUNTS = os.path.join(ROOT, "tests", "golden", "workload_counts.json")
METRIC = "Mrays/s (primary+shadow), 64-domain wavelets, 1024x1024 8spp, 1/2/4/8 GPU"
CAM = dict(pos=[90.172180, 84.141418, 82.480225], lookat=[30.0, 28.649426, 30.0],
           up=[0.0, 1.0, 0.0], fov=90.0)
W = H = 1024
SPP = 8
TILE_H = 128  # ImageScheduleTileList: 1M samples per rank -> 8 tiles of 1024x128
SHADE = [0.0, 500.0, 1000.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4, 10.0]  # light, --blinn
HBM_PEAK_GBS = 8000.0
# SPRAY_BENCH_REHEARSE=1: rehearse the N > 1 code path on a one-GPU box (all
# ranks share GPU 0; torch.distributed "gloo"; in-situ exchanges through the
# engine's host transport instead of RCCL).  Never used for measurements.
REHEARSE = os.environ.get("SPRAY_BENCH_REHEARSE") == "1"  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def tiles():
    return [(0, y, W, TILE_H) for y in range(0, H, TILE_H)]


def algorithmic_bytes(n_rays, nodes, tris, out_bytes):
    """sum_rays (32 + out) + sum_visits (64 N_node + 48 N_tri).
    A work index of the per-ray traversal, not traffic: the packet walk
    fetches a node once per wave, and the scene stays in L2 / MALL."""
    return n_rays * (32 + out_bytes) + 64 * nodes + 48 * tris


# the dominant kernels' names in the rocprofv3 summaries (profiles/)
KERNEL_FUSED = "k_scene<1, false, false, 3, 16, 1>"  # closest hit + PT spawn + shadow any hit
KERNEL_AO = "k_scene<1, true, false, 0, 16, 0>"      # per-lane any hit (AO rays)
KERNEL_AO_GEN = "k_scene<1, true, false, 5, 16, 0>"  # per-lane any hit, AO rays made in the lane
PMC = os.path.join(ROOT, "profiles", "pmc_counters.json")


def scene_bytes(sc, rt):
    """Bytes of the resident scene image a launch has to read at least once:
    per domain the BVH2 nodes (64 B), triangle records (48 B), leaf map (4 B),
    faces (12 B), colors (4 B / vertex) and normals (12 B / vertex)."""
    total = 0
    for d in range(sc.getNumDomains()):
        i = rt.slot_info(sc.load(d))
        v, f, _, _ = sc.domain_mesh(d)
        total += 64 * i["nodes"] + 52 * i["tris"] + 12 * len(f) + 16 * len(v)
    return total


def roofline(kernel, launch_s, compulsory, index_bytes, index_note):
    """The roofline object of one kernel.  The traversal kernels are bound by
    memory latency (dependent node fetches from L2 / MALL), not by HBM
    bandwidth: "bound" says so and "ceilings" carries the counters that show
    it.  achieved / frac stay the HBM-roofline figures: the kernel's
    compulsory HBM bytes per launch -- rays in, results out, the scene image
    once -- over the launch time measured here, against the 8 TB/s peak.
    traffic = the HBM bytes its PMC passes measured
    (profiles/pmc_counters.json), attached only when that profile measured
    this very library build (build id of spray_amd/lib, spray_amd/build.py)."""
    out = {"bound": "latency", "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "achieved": round(compulsory / launch_s / 1e9, 1),
           "frac": round(compulsory / launch_s / 1e9 / HBM_PEAK_GBS, 4),
           "frac_basis": "HBM roofline (secondary): compulsory bytes per launch / launch time / "
                         "8 TB/s; the walk is latency-bound (see ceilings)",
           "algorithmic_bytes_per_launch": compulsory, "avg_launch_ms": round(launch_s * 1e3, 4),
           "kernel": kernel, "traffic": None,
           "index_8d": {"bytes_per_launch": index_bytes,
                        "GB_s": round(index_bytes / launch_s / 1e9, 1), "note": index_note}}
    if os.path.exists(PMC):
        try:
            pm = json.load(open(PMC))
            dv = pm["kernels"][kernel]["derived"]
        except (KeyError, ValueError):
            return out
        from spray_amd import build as spray_build
        bid = spray_build.build_id()
        if not bid or pm.get("build_id") != bid:
            out["traffic_source"] = ("not attached: profiles/pmc_counters.json (%s) measured "
                                     "library build %s, this run loads build %s"
                                     % (pm.get("round"), pm.get("build_id"), bid))
            return out
        t = dv.get("traffic_bytes")
        out["traffic"] = round(t) if t else None
        out["traffic_source"] = ("profiles/pmc_counters.json (%s, library build %s = this run's): "
                                 "2 x FETCH_SIZE + WRITE_SIZE of this kernel, separate --pmc "
                                 "passes" % (pm.get("round"), bid))
        if t:
            out["traffic_frac"] = round(t / launch_s / 1e9 / HBM_PEAK_GBS, 4)
        ceil = {}
        if "l2_request_bytes" in dv:
            ceil["l2"] = {"request_bytes": round(dv["l2_request_bytes"]),
                          "frac": round(dv["l2_request_bytes"] / launch_s / 34.5e12, 4),
                          "peak_GBs": 34500.0, "l2_hit": round(dv.get("l2_hit", 0), 4)}
        for k in ("valu_issue", "salu_issue", "valu_lane_util", "scalar_cache_hit", "ta_busy",
                  "wait_any_frac"):
            if k in dv:
                ceil[k] = round(dv[k], 4)
        out["ceilings"] = ceil
    return out


def cpu_baseline(target_s=10.0):
    """Oracle (C/OpenMP port of the reference path) on a bounded sample of the
    same frame: whole 1024-pixel rows, 8 spp, primary + PT shadow rays."""
    from oracle import pyoracle as po
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    sc, doms, lights = po.load_scene(SCENE, SCENES)
    cam = po.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)

    def run(y0, rows):
        org, d, _, _ = po.eye_rays_ooc(cam, W, SPP, (0, y0, W, rows))
        t0 = time.perf_counter()
        hits, _ = sc.intersect(org, d, threads)
        so, sd, _ = po.spawn_shadows_pt(org, d, hits, SHADE[0:3], SHADE[3:6], SHADE[6:9],
                                        SHADE[9])
        sc.occluded(so, sd, threads)
        return time.perf_counter() - t0, len(org) + len(so)

    # one whole frame (8 blocking tiles), repeated until ~target_s of CPU work
    run(0, 4)  # warm (page-in, thread pool)
    dt, n, reps = 0.0, 0, 0
    while dt < target_s and reps < 64:
        for y in range(0, H, TILE_H):
            a, b = run(y, TILE_H)
            dt += a
            n += b
        reps += 1
    y0, rows = 0, H
    try:  # the reference's Embree path is the baseline only if Embree exists
        import subprocess
        ld = subprocess.run(["ldconfig", "-p"], capture_output=True, text=True, timeout=20).stdout
        hits = [l.strip() for l in ld.splitlines() if "embree" in l.lower()]
        probe = ("ldconfig -p on this host lists %s" % "; ".join(hits)) if hits else \
            "ldconfig -p on this host lists no libembree: the reference's Embree path cannot run, " \
            "the oracle port is the baseline"
    except Exception as e:  # noqa: BLE001
        probe = "ldconfig probe failed: %s" % e
    return {"value": round(n / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads,
            "kind": "port", "embree_probe": probe,
            "sample": "%d x the full 1024x1024x8spp frame (8 tiles of 1024x128): %d "
                      "primary+shadow rays, oracle/oracle.c (C, OpenMP, %d threads), "
                      "%.1f s traversal+spawn" % (reps, n, threads, dt)}


PARTITIONS = {"close": 0, "rr": 1, "view": 2}  # insitu.PARTITION_*
PARTITION_NAMES = {"close": "Morton, close groups (the reference's compiled mode)",
                   "rr": "Morton, round robin", "view": "view-aligned"}


def run_insitu(args, dist, world, rank, local, cam, kind="pt", protocol=False, partition=None):
    """configs[2] (kind "pt": one bounce, the scene's point light) and
    configs[4] (kind "ao": 16 AO rays per hit): one in-situ frame per step,
    the domains sharded by the reference's Morton partition (64/N per GPU;
    --partition: GROUP_CLOSE or ROUND_ROBIN).

    PT at N > 1 is the camera frame (spray_rt_insitu_trace_camera): every
    rank generates in its lanes the eye rays of the pixels its domains may be
    seen through (their screen footprints) and traces them over its domains,
    any-hits the shadow rays of the hit points whose shadow rays may cross
    its domains, and the ranks agree on every ray's winner with MIN
    all-reduces of the t bits and list positions and on every shadow ray's
    occlusion with one SUM all-reduce of bytes -- no ray crosses the wire.
    AO at N > 1 is the camera AO frame: the same keys, the winners' normals
    and colours SUM-all-reduced, every rank any-hits the AO rays entering its
    boxes, occlusion count fields SUM-all-reduced, rank 0 films the whole
    frame.  Both leave the whole image on rank 0 (PT: per-pixel sums reduced
    there).  At N = 1 the camera frame is the eye rays + the all-local fused
    frame.  protocol=True is the stripe protocol
    (spray_rt_insitu_trace): each rank its horizontal stripe of eye rays,
    count-first RCCL all-to-all-v exchanges of rays to their owners, key
    composite, shading at the winner, shadow exchange; the ranks' images are
    composited by one RCCL reduce (HdrImage::composite); its eye rays are made
    once before timing.  RCCL is used at every N, N = 1 included.  Timed like the
    main line (barrier + max over ranks); the per-phase device times come
    from a separate pass with HIP-event timing on."""
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    dev = torch.device("cuda", local)
    boxes, lights = host_parse_scene(SCENE, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    mode = PARTITIONS[partition or args.partition]
    owner = insitu.partition(boxes, bound, world, mode, cam)
    rt = spray_amd.RtContext(local)
    insitu.setup_rank_context(rt, SCENE, SCENES, owner, rank)
    rt.set_bsdfs(host_scene_bsdfs(SCENE))
    rt.set_stream(torch.cuda.current_stream(dev))
    eng = insitu.InsituEngine(rt, world, rank, dist=dist if world > 1 else None,
                              transport="host" if REHEARSE else "rccl")
    replicated = not protocol
    if not replicated:  # the protocol's stripe of eye rays, made before timing
        stripe = insitu.horizontal_stripe(world, rank, (0, 0, W, H))
        n = stripe[2] * stripe[3] * SPP
        rays = torch.empty((max(n, 1), 8), dtype=torch.float32, device=dev)[:n]
        pix = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
        sam = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
        rt.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), stripe, rays, pix, sam)
    if kind == "ao":
        sh = spray_amd.frame.make_shader("ao", 1, 16, ks=SHADE[6:9], shininess=SHADE[9],
                                         lights=lights)
    else:
        sh = spray_amd.frame.make_shader("pt", 1, 1, ks=SHADE[6:9], shininess=SHADE[9],
                                         lights=lights)
    image = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    old_local = os.environ.get("SPRAY_INSITU_LOCAL")
    if protocol:
        os.environ["SPRAY_INSITU_LOCAL"] = "0"  # the whole protocol, even at one rank
    # camera frames leave the whole image on rank 0: no composite
    def frame():
        image.zero_()
        if replicated:
            return eng.trace_camera(sh, cam, W, H, SPP, image)
        t = eng.trace(sh, rays, pix, sam, SPP, image)
        eng.composite(image)
        return t

    try:
        tot = None
        for _ in range(max(args.warmup, 1)):
            tot = frame()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        s0 = eng.stats()
        eng.collective_log()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tot = frame()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        s1 = eng.stats()
        clog = eng.collective_log()
        # per-phase device times (HIP events on the stream), a separate pass
        eng.set_timing(True)
        eng.phase_times()
        nph = 3
        for _ in range(nph):
            frame()
        torch.cuda.synchronize()
        phases = {k: round(v / nph, 4) for k, v in eng.phase_times().items()}
        eng.set_timing(False)
    finally:
        if protocol:
            if old_local is None:
                os.environ.pop("SPRAY_INSITU_LOCAL", None)
            else:
                os.environ["SPRAY_INSITU_LOCAL"] = old_local
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    rays_step = tot[0] + tot[1]
    k = args.steps
    form = ("camera frame: each rank's eye rays generated in the lanes over its domains' "
            "screen footprints, keyed closest hit + shading over its domains, t-bits and "
            "list-position MINs all-reduced, shadow rays from the minimum t over its shadow "
            "footprint, occlusion bytes SUM-all-reduced, per-pixel sums reduced to rank 0"
            if replicated and world > 1 and kind == "pt"
            else "camera AO frame: keys MIN-all-reduced, winners' normals and colours "
            "SUM-all-reduced, every rank any-hits the AO pairs entering its boxes "
            "(compacted), occlusion count fields SUM-all-reduced, film on rank 0"
            if replicated and world > 1
            else "the eye rays of the pixels some box's footprint covers (the others counted as "
                 "misses) + all-local frame" if replicated or (world == 1 and not protocol)
            else "stripe protocol: speculative ray exchange over RCCL all-to-all-v, image "
                 "composite by RCCL reduce")
    out = {"value": round(rays_step * k / el / 1e6, 3), "unit": "Mrays/s",
           "ms_per_step": round(el / k * 1e3, 4), "scaling": "strong",
           "rays_per_step": rays_step, "radiance_rays": tot[0], "shadow_rays": tot[1],
           "rank0_MB_sent_per_step": round((s1["bytes_sent"] - s0["bytes_sent"]) / k / 1e6, 2),
           "rank0_host_count_reads_per_step": (s1["host_count_reads"] -
                                               s0["host_count_reads"]) / k,
           "rank0_collectives_per_step": (s1["collectives"] - s0["collectives"]) / k,
           # one frame's issue sequence (op, count, stream): identical on every
           # rank (RCCL's rule; tests/test_gpu_insitu.py::same_collectives)
           "rank0_collective_log": [list(c) for c in clog[:len(clog) // max(k, 1)]],
           "rank0_phases_ms": phases,
           "image_mean": round(float(image.view(-1, 4)[:, :3].mean()), 6) if rank == 0 else None,
           "partition": partition or args.partition,
           "config": "%s: 64 domains, %d per GPU (%s partition), 1024x1024x8spp, %s, %s"
                     % ("configs[4]" if kind == "ao" else "configs[2]",
                        int(np.bincount(owner, minlength=world)[rank]),
                        PARTITION_NAMES[partition or args.partition],
                        "AO-16 rays per hit" if kind == "ao" else "PT point-light shadows", form)}
    eng.close()
    rt.close()
    return out


def run_image(args, dist, world, rank, local, cam):
    """The image-parallel strong split of configs[1] (the
    reference's ooc mode shards as replicas, only the image is composited;
    spray_rt_insitu_trace_image): every GPU holds all 64 domains (24 MB) and
    traces its row bands of the 1024x1024x8spp frame (eye rays in a pass,
    the fused closest hit + PT spawn + shadow any hit launch, film), then the
    rows go to rank 0 in one RCCL gather (each rank sends 1/N of the image)
    and the totals in one 24-B all-reduce.  Strong scaling: the frame is
    fixed, N GPUs share it.  Timed like the main line (barrier + max over
    ranks); max_rank_frame_ms = the busiest rank's device time outside the
    collectives (HIP events, a separate pass)."""
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene, host_scene_bsdfs
    dev = torch.device("cuda", local)
    boxes, lights = host_parse_scene(SCENE, SCENES)
    rt = spray_amd.RtContext(local)
    insitu.setup_rank_context(rt, SCENE, SCENES, np.full(len(boxes), rank, np.int32), rank)
    rt.set_bsdfs(host_scene_bsdfs(SCENE))
    rt.set_stream(torch.cuda.current_stream(dev))
    eng = insitu.InsituEngine(rt, world, rank, dist=dist if world > 1 else None,
                              transport="host" if REHEARSE else "rccl")
    sh = spray_amd.frame.make_shader("pt", 1, 1, ks=SHADE[6:9], shininess=SHADE[9],
                                     lights=lights)
    image = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    bands = args.image_bands
    if not bands:  # interleaved bands of 16 rows from 4 ranks on (uniform: world x bands | H)
        bands = 1 if world <= 2 else max(1, H // (16 * world))
        while bands > 1 and H % (world * bands):
            bands -= 1
    if world == 1:
        bands = 1

    def frame():
        image.zero_()
        return eng.trace_image(sh, cam, W, H, SPP, image, bands)

    tot = None
    for _ in range(max(args.warmup, 1)):
        tot = frame()
    eng.collective_log()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tot = frame()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    clog = eng.collective_log()
    eng.set_timing(True)
    eng.phase_times()
    nph = 3
    for _ in range(nph):
        frame()
    torch.cuda.synchronize()
    phases = {k: round(v / nph, 4) for k, v in eng.phase_times().items()}
    eng.set_timing(False)
    mx = phases.get("frame", 0.0)
    if world > 1:
        e = torch.tensor([el, mx], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el, mx = float(e[0].item()), float(e[1].item())
    rays_step = tot[0] + tot[1]
    k = args.steps
    out = {"value": round(rays_step * k / el / 1e6, 3), "unit": "Mrays/s",
           "ms_per_step": round(el / k * 1e3, 4), "scaling": "strong",
           "rays_per_step": rays_step, "radiance_rays": tot[0], "shadow_rays": tot[1],
           "max_rank_frame_ms": round(mx, 4), "rank0_phases_ms": phases,
           "bands_per_rank": bands,
           "rank0_collective_log": [list(c) for c in clog[:len(clog) // max(k, 1)]],
           "image_mean": round(float(image.view(-1, 4)[:, :3].mean()), 6) if rank == 0 else None,
           "config": "configs[1] frame split by image rows over %d GPU(s): all 64 domains resident "
                     "per GPU, %d row band(s) per rank, the eye rays of the band pixels some box's "
                     "footprint covers (the others counted as misses) + fused closest hit / PT shadow "
                     "any hit + film per rank, those pixels' RGB gathered to rank 0 over RCCL"
                     % (world, bands)}
    eng.close()
    rt.close()
    return out


def run_ao(args, dist, world, rt, prim, pixid, n_prim, sbytes, nsamples=16):
    """configs[4] workload on one GPU (all 64 domains resident): closest hit
    of the frame, ooc::ShaderAo spawn of 16 rays per hit on the device, any
    hit of all of them (count stays on the device).  The AO any hit is the
    kernel with the most GPU time in the bench; its launch is timed with HIP
    events for its roofline object."""
    import torch
    dev = prim.device
    stream = torch.cuda.current_stream(dev)
    hits = torch.empty(n_prim * 48, dtype=torch.uint8, device=dev)
    fused = bool(args.ao_fused)
    traced = bool(args.ao_traced)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    occ = torch.empty(n_prim * nsamples, dtype=torch.uint8, device=dev)
    src = torch.empty(n_prim * nsamples, dtype=torch.int32, device=dev)
    if fused:  # the (pixel, sample) local hemisphere samples, the hits' frames
        lv = torch.empty(W * H * nsamples * 4, dtype=torch.float32, device=dev)
        rec = torch.empty(n_prim * 16, dtype=torch.float32, device=dev)
    else:
        ao = torch.empty(n_prim * nsamples * 32, dtype=torch.uint8, device=dev)
        order = None if traced else torch.empty(n_prim * nsamples, dtype=torch.int32, device=dev)

    def frame(ev=None):
        rt.set_coherence(rt.RAYS_COHERENT)  # camera rays: packets
        # the spp rays of a pixel share every sample direction (seed
        # pixid * (l + 1)): traced sample-major, they sit on neighbouring
        # lanes -- as (source, sample) pairs (fused), written rays in that
        # order (traced), or permuted through order
        rt.intersect_scene(prim, hits)
        if fused:
            # (source << 5 | sample) pairs; the any-hit lanes make the rays
            rt.spawn_shadows_ao_pairs(prim, hits, pixid, n_prim, nsamples, src, lv, rec, cnt)
        else:
            rt.spawn_shadows_ao(prim, hits, pixid, n_prim, nsamples, ao, src, cnt, order=order,
                                traced=traced)
        rt.set_coherence(rt.RAYS_INCOHERENT)  # hemisphere rays: one walk per lane
        if ev:
            ev[0].record(stream)
        if fused:
            rt.occluded_ao_pairs(n_prim * nsamples, src, rec, lv, nsamples, cnt, occ)
        else:
            rt.occluded_scene_order(ao, n_prim * nsamples, order, cnt, occ)
        if ev:
            ev[1].record(stream)

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        frame(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    n_ao = int(cnt.item())
    ah_s = float(np.mean([e[0].elapsed_time(e[1]) for e in evs])) * 1e-3
    # canonical counts of the AO rays (counting build, outside the timing)
    ctr = torch.zeros(3, dtype=torch.int64, device=dev)
    if fused:
        rt.occluded_ao_pairs(n_prim * nsamples, src, rec, lv, nsamples, cnt, occ, counters=ctr)
    else:
        rt.occluded_scene(ao[:n_ao * 32], occ[:n_ao], counters=ctr)
    torch.cuda.synchronize()
    idx = algorithmic_bytes(n_ao, int(ctr[0]), int(ctr[1]), 4)
    if fused:
        # compulsory bytes: a 4-B (source, sample) pair in and 1 B out per AO
        # ray, the 64-B frame record of each spawning source ray and the
        # 16-B (pixel, sample) local samples once, and the scene once
        n_src = int(torch.unique(src[:n_ao] >> 5).numel())
        comp = n_ao * (4 + 1) + n_src * 64 + W * H * nsamples * 16 + sbytes
    else:
        # 32-B rays (+ 4-B trace order) in, 1 B out, the scene once
        comp = n_ao * (32 + (0 if traced else 4) + 1) + sbytes
    rt.set_coherence(rt.RAYS_ADAPTIVE)
    return {"value": round((n_prim + n_ao) * world * args.steps / el / 1e6, 3),
            "unit": "Mrays/s", "ms_per_step": round(el / args.steps * 1e3, 4),
            "scaling": "weak", "rays_per_step": n_prim + n_ao, "ao_rays": n_ao,
            "canonical_counts": {"nodes": int(ctr[0]), "tris": int(ctr[1]),
                                 "visits": int(ctr[2]), "rays": n_ao},
            "roofline": roofline(KERNEL_AO_GEN if fused else KERNEL_AO, ah_s, comp, idx,
                                 "SURVEY 8(d) per-ray bytes over the AO rays' canonical counts "
                                 "(counting build of this run)"),
            "config": "configs[4] workload on one GPU: 64 domains resident, primary + "
                      "AO-%d rays per hit traced sample-major per pixel%s"
                      % (nsamples, ", spawned as (source, sample) pairs and generated in the "
                                   "any-hit lanes" if fused else "")}


def run_frame(args, dist, world, rt, cam, lights):
    """The whole ooc-mode frame of configs[1] on the device (spray_amd/frame.py):
    the reference's tile schedule (8 tiles of 1024x128 at 1M samples per
    rank), per tile eye rays -> closest hit -> ooc::ShaderPt -> any hit of the
    shadows -> film into the HDR image; frame replicas across ranks."""
    import torch
    import spray_amd
    sh = spray_amd.frame.make_shader("pt", 1, 1, ks=SHADE[6:9], shininess=SHADE[9],
                                     lights=lights)
    rt.set_bsdfs(spray_amd.engine.host_scene_bsdfs(SCENE))
    dev = torch.device("cuda", torch.cuda.current_device())
    image = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    _, (nrad, nsh) = spray_amd.frame.render_frame(rt, sh, cam, W, H, SPP, image=image)
    for _ in range(args.warmup):
        spray_amd.frame.render_frame(rt, sh, cam, W, H, SPP, image=image, stats=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        spray_amd.frame.render_frame(rt, sh, cam, W, H, SPP, image=image, stats=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    rt.frame_stats(reset=True)
    img = image.view(-1, 4)[:, :3]
    return {"value": round((nrad + nsh) * world * args.steps / el / 1e6, 3),
            "unit": "Mrays/s", "ms_per_step": round(el / args.steps * 1e3, 4),
            "scaling": "weak", "rays_per_step": nrad + nsh, "radiance_rays": nrad,
            "shadow_rays": nsh, "image_mean": round(float(img.mean()), 6),
            "config": "configs[1] as a whole frame: 8 tiles of 1024x128x8spp, eye rays + "
                      "closest hit + PT shading + any hit + film on the device, bounces=1 "
                      "(frame replicas x%d)" % world}


def run_ooc(args, rt_main, prim, n_prim, slots=4):
    """configs[3]: the same frame with at most `slots` domains resident in HBM
    (spray_rt_ooc_*): closest hit with the domains streamed through the LRU
    cache in ascending order, PT shadow spawn (compacted), any hit with the
    domains in descending order.  The H2D copies of the domain images are
    inside the timed region."""
    import torch
    import spray_amd
    dev = prim.device
    rt, oc = spray_amd.ooc_scene(SCENE, SCENES, slots, device=dev.index or 0)
    rt.set_stream(torch.cuda.current_stream(dev))
    # the drains walk packets (the context's default coherence)
    hits = torch.empty(n_prim * 48, dtype=torch.uint8, device=dev)
    shadow = torch.empty(n_prim * 32, dtype=torch.uint8, device=dev)
    src = torch.empty(n_prim, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    occ = torch.empty(n_prim, dtype=torch.uint8, device=dev)

    def frame():
        oc.intersect(prim, hits)
        rt.spawn_shadows_pt(prim, hits, n_prim, SHADE, shadow, src, cnt)
        ns = int(cnt.item())
        oc.occluded(shadow[:ns * 32], None, occ[:ns])
        return ns

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    s0 = oc.stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ns = frame()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s1 = oc.stats()
    k = args.steps
    out = {"value": round((n_prim + ns) * k / el / 1e6, 3), "unit": "Mrays/s",
           "ms_per_step": round(el / k * 1e3, 4), "cache_slots": slots,
           "loads_per_step": (s1["loads"] - s0["loads"]) / k,
           "hits_per_step": (s1["hits"] - s0["hits"]) / k,
           "h2d_MB_per_step": round((s1["bytes"] - s0["bytes"]) / k / 1e6, 2),
           "rays_per_step": n_prim + ns,
           "config": "configs[3]: 64 domains, %d-slot HBM LRU cache, images streamed from "
                     "pinned host memory (H2D inside the timed region)" % slots}
    oc.close()
    rt.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--insitu", type=int, default=1,
                    help="also measure configs[2] through the engine's RCCL in-situ tracer "
                         "(always on with more than one rank: it is the headline there)")
    ap.add_argument("--partition", choices=("close", "rr", "view"), default="view",
                    help="in-situ domain partition: close (GROUP_CLOSE_DOMAINS, the reference's "
                         "compiled mode), rr (round robin over the Morton order) or view (the "
                         "view-aligned partition: domains along neighbouring lines of sight "
                         "grouped per rank); at N > 1 the other partitions are timed too")
    ap.add_argument("--image", type=int, default=1,
                    help="also measure the image-parallel strong split (spray_rt_insitu_trace_image)")
    ap.add_argument("--image-bands", type=int, default=0,
                    help="row bands per rank of the image-parallel split (interleaved); 0: 1 up "
                         "to 2 ranks, bands of 16 rows above (profiles/r6_image_bands.txt)")
    ap.add_argument("--ooc", type=int, default=-1,
                    help="also measure configs[3] (default: on one rank)")
    ap.add_argument("--ao", type=int, default=1, help="also measure the configs[4] workload")
    ap.add_argument("--ao-fused", type=int, default=1,
                    help="1: AO rays generated in the any-hit lanes from (source, sample) pairs; "
                         "0: spawned rays written in trace order and read back")
    ap.add_argument("--ao-traced", type=int, default=1,
                    help="AO rays spawned in their trace order (0: compacted + order permutation)")
    ap.add_argument("--frame", type=int, default=1,
                    help="also measure the whole device frame (shading + film)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if REHEARSE:  # every rank on GPU 0, "gloo" + the engine's host transport
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if REHEARSE:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import spray_amd
    sc = spray_amd.Scene(SCENE, SCENES, cache_size=-1, device=local)
    rt = sc.rt
    stream = torch.cuda.Stream()  # events and kernels on one (non-null) stream
    torch.cuda.set_stream(stream)
    rt.set_stream(stream)
    dev = torch.device("cuda", local)

    # ---- resident inputs: the frame's primary rays (8 tiles, tile-local seeds)
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    n_prim = W * H * SPP
    per_tile = W * TILE_H * SPP
    prim = torch.empty(n_prim * 32, dtype=torch.uint8, device=dev)
    pixid = torch.empty(n_prim, dtype=torch.int32, device=dev)
    for k, t in enumerate(tiles()):
        rt.eye_rays_ooc(cam, W, SPP, t, prim[k * per_tile * 32:(k + 1) * per_tile * 32],
                        pixid[k * per_tile:(k + 1) * per_tile])
    hits = torch.empty(n_prim * 48, dtype=torch.uint8, device=dev)
    shadow = torch.empty(n_prim * 32, dtype=torch.uint8, device=dev)
    src = torch.empty(n_prim, dtype=torch.int32, device=dev)
    valid = torch.empty(n_prim, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    nsh = torch.zeros(1, dtype=torch.int32, device=dev)
    occ = torch.empty(n_prim, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    # ---- canonical traversal counts (counting build, outside the timing)
    ctr = torch.zeros(3, dtype=torch.int64, device=dev)
    ctr2 = torch.zeros(3, dtype=torch.int64, device=dev)
    rt.intersect_scene(prim, hits, counters=ctr)
    rt.spawn_shadows_pt(prim, hits, n_prim, SHADE, shadow, src, cnt)
    rt.occluded_scene_devcount(shadow, n_prim, cnt, occ, counters=ctr2)
    torch.cuda.synchronize()
    n_shadow = int(cnt.item())
    gpu_counts = {"primary": {"nodes": int(ctr[0]), "tris": int(ctr[1]), "visits": int(ctr[2]),
                              "rays": n_prim},
                  "shadow": {"nodes": int(ctr2[0]), "tris": int(ctr2[1]), "visits": int(ctr2[2]),
                             "rays": n_shadow}}
    counts_src = "gpu counting build"
    if os.path.exists(COUNTS):
        ref = json.load(open(COUNTS))
        if ref.get("primary") == gpu_counts["primary"] and ref.get("shadow") == gpu_counts["shadow"]:
            counts_src = "oracle fixture tests/golden/workload_counts.json (== gpu counting build)"
        else:
            counts_src = "gpu counting build (MISMATCH vs oracle fixture)"

    rt.set_coherence(rt.RAYS_COHERENT)  # camera rays and point-light shadow rays

    def step(ev=None):
        # closest hit + PT shadow spawn + the shadow rays' any hit, one launch
        if ev:
            ev[0].record(stream)
        rt.intersect_scene_shadow_pt(prim, hits, SHADE, occ, valid, nsh)
        if ev:
            ev[1].record(stream)

    def step_unfused(ev):
        # the same as two launches: closest hit with the fused positional
        # spawn, then select + any hit of the spawned rays
        ev[0].record(stream)
        rt.intersect_scene_spawn_pt(prim, hits, SHADE, shadow, valid, nsh)
        ev[1].record(stream)
        rt.occluded_scene_masked(shadow, valid, occ)
        ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    assert int(nsh.item()) == n_shadow
    fused_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    ms_step = elapsed / args.steps * 1e3
    rays_step = n_prim + n_shadow
    value = rays_step * world * args.steps / elapsed / 1e6

    # the two-launch form of the same step, for comparison (untimed by the
    # step clock above)
    uev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for k in range(args.steps):
        step_unfused(uev[k])
    torch.cuda.synchronize()
    ch_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in uev]))
    ah_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in uev]))

    pc, sh = gpu_counts["primary"], gpu_counts["shadow"]
    ch_bytes = algorithmic_bytes(n_prim, pc["nodes"], pc["tris"], 32)
    ah_bytes = algorithmic_bytes(n_shadow, sh["nodes"], sh["tris"], 4)
    fused_bytes = ch_bytes + ah_bytes
    sbytes = scene_bytes(sc, rt)
    # compulsory bytes of the fused launch: 32-B rays in, 48-B records + the
    # shadow valid / occluded bytes out (the shadow rays never leave the chip),
    # the scene image once
    fused_compulsory = n_prim * (32 + 48 + 1 + 1) + sbytes
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (reference example mesh wavelet.ply x64, deterministic camera rays)",
        "config": {"workload": "wavelets64 1024x1024x8spp PT primary+shadow, all 64 domains "
                               "resident per GPU (configs[1])",
                   "rays_per_step": rays_step, "primary_rays": n_prim, "shadow_rays": n_shadow,
                   "parallelism": "one GPU, the whole frame"},
        "roofline": roofline(KERNEL_FUSED, fused_ms * 1e-3, fused_compulsory, fused_bytes,
                             "SURVEY 8(d) per-ray node/triangle bytes over the canonical counts "
                             "(%s); a work index, not traffic (one node fetch per wave, scene "
                             "in L2/MALL)" % counts_src),
        "kernels_ms": {"intersect_scene_shadow_pt": round(fused_ms, 4),
                       "unfused": {"intersect_scene_spawn_pt": round(ch_ms, 4),
                                   "occluded_scene_masked": round(ah_ms, 4)}},
        "canonical_counts": gpu_counts,
    }
    if args.insitu != 0 or world > 1:
        out["insitu"] = run_insitu(args, dist, world, rank, local, cam)
    if world == 1 and args.insitu != 0:
        # the exchange protocol N > 1 AO frames use, timed at one rank through
        # the one-rank RCCL communicator (SPRAY_INSITU_LOCAL=0), phase split
        out["insitu_protocol"] = run_insitu(args, dist, world, rank, local, cam, protocol=True)
    if world > 1:
        # the same frame under the other partitions (the reference's compiled
        # GROUP_CLOSE among them), each a secondary key
        out["insitu_partitions"] = {
            p: {k: v for k, v in run_insitu(args, dist, world, rank, local, cam,
                                            partition=p).items()
                if k in ("value", "ms_per_step", "rank0_phases_ms")}
            for p in PARTITIONS if p != args.partition}
        # configs[2] is the N > 1 headline: the frame split across the GPUs by
        # domain (strong scaling); the frame replicas stay as a secondary key
        ins = out["insitu"]
        out["replicas"] = {"value": out["value"], "ms_per_step": out["ms_per_step"],
                           "scaling": "weak",
                           "config": "configs[1] frame replicas x%d (every GPU traces the "
                                     "whole frame; no data-path collective)" % world}
        out["value"], out["ms_per_step"] = ins["value"], ins["ms_per_step"]
        out["config"] = {"workload": ins["config"], "rays_per_step": ins["rays_per_step"],
                         "primary_rays": ins["radiance_rays"], "shadow_rays": ins["shadow_rays"],
                         "parallelism": "domain-parallel in-situ x%d (strong), %s partition%s"
                                        % (world, args.partition,
                                           " (NOT the reference's: its compiled GROUP_CLOSE is "
                                           "timed under insitu_partitions.close)"
                                           if args.partition != "close" else
                                           " (the reference's compiled GROUP_CLOSE)")}
    if args.image:
        out["image_parallel"] = run_image(args, dist, world, rank, local, cam)
    if args.ao:
        if world > 1:  # configs[4]: AO-16 on the domain-sharded frame
            out["ao"] = run_insitu(args, dist, world, rank, local, cam, kind="ao")
        else:
            out["ao"] = run_ao(args, dist, world, rt, prim, pixid, n_prim, sbytes)
    if args.frame:
        _, lights = spray_amd.engine.host_parse_scene(SCENE, SCENES)
        out["frame"] = run_frame(args, dist, world, rt, cam, lights)
    if args.ooc == 1 or (args.ooc < 0 and world == 1):
        out["ooc"] = run_ooc(args, rt, prim, n_prim)
    if rank == 0 and world == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    sc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
