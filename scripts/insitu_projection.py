"""Per-rank in-situ volumes of the bench frame at N = 1 / 2 / 4 / 8 ranks, and
a frame-time projection from measured N = 1 phase times.

The volumes are exact: the oracle's domain lists of the configs[2] frame
(1024x1024x8 spp eye rays, each rank's horizontal stripe) and of its PT
shadow rays, the engine's Morton partition (spray_rt_insitu_partition), and
the protocol of spray_amd/csrc/insitu.cpp (one copy per (ray, owner rank),
keys back and winners forward at 8 B per copy, shadow rays to their owners,
one occlusion byte back).  The projection then charges:

* every device phase of the N = 1 protocol frame (rocprofv3 kernel trace,
  SPRAY_INSITU_LOCAL=0, profiles/r3i_insitu_proto_trace.txt) scaled by the busiest
  rank's share of that phase's work (copies, visits),
* a per-launch floor (the stream runs ~40 launches per frame, each at least
  ~4.5 us whatever its size) and the frame's two host round trips,
* RCCL: a per-collective latency and a per-GPU all-to-all bandwidth over
  xGMI (ASSUMED figures, command-line flags: no multi-GPU box was available
  to measure them), and the image reduce.

Test infrastructure only (imports the oracle).  Run from the repo root:
    python scripts/insitu_projection.py [--lat-us 30] [--a2a-GBs 300]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from spray_amd import insitu  # noqa: E402

RAD_REC, SHADOW_REC, KEY, OCC = 48, 24, 8, 1  # insitu_kernels.h record bytes


def owners_of(ids, cnt, owner, nranks):
    """[n, nranks] bool: rank r owns a domain on ray i's list."""
    n = len(cnt)
    m = np.zeros((n, nranks), bool)
    for k in range(ids.shape[1]):
        d = ids[:, k]
        ok = (k < cnt) & (d >= 0)
        m[np.nonzero(ok)[0], owner[d[ok]]] = True
    return m


def visits_per_rank(ids, cnt, owner, nranks):
    v = np.zeros(nranks, np.int64)
    for k in range(ids.shape[1]):
        d = ids[:, k]
        ok = (k < cnt) & (d >= 0)
        v += np.bincount(owner[d[ok]], minlength=nranks)
    return v


def volumes(nranks, sc, boxes, cam, threads):
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    owner = insitu.morton_partition(boxes, bound, nranks)
    out = {"ranks": nranks, "domains_per_rank": np.bincount(owner, minlength=nranks).tolist()}
    held = np.zeros(nranks, np.int64)
    sent = np.zeros(nranks, np.int64)       # remote radiance copies sent
    recv = np.zeros(nranks, np.int64)       # radiance copies traced (own + remote)
    visits = np.zeros(nranks, np.int64)
    shadow_held = np.zeros(nranks, np.int64)
    s_sent = np.zeros(nranks, np.int64)
    s_recv = np.zeros(nranks, np.int64)
    s_visits = np.zeros(nranks, np.int64)
    single = 0
    total = 0
    for r in range(nranks):
        st = insitu.horizontal_stripe(nranks, r, (0, 0, bench.W, bench.H))
        if st[2] * st[3] == 0:
            continue
        org, d, _, _ = po.eye_rays_insitu(cam, bench.W, bench.SPP, (0, 0, bench.W, bench.H), st)
        ids, _, cnt, _ = po.domain_query(org, d, boxes, 64)
        om = owners_of(ids, cnt, owner, nranks)
        held[r] += len(org)
        total += len(org)
        ncopy = om.sum(1)
        single += int((ncopy == 1).sum())
        sent[r] += int(ncopy.sum() - om[:, r].sum())
        recv += om.sum(0)
        visits += visits_per_rank(ids, cnt, owner, nranks)
        # the winner (owner of the hit domain) spawns the shadow ray
        hits, _ = sc.intersect(org, d, threads)
        so, sdir, src = po.spawn_shadows_pt(org, d, hits, bench.SHADE[0:3], bench.SHADE[3:6],
                                            bench.SHADE[6:9], bench.SHADE[9])
        win = owner[hits["domain"][src]]
        sids, _, scnt, _ = po.domain_query(so, sdir, boxes, 64)
        sm = owners_of(sids, scnt, owner, nranks)
        for q in range(nranks):
            sel = win == q
            shadow_held[q] += int(sel.sum())
            s_sent[q] += int(sm[sel].sum() - sm[sel, q].sum())
        s_recv += sm.sum(0)
        s_visits += visits_per_rank(sids, scnt, owner, nranks)
    out.update(rays=int(total), single_owner_frac=round(single / max(total, 1), 4),
               held=held.tolist(), rad_copies_traced=recv.tolist(), rad_remote_sent=sent.tolist(),
               ch_visits=visits.tolist(), shadow_held=shadow_held.tolist(),
               shadow_copies_traced=s_recv.tolist(), shadow_remote_sent=s_sent.tolist(),
               ah_visits=s_visits.tolist())
    return out


# N = 1 protocol frame (rocprofv3 kernel trace, SPRAY_INSITU_LOCAL=0, frame 10
# of profiles/r3i_insitu_proto_trace.txt): each launch's device time in
# microseconds and the work it scales with at N ranks.  Every launch keeps a
# floor (the trace's smallest launches, copies of a few bytes included, take
# 4.4-5.2 us).  The two host round trips of the frame (count reads after the
# route, 43 + 112 us of idle GPU at N = 1) stay per frame.
LAUNCHES_N1 = [
    ("route", 143.0, "held"), ("plan", 44.9, "held"), ("count copies", 9.6, None),
    ("gather own radiance", 44.9, "rad_copies_traced"), ("fill", 4.9, None),
    ("keyed closest hit", 380.2, "ch_visits"), ("copy", 7.1, None),
    ("fill keys", 12.6, "held"), ("key min", 15.2, "held"), ("gather rows", 11.1, "held"),
    ("copy", 7.2, None), ("winners", 8.7, "rad_copies_traced"), ("copy", 5.1, None),
    ("shade", 129.6, "rad_copies_traced"), ("fills", 10.2, None),
    ("route shadows", 48.3, "shadow_held"), ("plan shadows", 32.8, "shadow_held"),
    ("count copies", 9.4, None), ("gather own shadows", 26.8, "shadow_copies_traced"),
    ("any hit", 250.7, "ah_visits"), ("copy", 5.2, None), ("occ return", 5.0, "shadow_held"),
    ("film", 22.0, "rad_copies_traced"), ("totals copies", 19.6, None), ("fills", 5.9, None),
]
HOST_GAPS_US = 155.0
FLOOR_US = 4.5


def project(v, v1, lat_us, a2a_gbs, reduce_gbs):
    n = v["ranks"]
    dev = 0.0
    for _, t1, key in LAUNCHES_N1:
        share = max(v[key]) / max(sum(v1[key]), 1) if key else 1.0
        dev += max(t1 * share, FLOOR_US)
    # all-to-all bytes of the busiest sender (remote copies only): radiance
    # records out, keys back, winners forward, shadow records out, occlusion back
    b = [(RAD_REC + 2 * KEY) * v["rad_remote_sent"][r]
         + (SHADOW_REC + OCC) * v["shadow_remote_sent"][r] for r in range(n)]
    a2a_us = max(b) / (a2a_gbs * 1e3) if n > 1 else 0.0
    # 2 count + 5 data all-to-all-v, the totals all-reduce, the image reduce
    ncoll = 9 if n > 1 else 0
    coll_us = ncoll * lat_us
    img = bench.W * bench.H * 16
    red_us = (img * 2 * (n - 1) / n) / (reduce_gbs * 1e3) if n > 1 else 0.0
    total = dev + HOST_GAPS_US + a2a_us + coll_us + red_us
    return {"device_us": round(dev, 1), "host_gaps_us": HOST_GAPS_US,
            "a2a_MB_busiest": round(max(b) / 1e6, 2), "a2a_us": round(a2a_us, 1),
            "collectives": ncoll, "latency_us": round(coll_us, 1),
            "image_reduce_us": round(red_us, 1), "frame_us": round(total, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lat-us", type=float, default=30.0, help="RCCL latency per collective (assumed)")
    ap.add_argument("--a2a-GBs", type=float, default=300.0,
                    help="all-to-all-v bytes/s per GPU over 7 xGMI links (assumed)")
    ap.add_argument("--reduce-GBs", type=float, default=300.0, help="image reduce bus bandwidth (assumed)")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    sc, doms, _ = po.load_scene(bench.SCENE, bench.SCENES)
    boxes = np.array([d["world_bound"] for d in doms], np.float32).reshape(-1, 6)
    cam = po.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"], bench.CAM["fov"],
                         bench.W, bench.H)
    vol = [volumes(n, sc, boxes, cam, a.threads) for n in (1, 2, 4, 8)]
    rows = []
    for v in vol:
        p = project(v, vol[0], a.lat_us, a.a2a_GBs, a.reduce_GBs)
        rows.append({**v, "projection": p})
        print("N=%d domains/rank %s single-owner %.3f | busiest: held %d, traced %d, CH visits %d, "
              "AH visits %d, remote sent %d rad + %d shadow | device %.0f us, a2a %.0f us "
              "(%.1f MB), %d collectives %.0f us, reduce %.0f us -> frame %.0f us"
              % (v["ranks"], v["domains_per_rank"], v["single_owner_frac"], max(v["held"]),
                 max(v["rad_copies_traced"]), max(v["ch_visits"]), max(v["ah_visits"]),
                 max(v["rad_remote_sent"]), max(v["shadow_remote_sent"]), p["device_us"],
                 p["a2a_us"], p["a2a_MB_busiest"], p["collectives"],
                 p["latency_us"], p["image_reduce_us"], p["frame_us"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"assumed": {"lat_us": a.lat_us, "a2a_GBs": a.a2a_GBs,
                                   "reduce_GBs": a.reduce_GBs, "floor_us": FLOOR_US,
                                   "host_gaps_us": HOST_GAPS_US},
                       "launches_n1_us": LAUNCHES_N1, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
