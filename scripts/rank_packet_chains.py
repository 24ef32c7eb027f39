"""Latency model of a rank's packet walks in the replicated in-situ frame
(research tool; CPU, walk_sim.cpp): per rank of an N-way domain partition,
the dependent fetch chain of every 64-ray packet of its own eye rays
(node + leaf fetch round trips of scene_ray_packet over the rank's domains)
-- whole packets vs packets split by domain -- and of its shadow rays.  The
longest chain bounds a launch from below when the rank has fewer packets
than the GPU has wave slots.

    python scripts/rank_packet_chains.py [world] [close|rr]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import walk_sim as ws  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

PK = 64


def restrict(ids, cnt, keep):
    """domain lists with only the domains in `keep` (order kept)"""
    n, m = ids.shape
    out = np.full_like(ids, -1)
    oc = np.zeros_like(cnt)
    valid = np.arange(m)[None, :] < cnt[:, None]
    k = valid & np.isin(ids, keep)
    # stable compaction of each row
    pos = np.cumsum(k, axis=1) - 1
    r, c = np.nonzero(k)
    out[r, pos[r, c]] = ids[r, c]
    oc[:] = k.sum(1)
    return np.ascontiguousarray(out), np.ascontiguousarray(oc.astype(cnt.dtype))


def chains(L, s, any_, org, d, ids, cnt):
    n = len(org)
    nw = (n + PK - 1) // PK
    out = np.zeros((nw, 5), np.int64)
    L.ws_packet(s, int(any_), ws.p(org), ws.p(d), n, ws.p(ids), ws.p(cnt), ws.MAXH, PK, ws.p(out))
    return out[:, 0] + out[:, 1], out[:, 2]


def project(cam, X):
    """pixel coordinates (x, y) and depth factor of points X under the
    camera of k_eye_rays_insitu: dir ~ A + U u + V v - E, u = x / W"""
    E, A, U, V = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    M = np.stack([A - E, U, V], axis=1).astype(np.float64)
    abc = np.linalg.solve(M, (X - E).T.astype(np.float64)).T
    lam = abc[:, 0]
    return abc[:, 1] / lam * cam[12], abc[:, 2] / lam * cam[13], lam


def view_partition(cam, boxes, world):
    """domains grouped by screen position: recursive median splits of the
    projected box centres (x, then y, ...) into `world` groups of equal
    count -- each group a set of domains along neighbouring lines of sight"""
    c = (boxes[:, :3] + boxes[:, 3:]) * 0.5
    x, y, _ = project(cam, c)
    owner = np.zeros(len(boxes), np.int64)

    def split(ids, ranks, axis):
        if len(ranks) == 1:
            owner[ids] = ranks[0]
            return
        key = x[ids] if axis == 0 else y[ids]
        o = ids[np.lexsort((ids, key))]
        h = len(ranks) // 2
        cut = len(ids) * h // len(ranks)
        split(o[:cut], ranks[:h], 1 - axis)
        split(o[cut:], ranks[h:], 1 - axis)

    split(np.arange(len(boxes)), list(range(world)), 0)
    return owner


def summary(ch, label):
    a = ch[ch > 0]
    if not len(a):
        return "%s: none" % label
    return ("%s: %d packets, work %d, chain max %d p99 %d p90 %d mean %.1f"
            % (label, len(a), a.sum(), a.max(), np.percentile(a, 99), np.percentile(a, 90),
               a.mean()))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    mode = sys.argv[2] if len(sys.argv) > 2 else "close"
    from spray_amd import insitu
    L = ws.lib()
    s, boxes = ws.scene(L)
    sc, _, _ = po.load_scene(ws.SCENE, ws.SCENES)
    cam = po.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0],
                         [0.0, 1.0, 0.0], 90.0, ws.W, ws.H)
    t0 = time.time()
    org, d, pix, sam = po.eye_rays_insitu(cam, ws.W, ws.SPP, (0, 0, ws.W, ws.H),
                                          (0, 0, ws.W, ws.H))
    org = np.ascontiguousarray(org)
    d = np.ascontiguousarray(d)
    hits, _ = sc.intersect(org, d)
    so, sd, src = po.spawn_shadows_pt(org, d, hits, ws.SHADE[0:3], ws.SHADE[3:6], ws.SHADE[6:9],
                                      ws.SHADE[9])
    so = np.ascontiguousarray(so)
    sd = np.ascontiguousarray(sd)
    ids, cnt = ws.lists(org, d, boxes)
    sids, scnt = ws.lists(so, sd, boxes)
    print("frame: %d eye rays, %d shadow rays (%.1f s)" % (len(org), len(so), time.time() - t0))
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    if mode == "view":
        owner = view_partition(cam, boxes, world)
    else:
        owner = insitu.morton_partition(boxes, bound, world,
                                        insitu.PARTITION_ROUND_ROBIN if mode == "rr"
                                        else insitu.PARTITION_GROUP_CLOSE)
    print("owner", owner.tolist())
    ch, _ = chains(L, s, False, org, d, ids, cnt)
    print(summary(ch, "N=1 eye"))
    ch, _ = chains(L, s, True, so, sd, sids, scnt)
    print(summary(ch, "N=1 shadow"))
    for r in range(world):
        mine = np.flatnonzero(owner == r)
        i2, c2 = restrict(ids, cnt, mine)
        ch, _ = chains(L, s, False, org, d, i2, c2)
        line = [summary(ch, "rank %d eye whole" % r)]
        mx = np.zeros(len(ch), np.int64)
        tot = 0
        for dm in mine:
            i3, c3 = restrict(ids, cnt, [dm])
            c1, _ = chains(L, s, False, org, d, i3, c3)
            mx = np.maximum(mx, c1)
            tot += c1.sum()
        line.append("split by domain: work %d, chain max %d p99 %d"
                    % (tot, mx.max(), np.percentile(mx[mx > 0], 99)))
        i4, c4 = restrict(sids, scnt, mine)
        ch, _ = chains(L, s, True, so, sd, i4, c4)
        line.append(summary(ch, "shadow"))
        print("\n   ".join(line), flush=True)


if __name__ == "__main__":
    main()
