"""Schedule model for DESIGN section 8 item 2 (the verdict's "heavy packets
first" question): per-packet walk costs of the bench frame from the walk
simulator (node + leaf fetches of each 64-ray closest-hit packet), dealt to
the fused launch's 6144 persistent waves as the queues do (4-packet chunks in
band order, greedy: the next chunk to the wave that frees first) against the
same chunks with heavy packets first inside each chunk and against a global
longest-first order.  Prints the makespans in fetch units.

    python scripts/lpt_model.py"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import walk_sim as ws  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

WAVES = 6144
CHUNK = 4


def makespan(costs):
    """greedy list schedule of jobs (in order) on WAVES identical servers"""
    h = [0.0] * WAVES
    heapq.heapify(h)
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h), sum(costs) / WAVES


def main():
    L = ws.lib()
    s, boxes = ws.scene(L)
    cam = po.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0], [0, 1, 0],
                         90.0, 1024, 1024)
    per = []
    for y0 in range(0, 1024, 128):  # the bench's 8 tiles, tile-local seeds
        org, d, _, _ = po.eye_rays_ooc(cam, 1024, 8, (0, y0, 1024, 128))
        org = np.ascontiguousarray(org, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        ids, cnt = ws.lists(org, d, boxes)
        n = len(org)
        out = np.zeros((n // 64, 5), np.int64)
        L.ws_packet(s, 0, ws.p(org), ws.p(d), n, ws.p(ids), ws.p(cnt), ws.MAXH, 64, ws.p(out))
        per.append(out[:, 0] + out[:, 1] + 2)  # + ray load / epilogue round trips
    c = np.concatenate(per).astype(np.float64)
    chunks = c.reshape(-1, CHUNK).sum(1)
    base, lb = makespan(chunks)
    # heavy first inside a chunk: the same chunk sums (a wave walks its chunk's
    # packets back to back), so the same schedule
    lpt, _ = makespan(np.sort(chunks)[::-1])
    pk, _ = makespan(np.sort(c)[::-1])
    print("packets %d, mean cost %.1f fetches, max %.0f" % (len(c), c.mean(), c.max()))
    print("makespan (fetch units): queues in band order %.0f; heavy-first inside chunks %.0f "
          "(identical: a chunk's packets run back to back on one wave); chunks longest-first "
          "%.0f; packets longest-first %.0f; lower bound (mean load) %.0f"
          % (base, base, lpt, pk, lb))
    print("predicted gain of heavy-first inside chunks: 0 %%; of a global longest-first "
          "order: %.1f %% of the walk" % (100.0 * (base - pk) / base))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def proxy_main():
    """the same with the order taken from a cheap proxy (domain visits of the
    packet's walk = the union of its lanes' domain lists)"""
    L = ws.lib()
    s, boxes = ws.scene(L)
    cam = po.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0], [0, 1, 0],
                         90.0, 1024, 1024)
    cs, px = [], []
    for y0 in range(0, 1024, 128):
        org, d, _, _ = po.eye_rays_ooc(cam, 1024, 8, (0, y0, 1024, 128))
        org = np.ascontiguousarray(org, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        ids, cnt = ws.lists(org, d, boxes)
        n = len(org)
        out = np.zeros((n // 64, 5), np.int64)
        L.ws_packet(s, 0, ws.p(org), ws.p(d), n, ws.p(ids), ws.p(cnt), ws.MAXH, 64, ws.p(out))
        cs.append(out[:, 0] + out[:, 1] + 2)
        px.append(out[:, 2])
    c = np.concatenate(cs).astype(np.float64)
    p = np.concatenate(px).astype(np.float64)
    o = np.argsort(-p, kind="stable")
    m, lb = makespan(c[o])
    print("proxy (domain visits) longest-first: makespan %.0f (corr %.2f); band order %.0f; "
          "lower bound %.0f" % (m, np.corrcoef(c, p)[0, 1], makespan(c.reshape(-1, CHUNK).sum(1))[0], lb))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "proxy":
    proxy_main()


def band_main():
    """longest-first by the proxy inside each of the launch's 64 queue bands
    (each XCD keeps its image region), the bands drained side by side"""
    L = ws.lib()
    s, boxes = ws.scene(L)
    cam = po.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0], [0, 1, 0],
                         90.0, 1024, 1024)
    cs, px = [], []
    for y0 in range(0, 1024, 128):
        org, d, _, _ = po.eye_rays_ooc(cam, 1024, 8, (0, y0, 1024, 128))
        org = np.ascontiguousarray(org, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        ids, cnt = ws.lists(org, d, boxes)
        n = len(org)
        out = np.zeros((n // 64, 5), np.int64)
        L.ws_packet(s, 0, ws.p(org), ws.p(d), n, ws.p(ids), ws.p(cnt), ws.MAXH, 64, ws.p(out))
        cs.append(out[:, 0] + out[:, 1] + 2)
        px.append(out[:, 2])
    c = np.concatenate(cs).astype(np.float64)
    p = np.concatenate(px).astype(np.float64)
    nb = 64
    band = np.arange(len(c)) * nb // len(c)
    for name, key in (("band order", np.zeros_like(p)), ("proxy-first in bands", -p),
                      ("cost-first in bands", -c)):
        o = np.lexsort((np.arange(len(c)), key, band))  # within band: by key, stable
        rank = np.empty(len(c), np.int64)
        for b in range(nb):
            sel = o[band[o] == b]
            rank[sel] = np.arange(len(sel))
        seq = np.lexsort((band, rank))  # the bands drained side by side
        cc = c[seq]
        m, lb = makespan(cc.reshape(-1, CHUNK).sum(1) if name == "band order" else cc)
        print("%s: makespan %.0f (lower bound %.0f)" % (name, m, lb))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "band":
    band_main()
