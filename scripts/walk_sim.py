"""CPU model of the GPU walks' wave-level execution (scripts/walk_sim.cpp):
wave loop iterations (dependent fetch round trips) and SIMD lane utilisation
of the per-lane AO any hit and of the packet walks, on the bench frame's
rays -- for weighing traversal changes before spending GPU time.

    python scripts/walk_sim.py [ao|packet|all] [tiles]

Research tool: builds scripts/_build/libwalksim.so from walk_sim.cpp and the
engine's host BVH builder, takes rays and domain lists from the oracle."""
import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
SCENE = os.path.join(SCENES, "wavelets64.spray")
LIB = os.path.join(ROOT, "scripts", "_build", "libwalksim.so")
W = H = 1024
SPP = 8
SHADE = [0.0, 500.0, 1000.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4, 10.0]
MAXH = 16


def lib():
    src = [os.path.join(ROOT, "scripts", "walk_sim.cpp"),
           os.path.join(ROOT, "spray_amd", "csrc", "bvh_build.cpp")]
    if not os.path.exists(LIB) or any(os.path.getmtime(s) > os.path.getmtime(LIB) for s in src):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", "-shared", "-fPIC",
                        "-I" + os.path.join(ROOT, "spray_amd", "csrc"), *src, "-o", LIB],
                       check=True)
    L = C.CDLL(LIB)
    L.ws_scene_create.restype = C.c_void_p
    L.ws_scene_create.argtypes = [C.c_int]
    L.ws_set_domain.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p,
                                C.c_size_t, C.c_void_p]
    L.ws_lane_ah.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                             C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    L.ws_set_mode.argtypes = [C.c_int]
    L.ws_lane_ah2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                              C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    L.ws_packet.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                            C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    return L


def p(a):
    return a.ctypes.data


def scene(L):
    doms, _ = po.parse_spray(SCENE, SCENES)
    s = L.ws_scene_create(len(doms))
    boxes = []
    cache = {}
    for d in doms:
        key = (d["file"], d["transform"].tobytes())
        if key not in cache:
            cache[key] = po.load_domain_mesh(d)
        v, f, _, _ = cache[key]
        b = np.ascontiguousarray(d["world_bound"], np.float32)
        L.ws_set_domain(s, d["id"], p(v), len(v), p(f), len(f), p(b))
        boxes.append(b)
    return s, np.array(boxes, np.float32)


def lists(org, d, boxes):
    ids, _, cnt, over = po.domain_query(org, d, boxes, MAXH)
    assert over == 0 or True
    return np.ascontiguousarray(ids), np.ascontiguousarray(cnt)


def ao_trace_order(src, nsrc_per_block=8):
    """The sample-major trace order of the AO spawn: within each aligned
    block of 8 source rays, (k-th spawned sample, ray) ascending (k stands
    for the sample id; all 16 samples of a hit spawn in the bench frame but
    for unlit colour channels)."""
    first = np.searchsorted(src, src)
    k = np.arange(len(src)) - first
    key = (src // nsrc_per_block) * 4096 + k * nsrc_per_block + src % nsrc_per_block
    return np.argsort(key, kind="stable")


def run_ao(L, s, boxes, org, d, hits, pix):
    for mode in (0, 1):
        L.ws_set_mode(mode)
        print("AO mode: %s" % ("per-lane leaf tests", "leaf triangles spread over the wave")[mode])
        _run_ao(L, s, boxes, org, d, hits, pix)


def ao_rays(org, d, hits, pix, boxes):
    so, sd, src = po.spawn_shadows_ao(org, d, pix, hits, 16)
    o = ao_trace_order(src)
    so, sd = np.ascontiguousarray(so[o]), np.ascontiguousarray(sd[o])
    ids, cnt = lists(so, sd, boxes)
    return so, sd, ids, cnt


def run_ao2(L, s, boxes, org, d, hits, pix):
    so, sd, ids, cnt = ao_rays(org, d, hits, pix, boxes)
    n = len(so)
    for chunk, refill in ((64, 0), (1024, 0), (1024, 1), (1024, 8), (1024, 16), (1024, 32),
                          (1024, 48)):
        nw = (n + chunk - 1) // chunk
        out = np.zeros((nw, 8), np.int64)
        occ = np.zeros(n, np.uint8)
        t0 = time.time()
        L.ws_lane_ah2(s, p(so), p(sd), n, p(ids), p(cnt), MAXH, chunk, refill, p(out), p(occ))
        tot = out.sum(0)
        w64 = n / 64.0
        print("AO state machine, chunk %d refill %d (%.1f s): occluded %.3f; per 64 rays: node "
              "iters %.1f (util %.3f), tri iters %.1f spread (util %.3f) / %.1f per lane, refill "
              "rounds %.1f (%.1f rays)"
              % (chunk, refill, time.time() - t0, occ.mean(), tot[0] / w64,
                 tot[1] / (64.0 * tot[0]), tot[2] / w64, tot[3] / (64.0 * max(tot[2], 1)),
                 tot[6] / w64, tot[4] / w64, tot[5] / w64))


def _run_ao(L, s, boxes, org, d, hits, pix):
    so, sd, ids, cnt = ao_rays(org, d, hits, pix, boxes)
    n = len(so)
    nw = (n + 63) // 64
    out = np.zeros((nw, 6), np.int64)
    occ = np.zeros(n, np.uint8)
    t0 = time.time()
    L.ws_lane_ah(s, p(so), p(sd), n, p(ids), p(cnt), MAXH, p(out), p(occ))
    tot = out.sum(0)
    print("AO rays %d (%.1f s): occluded %.3f, domains/ray %.2f" % (n, time.time() - t0,
                                                                   occ.mean(), cnt.mean()))
    print("  node loop: %d wave iterations, lane util %.3f (%.1f lane steps/ray)"
          % (tot[0], tot[1] / (64.0 * tot[0]), tot[1] / n))
    print("  leaf loop: %d wave tri iterations, lane util %.3f (%.1f tri tests/ray)"
          % (tot[2], tot[3] / (64.0 * tot[2]), tot[3] / n))
    print("  per wave: %.1f node iters, %.1f tri iters, %.2f domain rounds"
          % (tot[0] / nw, tot[2] / nw, tot[4] / nw))
    # ideal repacking bound: lane steps / 64 instead of wave iterations
    print("  ideal refill (lane steps / 64): node %.2fx fewer iterations, tri %.2fx"
          % (tot[0] * 64.0 / tot[1], tot[2] * 64.0 / tot[3]))
    return out, occ


def run_packet(L, s, boxes, org, d, any_, label, packets=(64, 128)):
    ids, cnt = lists(org, d, boxes)
    n = len(org)
    for pk in packets:
        nw = (n + pk - 1) // pk
        out = np.zeros((nw, 5), np.int64)
        t0 = time.time()
        L.ws_packet(s, int(any_), p(org), p(d), n, p(ids), p(cnt), MAXH, pk, p(out))
        tot = out.sum(0)
        print("%s packet %d: %d rays (%.1f s): node fetches %d (%.2f/ray, %.1f/wave), leaf "
              "fetches %d (%.2f/ray), domain visits/wave %.2f, slab lane util %.3f"
              % (label, pk, n, time.time() - t0, tot[0], tot[0] / n, tot[0] / nw, tot[1],
                 tot[1] / n, tot[2] / nw, tot[3] / (2.0 * pk * tot[0])))


def morton3(x, y, z, bits=10):
    """interleaved bits of three coordinates in [0, 1)"""
    out = np.zeros(len(x), np.uint64)
    q = [np.clip((c * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1).astype(np.uint64)
         for c in (x, y, z)]
    for b in range(bits):
        for k in range(3):
            out |= ((q[k] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + k)
    return out


def run_ooc_queues(L, s, boxes, org, d, any_, label):
    """The out-of-core drains' waves: 64 consecutive entries of ONE domain's
    queue walk that domain as a packet -- queues in ascending ray order (the
    shipped scatter) against queues sorted by the Morton code of the ray's
    entry point into the domain box."""
    ids, cnt = lists(org, d, boxes)
    n = len(org)
    rows = np.repeat(np.arange(n), cnt)
    k = np.arange(len(rows)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    dom = ids[rows, k]
    for sort in ("ascending", "entry-morton"):
        if sort == "ascending":
            o = np.lexsort((rows, dom))
        else:
            lo, hi = boxes[dom, :3], boxes[dom, 3:]
            inv = 1.0 / np.where(np.abs(d[rows]) < 1e-20, 1e-20, d[rows])
            t0 = np.maximum(np.max(np.minimum((lo - org[rows]) * inv, (hi - org[rows]) * inv), 1),
                            0.0)
            pt = org[rows] + t0[:, None] * d[rows]
            u = np.clip((pt - lo) / (hi - lo), 0, 0.999)
            key = morton3(u[:, 0], u[:, 1], u[:, 2])
            o = np.lexsort((rows, key, dom))
        r, dd = rows[o], dom[o]
        po = np.ascontiguousarray(org[r])
        pd = np.ascontiguousarray(d[r])
        pid = np.full((len(r), MAXH), -1, np.int32)
        pid[:, 0] = dd
        pc = np.ones(len(r), np.int32)
        # waves never straddle two queues: pad each queue to a multiple of 64
        starts = np.flatnonzero(np.r_[True, dd[1:] != dd[:-1]])
        lens = np.diff(np.r_[starts, len(dd)])
        tot_nodes = tot_waves = 0
        for a, ln in zip(starts, lens):
            nw = (ln + 63) // 64
            out = np.zeros((nw, 5), np.int64)
            L.ws_packet(s, int(any_), p(po[a:a + ln]), p(pd[a:a + ln]), int(ln),
                        p(np.ascontiguousarray(pid[a:a + ln])), p(pc[a:a + ln]), MAXH, 64, p(out))
            tot_nodes += out[:, 0].sum()
            tot_waves += nw
        print("%s OOC queue waves (%s): %d pairs, %d waves, node fetches %.1f/wave (%.2f/pair)"
              % (label, sort, len(r), tot_waves, tot_nodes / tot_waves, tot_nodes / len(r)))


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    tiles = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [3]
    L = lib()
    s, boxes = scene(L)
    sc, _, _ = po.load_scene(SCENE, SCENES)
    cam = po.camera_init([90.172180, 84.141418, 82.480225], [30.0, 28.649426, 30.0],
                         [0.0, 1.0, 0.0], 90.0, W, H)
    for t in tiles:
        org, d, pix, _ = po.eye_rays_ooc(cam, W, SPP, (0, 128 * t, W, 128))
        hits, _ = sc.intersect(org, d)
        print("tile %d: %d primary rays, hit %.3f" % (t, len(org), (hits["domain"] >= 0).mean()))
        if what in ("packet", "all"):
            run_packet(L, s, boxes, org, d, False, "primary CH")
            so, sd, src = po.spawn_shadows_pt(org, d, hits, SHADE[0:3], SHADE[3:6], SHADE[6:9],
                                              SHADE[9])
            run_packet(L, s, boxes, np.ascontiguousarray(so), np.ascontiguousarray(sd), True,
                       "shadow AH")
        if what in ("ooc", "all"):
            so, sd, src = po.spawn_shadows_pt(org, d, hits, SHADE[0:3], SHADE[3:6], SHADE[6:9],
                                              SHADE[9])
            run_ooc_queues(L, s, boxes, np.ascontiguousarray(so), np.ascontiguousarray(sd), True,
                           "shadow AH")
            run_ooc_queues(L, s, boxes, org, d, False, "primary CH")
        if what in ("ao", "all"):
            run_ao(L, s, boxes, org, d, hits, pix)
        if what in ("ao2", "all"):
            run_ao2(L, s, boxes, org, d, hits, pix)


if __name__ == "__main__":
    main()
