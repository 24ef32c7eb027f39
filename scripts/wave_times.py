"""Ramp and tail of the persistent scene launches (diagnostic build with
SPRAY_WAVE_TIMES=1, selected through SPRAY_RT_LIB): per wave the 100-MHz
wall-clock at entry, after the LDS staging, when its band queues ran dry,
and at exit, plus its chunk count and XCD.

    SPRAY_RT_LIB=spray_amd/lib/diag/libspray_rt_wavetimes.so python scripts/wave_times.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import spray_amd  # noqa: E402
from spray_amd import _native  # noqa: E402


def stamps(lib, nwaves):
    buf = np.zeros(5 * nwaves, dtype=np.uint64)
    f = lib.spray_rt_diag_wave_times
    f.argtypes = [C.c_void_p, C.c_size_t]
    assert f(buf.ctypes.data, buf.size) == 0
    w = buf.reshape(nwaves, 5)
    return w[w[:, 3] != 0]


def report(name, w):
    t0 = w[:, 0].min()
    rel = (w[:, :4] - t0).astype(np.float64) * 0.01  # us
    end = rel[:, 3].max()
    life = rel[:, 3] - rel[:, 0]
    q = lambda a: "p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f" % tuple(
        np.percentile(a, [0, 10, 50, 90, 100]))
    print("== %s: %d waves, launch span %.1f us, mean life / span %.3f" % (
        name, len(w), end, life.mean() / end))
    print("  entry     ", q(rel[:, 0]))
    print("  staged    ", q(rel[:, 1] - rel[:, 0]), "(after entry)")
    print("  queues dry", q(rel[:, 2]))
    print("  exit      ", q(rel[:, 3]))
    print("  drain-to-exit (shadow flush)", q(rel[:, 3] - rel[:, 2]))
    ch = (w[:, 4] & 0xFFFFFFFF).astype(np.int64)
    xcd = (w[:, 4] >> 32).astype(np.int64)
    print("  chunks/wave", q(ch))
    for x in range(8):
        s = xcd == x
        if s.any():
            print("   xcd %d: waves %d chunks %d exit p50 %.1f max %.1f dry p50 %.1f" % (
                x, s.sum(), ch[s].sum(), np.median(rel[s, 3]), rel[s, 3].max(),
                np.median(rel[s, 2])))


def packet_log(lib, name, run):
    """Per-packet event log of one launch: durations by kind, and what the
    last waves to exit were doing."""
    if not hasattr(lib, "spray_rt_diag_packet_log"):
        return
    f = lib.spray_rt_diag_packet_log
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    assert f(None, None, 1) == 0
    run()
    torch.cuda.synchronize()
    log = np.zeros(2 * 6144 * 256, dtype=np.uint64)
    cnt = np.zeros(6144, dtype=np.uint32)
    assert f(log.ctypes.data, cnt.ctypes.data, 0) == 0
    log = log.reshape(6144, 256, 2)
    ev = []
    for w in range(6144):
        for k in range(int(cnt[w])):
            a, b = int(log[w, k, 0]), int(log[w, k, 1])
            ev.append((w, a >> 24, a & 0xFFFFFF, b >> 40, b & ((1 << 40) - 1)))
    ev = np.array(ev, dtype=np.int64)
    t0 = ev[:, 1].min()
    st = (ev[:, 1] - t0) * 0.01
    du = ev[:, 2] * 0.01
    en = st + du
    print("== packet log %s: %d events" % (name, len(ev)))
    for kind, kn in ((0, "primary"), (1, "shadow"), (2, "flush")):
        s_ = ev[:, 3] == kind
        if s_.any():
            print("  %-8s n %6d  dur us p50 %.1f p90 %.1f p99 %.1f max %.1f  total %.0f" % (
                kn, s_.sum(), *np.percentile(du[s_], [50, 90, 99]), du[s_].max(), du[s_].sum()))
    # busy waves over time
    span = en.max()
    for q in (0.5, 0.6, 0.7, 0.8, 0.9, 0.95):
        t = q * span
        busy = len(np.unique(ev[(st <= t) & (en > t), 0]))
        print("  at %.0f us (%.0f%%): %d waves busy" % (t, q * 100, busy))
    last = np.argsort(-en)[:12]
    for e in last:
        print("   late: wave %d kind %d start %.1f dur %.1f index %d" % (
            ev[e, 0], ev[e, 3], st[e], du[e], ev[e, 4]))
    # primary packet duration by packet index band (the image rows)
    s_ = ev[:, 3] == 0
    idx = ev[s_, 4]
    nb = 16
    band = (idx * nb) // (idx.max() + 1)
    print("  primary mean dur by 1/16 of the frame:",
          " ".join("%.1f" % du[s_][band == b].mean() if (band == b).any() else "-"
                   for b in range(nb)))


def main():
    lib = _native.lib()
    sc = spray_amd.Scene(bench.SCENE, bench.SCENES)
    rt = sc.rt
    rt.set_stream(torch.cuda.current_stream())
    rt.set_coherence(rt.RAYS_COHERENT)
    cam = spray_amd.camera_init(bench.CAM["pos"], bench.CAM["lookat"], bench.CAM["up"],
                                bench.CAM["fov"], bench.W, bench.H)
    n = bench.W * bench.H * bench.SPP
    per = bench.W * bench.TILE_H * bench.SPP
    prim = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    for k, t in enumerate(bench.tiles()):
        rt.eye_rays_ooc(cam, bench.W, bench.SPP, t, prim[k * per * 32:(k + 1) * per * 32], None)
    hits = torch.empty(n * 48, dtype=torch.uint8, device="cuda")
    sh = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    valid = torch.empty(n, dtype=torch.uint8, device="cuda")
    occ = torch.empty(n, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(3):
        rt.intersect_scene_shadow_pt(prim, hits, bench.SHADE, occ, valid, cnt)
    torch.cuda.synchronize()
    report("fused CH + shadow (intersect_scene_shadow_pt)", stamps(lib, 16384))
    packet_log(lib, "fused", lambda: rt.intersect_scene_shadow_pt(prim, hits, bench.SHADE, occ,
                                                                  valid, cnt))
    for _ in range(3):
        rt.intersect_scene_spawn_pt(prim, hits, bench.SHADE, sh, valid, cnt)
    torch.cuda.synchronize()
    report("CH + spawn (intersect_scene_spawn_pt)", stamps(lib, 16384))


if __name__ == "__main__":
    main()
