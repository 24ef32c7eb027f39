"""Test infrastructure for the in-situ protocol: an oracle-backed stand-in
for the per-rank local work (spray_amd.insitu.GpuLocal), so the exchange,
compositing and partition logic run with world_size > 1 on the CPU ("gloo").
Imports the oracle: tests only, never the product path."""
import os

import numpy as np
import torch

from conftest import BENCH_CAMERA, SCENES, WAVELETS64

MISS_KEY = 0x7FFFFFFFFFFFFFFF
SHADE = [0.0, 500.0, 1000.0, 1.0, 1.0, 1.0, 0.4, 0.4, 0.4, 10.0]
IMG = 128               # the bench camera at 128x128: the whole scene in one tile
TILE = (0, 0, IMG, IMG)
SPP = 2


def rays_tensor(org, d):
    r = np.zeros((len(org), 8), np.float32)
    r[:, 0:3] = org
    r[:, 3] = 0.001
    r[:, 4:7] = d
    r[:, 7] = np.inf
    return torch.from_numpy(r)


def hits_f32(hits):
    return torch.from_numpy(np.ascontiguousarray(hits).view(np.float32).reshape(-1, 12).copy())


class OracleLocal:
    """Per-rank local work on the CPU oracle: a scene holding only this
    rank's meshes and every domain box."""

    def __init__(self, po, owner, rank, desc=WAVELETS64, ply=SCENES):
        mine = {d for d in range(len(owner)) if owner[d] == rank}
        self.po = po
        self.sc, self.domains, _ = po.load_scene(desc, ply, only=mine)
        self.boxes = np.array([d["world_bound"] for d in self.domains], np.float32)
        self.owner = np.asarray(owner)

    def _od(self, rays):
        r = rays.numpy()
        return np.ascontiguousarray(r[:, 0:3]), np.ascontiguousarray(r[:, 4:7])

    def _lists(self, rays):
        o, d = self._od(rays)
        ids, ts, cnt, _ = self.po.domain_query(o, d, self.boxes, len(self.boxes))
        return ids, cnt

    def route(self, rays):
        ids, cnt = self._lists(rays)
        m = np.zeros(len(ids), np.int64)
        for i in range(len(ids)):
            for k in range(cnt[i]):
                m[i] |= 1 << int(self.owner[ids[i, k]])
        return torch.from_numpy(m)

    def intersect_keyed(self, rays):
        o, d = self._od(rays)
        hits, _ = self.sc.intersect(o, d)
        ids, cnt = self._lists(rays)
        keys = np.full(len(hits), MISS_KEY, np.int64)
        h = hits["domain"] >= 0
        dom = hits["domain"][h].astype(np.int64)
        pos = np.argmax(ids[h] == dom[:, None], axis=1).astype(np.int64)
        tb = hits["t"][h].view(np.uint32).astype(np.int64)
        keys[h] = (tb << 32) | (pos << 16) | dom
        return hits_f32(hits), torch.from_numpy(keys)

    def spawn_pt(self, rays, hits, shade):
        o, d = self._od(rays)
        h = np.ascontiguousarray(hits.numpy()).view(self.po.HIT_DTYPE).reshape(-1)
        so, sd, src = self.po.spawn_shadows_pt(o, d, h, shade[0:3], shade[3:6], shade[6:9],
                                               shade[9])
        return rays_tensor(so, sd), torch.from_numpy(src.astype(np.int64))

    def occluded(self, rays):
        o, d = self._od(rays)
        occ, _ = self.sc.occluded(o, d)
        return torch.from_numpy(occ)


def full_reference(po, cam, tile, spp, desc=WAVELETS64, ply=SCENES):
    """Whole-scene oracle on the whole blocking tile, by sample id."""
    org, d, pix, sam = po.eye_rays_insitu(cam, IMG, spp, tile, tile)
    sc, _, _ = po.load_scene(desc, ply)
    hits, _ = sc.intersect(org, d)
    so, sd, src = po.spawn_shadows_pt(org, d, hits, SHADE[0:3], SHADE[3:6], SHADE[6:9],
                                      SHADE[9])
    occ, _ = sc.occluded(so, sd)
    n = len(org)
    hit_by_sam = np.zeros(n, po.HIT_DTYPE)
    hit_by_sam[sam] = hits
    occ_by_sam = np.zeros(n, np.uint8)
    occ_by_sam[sam[src]] = occ
    return hit_by_sam, occ_by_sam, len(so)


def bench_camera(po):
    c = BENCH_CAMERA
    return po.camera_init(c["pos"], c["lookat"], c["up"], c["fov"], IMG, IMG)


# ---------------------------------------------------------------------------
# whole-scene reference of an in-situ frame (multi-bounce, PT / AO)
# ---------------------------------------------------------------------------
def reference_frame(po, sh, bsdfs, cam, img_w, img_h, spp, block, desc=WAVELETS64, ply=SCENES):
    """The frame the in-situ ranks compute together, on the whole-scene
    oracle: eye rays of the whole blocking tile (insitu seeds), per bounce
    closest hit -> shade -> any hit -> film.  Returns (records by
    (bounce, samid) -> (hit bytes, svalid bits, occluded bits), image,
    (radiance rays, shadow rays))."""
    org, d, pix, sam = po.eye_rays_insitu(cam, img_w, spp, block, block)
    sc, _, _ = po.load_scene(desc, ply)
    n = len(org)
    ns = po.shadow_slots(sh)
    w = np.ones((n, 3), np.float32)
    valid = np.ones(n, np.uint8)
    hits = np.zeros(n, po.HIT_DTYPE)
    image = np.zeros(img_w * img_h * 4, np.float32)
    recs = {}
    nrad = nsh = 0
    for b in range(sh.bounces):
        live = np.flatnonzero(valid)
        nrad += len(live)
        if len(live):
            h, _ = sc.intersect(org[live], d[live])
            hits[live] = h
        shaded = live[hits["domain"][live] >= 0]
        so, sd, sw, sv, _ = po.shade(sh, bsdfs, b, org, d, hits, w, valid, pix, sam)
        occ = np.zeros(n * ns, np.uint8)
        sel = np.flatnonzero(sv)
        nsh += len(sel)
        if len(sel):
            occ[sel], _ = sc.occluded(so[sel], sd[sel])
        po.film(image, pix, spp, ns, sw, sv, occ, 1.0 / spp)
        for i in shaded:
            bv = bo = 0
            for k in range(ns):
                if sv[i * ns + k]:
                    bv |= 1 << k
                    if occ[i * ns + k]:
                        bo |= 1 << k
            recs[(b, int(sam[i]))] = (hits[i].tobytes(), bv, bo)
    return recs, image, (nrad, nsh)


def records_dict(recs):
    """Engine / restatement records -> {(bounce, samid): (hit bytes, bits, bits)};
    raises on a duplicate (a sample shaded twice in one bounce)."""
    out = {}
    if isinstance(recs, dict):  # InsituRecords.numpy()
        rows = zip(recs["bounce"], recs["samid"], recs["hits"], recs["svalid"], recs["occluded"])
        rows = [(int(b), int(s), np.ascontiguousarray(h).tobytes(), int(v), int(o))
                for b, s, h, v, o in rows]
    else:
        rows = recs
    for b, s, h, v, o in rows:
        assert (b, s) not in out, ("shaded twice", b, s)
        out[(b, s)] = (h, v, o)
    return out


def compare_records(got, ref):
    """Bit-exact per (bounce, sample): same set of shaded samples, same
    winning hit bytes, same spawned and occluded shadow slots."""
    assert set(got) == set(ref), (len(set(got) - set(ref)), len(set(ref) - set(got)))
    bad = [k for k in ref if got[k] != ref[k]]
    assert not bad, (len(bad), bad[:5])


def insitu_shader(po, kind, bounces, samples, lights=None):
    lights = [(0, 0.0, 500.0, 1000.0, 1.0, 1.0, 1.0)] if lights is None else lights
    return po.shader(kind, bounces, samples, (0.4, 0.4, 0.4), 10.0, lights)
