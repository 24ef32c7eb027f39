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
