"""CPU restatement of the in-situ frame protocol (TEST INFRASTRUCTURE ONLY).

The product protocol lives in the engine (spray_amd/csrc/insitu.cpp) and
needs a GPU.  This module restates its steps over ``torch.distributed`` on
CPU tensors, with each rank's local work done by the oracle, so that the
decomposition itself -- routing, count-first exchanges, the per-copy key
composite (VBuf::compositeTbuf, src/insitu/insitu_vbuf.h:109-129), winner
shading (ShaderPt / ShaderAo, src/insitu/insitu_shader_*.h), shadow exchange
with the occlusion OR at the spawner (compositeObuf), film, and the next
bounce held by the spawner -- is checked against the whole-scene oracle with
world_size > 1 on the CPU ("gloo").  Only tests/ import it.
"""
from __future__ import annotations

import numpy as np

MISS_KEY = 0x7FFFFFFFFFFFFFFF


class Comm:
    """The rank group; world == 1 makes every collective a local copy."""

    def __init__(self, dist=None, group=None):
        self.dist = dist
        self.group = group
        if dist is not None and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1

    def all_to_all(self, out, inp, out_splits, in_splits):
        if self.world == 1:
            out.copy_(inp)
            return out
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
        return out

    def all_reduce_sum(self, t):
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t


class Exchange:
    """One routed exchange: row i of a batch goes to every rank whose bit is
    set in mask[i] (dest-major, ascending i); ``forward`` moves per-row
    payloads to the owners, ``backward`` returns per-copy results."""

    def __init__(self, comm, mask):
        import torch as t
        W = comm.world
        self.comm = comm
        n = mask.shape[0]
        if n:
            bit = t.arange(W, dtype=t.int64).unsqueeze(1)
            sel = ((mask.unsqueeze(0) >> bit) & 1).bool()
            dest, self.idx = sel.nonzero(as_tuple=True)
        else:
            dest = t.zeros(0, dtype=t.int64)
            self.idx = dest
        send = t.bincount(dest, minlength=W).to(t.int64)
        recv = t.empty_like(send)
        comm.all_to_all(recv, send, None, None)  # the count phase
        self.sc, self.rc = send.tolist(), recv.tolist()
        self.n_sent, self.n_recv = sum(self.sc), sum(self.rc)

    def forward(self, payload):
        s = payload.index_select(0, self.idx)
        r = payload.new_empty((self.n_recv,) + tuple(payload.shape[1:]))
        return self.comm.all_to_all(r, s.contiguous(), self.rc, self.sc)

    def backward(self, result):
        r = result.new_empty((self.n_sent,) + tuple(result.shape[1:]))
        return self.comm.all_to_all(r, result.contiguous(), self.sc, self.rc)


def _rays(org, d):
    import torch
    r = np.zeros((len(org), 8), np.float32)
    r[:, 0:3] = org
    r[:, 3] = 0.001
    r[:, 4:7] = d
    r[:, 7] = np.inf
    return torch.from_numpy(r)


def trace_frame(po, local, comm, sh, bsdfs, org, d, pix, sam, spp, image):
    """This rank's eye rays through sh.bounces bounces (insitu.cpp's
    sequence).  local: route / intersect_keyed / occluded on this rank's
    domains (tests/insitu_helpers.OracleLocal).  image: float32 [w*h*4],
    the shaded copies' contributions added.  Returns (records, (group's
    radiance rays, shadow rays)); records: per shaded copy (bounce, samid,
    hit record, shadow valid bits, occluded bits)."""
    import torch as t
    ns = po.shadow_slots(sh)
    scale = 1.0 / spp
    org, d = np.ascontiguousarray(org, np.float32), np.ascontiguousarray(d, np.float32)
    w = np.ones((len(org), 3), np.float32)
    pix, sam = np.asarray(pix, np.int32), np.asarray(sam, np.int32)
    recs = []
    nrad = nsh = 0
    for b in range(sh.bounces):
        n = len(org)
        nrad += n
        rays = _rays(org, d)
        ex = Exchange(comm, local.route(rays))
        r_rays = ex.forward(rays)
        r_w = ex.forward(t.from_numpy(w))
        r_pix = ex.forward(t.from_numpy(pix)).numpy()
        r_sam = ex.forward(t.from_numpy(sam)).numpy()
        hits_t, keys = local.intersect_keyed(r_rays)
        best = t.full((n,), MISS_KEY, dtype=t.int64)
        back = ex.backward(keys)  # every rank takes part, even with nothing sent
        if ex.n_sent:
            best.scatter_reduce_(0, ex.idx, back, "amin")
        win = ((keys == ex.forward(best)) & (keys != MISS_KEY)).numpy()
        m = len(win)
        hits = np.ascontiguousarray(hits_t.numpy()).view(po.HIT_DTYPE).reshape(-1)
        o2 = np.ascontiguousarray(r_rays.numpy()[:, 0:3])
        d2 = np.ascontiguousarray(r_rays.numpy()[:, 4:7])
        w2 = np.ascontiguousarray(r_w.numpy())
        valid = win.astype(np.uint8)
        so, sd, sw, sv, _ = po.shade(sh, bsdfs, b, o2, d2, hits, w2, valid, r_pix, r_sam)
        # shadow rays to the owners of their domains, occlusion OR-ed back
        sel = np.flatnonzero(sv)
        nsh += len(sel)
        occ = np.zeros(m * ns, np.uint8)
        srays = _rays(so[sel], sd[sel])
        sx = Exchange(comm, local.route(srays))
        socc = t.zeros(len(sel), dtype=t.uint8)
        back = sx.backward(local.occluded(sx.forward(srays)))
        if sx.n_sent:
            socc.scatter_reduce_(0, sx.idx, back, "amax")
        occ[sel] = socc.numpy()
        # film of the shaded copies
        lit = np.flatnonzero(sv.astype(bool) & (occ == 0))
        if len(lit):
            img = image.reshape(-1, 4)
            add = (scale * sw[lit].astype(np.float64)).astype(np.float32)
            np.add.at(img[:, :3], r_pix[lit // ns], add)
        # records of the winners
        for i in np.flatnonzero(win):
            bits_v = bits_o = 0
            for k in range(ns):
                if sv[i * ns + k]:
                    bits_v |= 1 << k
                    if occ[i * ns + k]:
                        bits_o |= 1 << k
            recs.append((b, int(r_sam[i]), hits[i].tobytes(), bits_v, bits_o))
        # the spawned radiance rays stay with this rank for the next bounce
        nxt = np.flatnonzero(valid)
        org, d, w = o2[nxt], d2[nxt], w2[nxt]
        pix, sam = r_pix[nxt], r_sam[nxt]
    tot = t.tensor([nrad, nsh], dtype=t.int64)
    comm.all_reduce_sum(tot)
    return recs, (int(tot[0]), int(tot[1]))
