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

    def all_reduce_min(self, t):
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
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


def _shadow_from_t(org, d, t, lp):
    """RTCRayUtil::hitPosition + PointLight::sample (rays.h:436-441,
    light.h:47-53) in float32, glm's operation order: the shadow ray of a hit
    from (org, dir, t) alone."""
    f = np.float32
    pos = (d * t[:, None]).astype(f) + org
    lv = (np.asarray(lp, f)[None, :] - pos).astype(f)
    dot = ((lv[:, 0] * lv[:, 0] + lv[:, 1] * lv[:, 1]).astype(f) + lv[:, 2] * lv[:, 2]).astype(f)
    inv = (f(1.0) / np.sqrt(dot)).astype(f)
    return pos.astype(f), (lv * inv[:, None]).astype(f)


def trace_frame_replicated(po, local, comm, sh, bsdfs, org, d, pix, sam, spp, image):
    """The replicated-ray frame of insitu.cpp (trace_replicated): org / d /
    pix / sam are EVERY eye ray of the frame, the same on every rank.  Each
    rank: owner-rank masks of all rays; C = the rays with a non-empty domain
    list; keyed closest hit of the rays of C with a domain of its own over
    its own domains; MIN all-reduce of the keys over C; the point-light
    shadow ray of every hit from (org, dir, t) traced over its own domains;
    the winner shades (ooc::ShaderPt); SUM all-reduce of the occlusion bytes;
    film of the rays it won, summed on rank 0 (the whole image there).  PT,
    one bounce, one point light.  Returns
    (records, (group's radiance rays, shadow rays))."""
    import torch as t
    assert sh.bounces == 1
    if sh.shader == po.SHADER_AO:
        return _frame_replicated_ao(po, local, comm, sh, bsdfs, org, d, pix, sam, spp, image)
    assert sh.nlights == 1
    org, d = np.ascontiguousarray(org, np.float32), np.ascontiguousarray(d, np.float32)
    pix, sam = np.asarray(pix, np.int32), np.asarray(sam, np.int32)
    n = len(org)
    rays = _rays(org, d)
    mask = local.route(rays).numpy()
    C = np.flatnonzero(mask != 0)
    mine = ((mask[C] >> comm.rank) & 1).astype(bool)
    keys_c = np.full(len(C), MISS_KEY, np.int64)
    hits_c = np.zeros(len(C), po.HIT_DTYPE)
    if mine.any():
        h, k = local.intersect_keyed(rays[C[mine]])
        keys_c[mine] = k.numpy()
        hits_c[mine] = np.ascontiguousarray(h.numpy()).view(po.HIT_DTYPE).reshape(-1)
    own = keys_c.copy()
    best = comm.all_reduce_min(t.from_numpy(keys_c.copy())).numpy()
    hit = best != MISS_KEY
    win = hit & (own == best)
    # every hit's shadow ray, traced over this rank's domains
    tt = (best[hit] >> 32).astype(np.uint32).view(np.float32)
    lp = [sh.lights[0].pos[k] for k in range(3)]
    so, sd = _shadow_from_t(org[C[hit]], d[C[hit]], tt, lp)
    occ = np.zeros(len(C), np.int32)
    if len(so):
        occ[hit] = local.occluded(_rays(so, sd)).numpy()
    # the winners shade: spawn rule and light weight (ooc::ShaderPt)
    oc, dc = np.ascontiguousarray(org[C]), np.ascontiguousarray(d[C])
    w = np.ones((len(C), 3), np.float32)
    valid = win.astype(np.uint8)
    so2, sd2, sw, sv, _ = po.shade(sh, bsdfs, 0, oc, dc, hits_c, w, valid, pix[C], sam[C])
    sv = sv.astype(bool) & win
    # the winner's own shadow ray is the one every rank built from t
    so_c = np.zeros((len(C), 3), np.float32)
    sd_c = np.zeros((len(C), 3), np.float32)
    so_c[hit], sd_c[hit] = so, sd
    assert so2[sv].tobytes() == so_c[sv].tobytes() and sd2[sv].tobytes() == sd_c[sv].tobytes()
    tail = t.tensor([n if comm.rank == 0 else 0, int(sv.sum())], dtype=t.int64)
    occ_t = comm.all_reduce_sum(t.from_numpy(occ))
    comm.all_reduce_sum(tail)
    occ = occ_t.numpy() > 0
    # film of the won rays into per-pixel sums, reduced to rank 0
    lit = np.flatnonzero(sv & ~occ)
    acc = np.zeros((len(image) // 4, 3), np.float32)
    if len(lit):
        add = ((1.0 / spp) * sw[lit].astype(np.float64)).astype(np.float32)
        np.add.at(acc, pix[C[lit]], add)
    acc = comm.all_reduce_sum(t.from_numpy(acc)).numpy()
    if comm.rank == 0:
        image.reshape(-1, 4)[:, :3] += acc
    recs = [(0, int(sam[C[j]]), hits_c[j].tobytes(), int(sv[j]), int(sv[j] and occ[j]))
            for j in np.flatnonzero(win)]
    return recs, (int(tail[0]), int(tail[1]))


def _frame_replicated_ao(po, local, comm, sh, bsdfs, org, d, pix, sam, spp, image):
    """The replicated-ray AO frame (insitu.cpp trace_replicated_ao): the
    lists, keyed closest hits and key MIN of trace_frame_replicated; the
    winners publish their hit's shading normal and colour (SUM all-reduce);
    every rank shades every hit (ooc::ShaderAo: the same AO rays on every
    rank) and any-hits the rays over its own domains; a SUM all-reduce of
    the per-sample occlusion counts ORs the results; rank 0 films the whole
    frame.  Totals need no collective (every rank spawned every AO ray)."""
    import torch as t
    ns = po.shadow_slots(sh)
    org, d = np.ascontiguousarray(org, np.float32), np.ascontiguousarray(d, np.float32)
    pix, sam = np.asarray(pix, np.int32), np.asarray(sam, np.int32)
    n = len(org)
    rays = _rays(org, d)
    mask = local.route(rays).numpy()
    C = np.flatnonzero(mask != 0)
    mine = ((mask[C] >> comm.rank) & 1).astype(bool)
    keys_c = np.full(len(C), MISS_KEY, np.int64)
    hits_c = np.zeros(len(C), po.HIT_DTYPE)
    if mine.any():
        h, k = local.intersect_keyed(rays[C[mine]])
        keys_c[mine] = k.numpy()
        hits_c[mine] = np.ascontiguousarray(h.numpy()).view(po.HIT_DTYPE).reshape(-1)
    own = keys_c.copy()
    best = comm.all_reduce_min(t.from_numpy(keys_c.copy())).numpy()
    hit = best != MISS_KEY
    win = hit & (own == best)
    # the winners' normals and colours, on every rank
    pub = np.zeros((len(C), 4), np.int64)
    pub[win, 0:3] = np.ascontiguousarray(hits_c["ns"][win]).view(np.uint32)
    pub[win, 3] = hits_c["color"][win]
    pub = comm.all_reduce_sum(t.from_numpy(pub)).numpy().astype(np.uint32)
    hall = np.zeros(len(C), po.HIT_DTYPE)
    hall["t"] = np.inf
    hall["prim"] = 0xFFFFFFFF
    hall["domain"] = -1
    hall["t"][hit] = (best[hit] >> 32).astype(np.uint32).view(np.float32)
    hall["domain"][hit] = (best[hit] & 0xFFFF).astype(np.int32)
    hall["ns"] = np.ascontiguousarray(pub[:, 0:3]).view(np.float32)
    hall["color"] = pub[:, 3]
    # every hit's AO rays (the same on every rank)
    def shade(hits, valid):
        oc, dc = np.ascontiguousarray(org[C]), np.ascontiguousarray(d[C])
        w = np.ones((len(C), 3), np.float32)
        return po.shade(sh, bsdfs, 0, oc, dc, hits, w, valid.astype(np.uint8), pix[C], sam[C])
    so, sd, sw, sv, aborts = shade(hall, hit)
    assert aborts == 0
    sv = sv.astype(bool)
    # the winner's own shading spawns exactly those rays
    so2, sd2, sw2, sv2, _ = shade(hits_c, win)
    ws = np.repeat(win, ns)
    assert (sv2.astype(bool) == (sv & ws)).all()
    assert so2[sv2.astype(bool)].tobytes() == so[sv & ws].tobytes()
    assert sd2[sv2.astype(bool)].tobytes() == sd[sv & ws].tobytes()
    assert sw2[sv2.astype(bool)].tobytes() == sw[sv & ws].tobytes()
    sel = np.flatnonzero(sv)
    occ = np.zeros(len(C) * ns, np.int32)
    if len(sel):
        occ[sel] = local.occluded(_rays(so[sel], sd[sel])).numpy()
    occ = comm.all_reduce_sum(t.from_numpy(occ)).numpy() > 0
    if comm.rank == 0:
        lit = np.flatnonzero(sv & ~occ)
        if len(lit):
            img = image.reshape(-1, 4)
            add = ((1.0 / spp) * sw[lit].astype(np.float64)).astype(np.float32)
            np.add.at(img[:, :3], pix[C[lit // ns]], add)
    recs = []
    for j in np.flatnonzero(win):
        bv = bo = 0
        for k in range(ns):
            if sv[j * ns + k]:
                bv |= 1 << k
                if occ[j * ns + k]:
                    bo |= 1 << k
        recs.append((0, int(sam[C[j]]), hits_c[j].tobytes(), bv, bo))
    return recs, (n, int(sv.sum()))
