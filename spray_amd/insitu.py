"""In-situ (domain-sharded) tracing across ranks, one rank per GPU.

The reference's in-situ mode (src/insitu/) keeps every domain resident on
exactly one MPI rank and moves rays to the data:

* ``InsituPartition::partition`` (src/render/data_partition.h:59-137): domain
  centroids Morton-coded, sorted, dealt out in contiguous shares;
* ``TileList`` / ``makeHorizontalStripe`` (src/render/tile.cc:159-212): each
  rank generates the eye rays of one horizontal stripe of every blocking
  tile;
* ``Isector::intersect`` (src/insitu/insitu_isector.h:164-224): every ray is
  queued, speculatively, to every domain on its sorted domain list, and the
  queues of remote domains travel to their owners (insitu_comm.inl:28-101,
  MPI Isend/Iprobe/Recv);
* ``VBuf::compositeTbuf`` / ``compositeObuf`` (src/insitu/insitu_vbuf.h:
  74-152): the per-sample nearest t is reduced with MPI_Allreduce(MIN), and
  only the rank whose local hit equals it shades the sample and spawns its
  shadow ray; occlusion bits are reduced with MPI_Allreduce(MAX).

Here the queues become bulk exchanges over RCCL (torch.distributed "nccl"):
a count all-to-all, then one all-to-all of 32-B rays + 4-B sample ids per
bounce.  The tbuf is a 64-bit composite key (t, position in the ray's sorted
domain list, domain), reduced with MIN: the winner is then unique and equal
to the sequential walk of the whole list (spray_rt_intersect_scene_keyed),
where the reference leaves exact t ties to MPI's reduction order.

The protocol runs on torch tensors; the local work (routing, keyed closest
hit, shadow spawn, any hit) is a pluggable ``local`` object -- on a GPU the
HIP engine (:class:`GpuLocal`).  Collectives with the "gloo" backend stage
device tensors through host memory (tests; the product runs "nccl").
"""
from __future__ import annotations

import numpy as np

__all__ = ["morton_code", "morton_partition", "horizontal_stripe", "Comm", "GpuLocal",
           "InsituTracer", "MISS_KEY", "setup_rank_context"]

MISS_KEY = 0x7FFFFFFFFFFFFFFF


# ---------------------------------------------------------------------------
# partition and stripes
# ---------------------------------------------------------------------------
def _expand_bits(v):
    """Morton::expandBits (src/render/morton.h:44-50), uint32 arithmetic."""
    v = np.uint32(v)
    with np.errstate(over="ignore"):
        v = (v * np.uint32(0x00010001)) & np.uint32(0xFF0000FF)
        v = (v * np.uint32(0x00000101)) & np.uint32(0x0F00F00F)
        v = (v * np.uint32(0x00000011)) & np.uint32(0xC30C30C3)
        v = (v * np.uint32(0x00000005)) & np.uint32(0x49249249)
    return v


def morton_code(x, y, z):
    """Morton::compute (src/render/morton.h:32-41): 30-bit code of a point in
    the unit cube, float32 clamping as the reference."""
    f = np.float32
    c = []
    for a in (x, y, z):
        a = f(min(max(f(a) * f(1024.0), f(0.0)), f(1023.0)))
        c.append(_expand_bits(int(a)))
    with np.errstate(over="ignore"):
        return int((c[0] * np.uint32(4) + c[1] * np.uint32(2) + c[2]) & np.uint32(0xFFFFFFFF))


def morton_partition(boxes, scene_bound, nranks):
    """InsituPartition::partition with GROUP_CLOSE_DOMAINS
    (src/render/data_partition.h:59-137) -> owner rank per domain.

    boxes [n, 6] (lo, hi) world bounds in domain-id order, scene_bound [6].
    Codes are sorted by (code, domain id): std::sort leaves equal codes in an
    unspecified order, the domain id makes the map deterministic.  As in the
    reference, shares = n // nranks (0 when n < nranks: every domain then
    stays on rank 0) and the rank counter wraps."""
    f = np.float32
    boxes = np.asarray(boxes, f).reshape(-1, 6)
    sb = np.asarray(scene_bound, f).reshape(6)
    n = len(boxes)
    if nranks <= 0:
        raise ValueError("nranks must be > 0")
    diag = sb[3:] - sb[:3]
    scale = (f(1.0) / diag).astype(f)
    mn = (sb[:3] * scale).astype(f)
    off = (f(0.0) - mn).astype(f)
    codes = []
    for i in range(n):
        center = ((boxes[i, :3] + boxes[i, 3:]) * f(0.5)).astype(f)  # Aabb::getCenter
        c = (center * scale + off).astype(f)
        codes.append((morton_code(c[0], c[1], c[2]), i))
    codes.sort()
    owner = np.zeros(n, np.int32)
    shares = n // nranks
    rank, s = 0, 0
    for _, dom in codes:
        owner[dom] = rank
        s += 1
        if s == shares:
            s = 0
            rank += 1
            if rank == nranks:
                rank = 0
    return owner


def horizontal_stripe(nranks, rank, tile):
    """makeHorizontalStripe (src/render/tile.cc:187-209): tile = (x, y, w, h)
    -> this rank's stripe (x, y, w, h); w = h = 0 when empty."""
    x, y, w, h = tile
    hh = max(h // nranks, 1)
    oy = y + rank * hh
    yend = y + h
    if oy >= yend:
        return (0, oy, 0, 0)
    oh = yend - oy if (oy + hh > yend or rank == nranks - 1) else hh
    return (x, oy, w, oh)


# ---------------------------------------------------------------------------
# collectives
# ---------------------------------------------------------------------------
class Comm:
    """The rank group.  world == 1 makes every collective a no-op; "gloo"
    stages device tensors through host memory."""

    def __init__(self, dist=None, group=None, always=False):
        self.dist = dist
        self.group = group
        if dist is not None and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            self.staged = dist.get_backend(group) == "gloo"
        else:
            self.rank, self.world, self.staged = 0, 1, False
        # always: issue the collectives even for one rank (exercises RCCL)
        self.skip = self.world == 1 and not (always and dist is not None)

    def _host(self, t):
        return t.cpu() if (self.staged and t.is_cuda) else t

    def all_to_all(self, out, inp, out_splits, in_splits):
        if self.skip:
            out.copy_(inp)
            return out
        o, i = self._host(out), self._host(inp)
        self.dist.all_to_all_single(o, i, out_splits, in_splits, group=self.group)
        if o is not out:
            out.copy_(o)
        return out

    def all_reduce(self, t, op):
        if self.skip:
            return t
        h = self._host(t)
        self.dist.all_reduce(h, op=op, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def op(self, name):
        return getattr(self.dist.ReduceOp, name) if self.dist is not None else None


# ---------------------------------------------------------------------------
# local work on one GPU
# ---------------------------------------------------------------------------
class GpuLocal:
    """Local work of one rank through the HIP engine (device tensors).
    Rays are float32 [n, 8] (org, tnear, dir, tfar), hits float32 [n, 12]
    (spray_rt_hit), keys / rank masks int64 [n]."""

    def __init__(self, rt, device, stream=None):
        import torch
        self.torch = torch
        self.rt = rt
        self.device = device
        # the engine enqueues on torch's stream: the protocol's torch ops and
        # the kernels stay ordered without host synchronisation
        rt.set_stream(stream if stream is not None else torch.cuda.current_stream(device))

    def route(self, rays):
        m = self.torch.empty(rays.shape[0], dtype=self.torch.int64, device=self.device)
        if rays.shape[0]:
            self.rt.route(rays, m)
        return m

    def intersect_keyed(self, rays):
        n = rays.shape[0]
        hits = self.torch.empty((n, 12), dtype=self.torch.float32, device=self.device)
        keys = self.torch.empty(n, dtype=self.torch.int64, device=self.device)
        if n:
            self.rt.intersect_scene_keyed(rays, hits, keys)
        return hits, keys

    def spawn_pt(self, rays, hits, shade):
        t = self.torch
        n = rays.shape[0]
        out = t.empty((max(n, 1), 8), dtype=t.float32, device=self.device)
        src = t.empty(max(n, 1), dtype=t.int32, device=self.device)
        cnt = t.zeros(1, dtype=t.int32, device=self.device)
        if n:
            self.rt.spawn_shadows_pt(rays, hits, n, shade, out, src, cnt)
        k = int(cnt.item()) if n else 0
        return out[:k], src[:k].long()

    def plan(self, mask, world):
        """Per-destination ascending ray lists of a routed batch (device):
        bounds first (one host read sizes the list), then the lists."""
        t = self.torch
        starts = t.empty(world + 1, dtype=t.int64, device=self.device)
        self.rt.exchange_plan(mask, world, None, starts)
        total = int(starts[-1])
        idx = t.empty(max(total, 1), dtype=t.int64, device=self.device)
        self.rt.exchange_plan(mask, world, idx, starts)
        return idx[:total], starts

    def gather(self, src, idx, dst):
        """Exchange packing through the engine (torch's row gather is several
        times slower for 32- and 48-byte rows)."""
        self.rt.gather_rows(src, idx, dst)

    def occluded(self, rays):
        t = self.torch
        occ = t.zeros(rays.shape[0], dtype=t.uint8, device=self.device)
        if rays.shape[0]:
            self.rt.occluded_scene(rays, occ)
        return occ


def setup_rank_context(rt, desc, ply_path, owner, rank):
    """Loads the domains ``owner`` assigns to ``rank`` into slots 0..k-1 of
    the engine context and installs the full domain box set and owner map
    (every rank computes the same domain lists)."""
    from .engine import host_domain_mesh, host_parse_scene
    boxes, _ = host_parse_scene(desc, ply_path)
    rt.domain_bounds(boxes)
    mine = [d for d in range(len(boxes)) if owner[d] == rank]
    for slot, d in enumerate(mine):
        v, f, c, n = host_domain_mesh(desc, ply_path, d)
        rt.upload_domain(slot, v, f, c, n)
        rt.map_domain(d, slot)
    rt.set_owners(owner)
    return mine


# ---------------------------------------------------------------------------
# the per-tile protocol
# ---------------------------------------------------------------------------
class Exchange:
    """One routed exchange: row i of a ray batch goes to every rank whose bit
    is set in mask[i].  ``forward`` moves per-ray payloads to the owners
    (grouped by source rank, in the sender's order); ``backward`` returns
    per-copy results to the sender, in the order the copies were sent."""

    def __init__(self, comm, mask, gather=None, plan=None):
        import torch as t
        W = comm.world
        self.comm = comm
        self.gather = gather
        n = mask.shape[0]
        if plan is not None and mask.is_cuda:
            # device plan: per-rank lists + bounds in four small kernels
            self.idx, starts = plan(mask, W)
            send = starts[1:] - starts[:-1]
        else:
            if n:
                bit = t.arange(W, device=mask.device, dtype=t.int64).unsqueeze(1)
                sel = ((mask.unsqueeze(0) >> bit) & 1).bool()  # [W, n], dest-major
                dest, self.idx = sel.nonzero(as_tuple=True)
            else:
                dest = t.zeros(0, dtype=t.int64, device=mask.device)
                self.idx = dest
            send = t.bincount(dest, minlength=W).to(t.int64)
        recv = t.empty_like(send)
        comm.all_to_all(recv, send, None, None)  # the count phase
        self.sc, self.rc = send.tolist(), recv.tolist()
        self.n_sent, self.n_recv = sum(self.sc), sum(self.rc)

    def forward(self, payload):
        """payload: per-ray rows [n, ...] of the sender's batch."""
        if self.gather is not None and payload.is_cuda:
            s = payload.new_empty((self.idx.numel(),) + tuple(payload.shape[1:]))
            self.gather(payload, self.idx, s)
        else:
            s = payload.index_select(0, self.idx)
        if self.comm.skip:
            return s
        r = payload.new_empty((self.n_recv,) + tuple(payload.shape[1:]))
        return self.comm.all_to_all(r, s, self.rc, self.sc)

    def backward(self, result):
        """result: per received copy [n_recv, ...] -> per sent copy."""
        if self.comm.skip:
            return result
        r = result.new_empty((self.n_sent,) + tuple(result.shape[1:]))
        return self.comm.all_to_all(r, result.contiguous(), self.sc, self.rc)


class InsituTracer:
    """One bounce (primary closest hit + point-light shadow rays) of a
    blocking tile, distributed by domain ownership.

    Compositing happens per ray copy instead of over a whole-tile buffer:
    the owners' keys travel back to the ray's sender (reverse all-to-all),
    the sender's minimum travels out again, and the one owner whose key
    equals it shades the sample and spawns its shadow ray; the shadow ray's
    occlusion bits come back to that rank and are OR-ed there.  This is the
    tbuf MIN / obuf MAX compositing of VBuf (insitu_vbuf.h:74-152) at the
    cost of 8 B (keys) and 1 B (occlusion) per remote copy, instead of
    all-reduces over every sample of the tile."""

    def __init__(self, local, comm):
        import torch
        self.torch = torch
        self.local = local
        self.comm = comm

    def trace_tile(self, rays, samid, shade):
        """rays float32 [n, 8] of this rank's stripe, samid [n] (blocking-
        tile sample ids).

        Returns a dict: ``samid`` / ``hits`` of the samples whose nearest hit
        lies in this rank's domains (this rank shades them), ``shadow_samid``
        / ``shadow_occ`` of the shadow rays it spawned, and the job totals
        ``n_rays`` and ``n_shadow``."""
        t = self.torch
        L, C = self.local, self.comm
        samid = samid.to(t.int32)
        n = rays.shape[0]
        # primary rays to the owners of their domains, keyed closest hit there
        gather, plan = getattr(L, "gather", None), getattr(L, "plan", None)
        ex = Exchange(C, L.route(rays), gather, plan)
        rrays, rsam = ex.forward(rays), ex.forward(samid)
        hits, keys = L.intersect_keyed(rrays)
        # composite: minimum key per ray at its sender, back to the owners
        best = t.full((n,), MISS_KEY, dtype=t.int64, device=rays.device)
        if ex.n_sent:
            best.scatter_reduce_(0, ex.idx, ex.backward(keys), "amin")
        win = (keys == ex.forward(best)) & (keys != MISS_KEY)
        out_hits = hits[win]
        # only the winner shades: the others' hits become misses
        hits.view(t.int32)[:, 11].masked_fill_(~win, -1)  # spray_rt_hit.domain
        srays, src = L.spawn_pt(rrays, hits, shade)
        # shadow rays to the owners of their domains, any hit, OR at the spawner
        sx = Exchange(C, L.route(srays), gather, plan)
        occ = L.occluded(sx.forward(srays))
        socc = t.zeros(srays.shape[0], dtype=t.uint8, device=rays.device)
        if sx.n_sent:
            socc.scatter_reduce_(0, sx.idx, sx.backward(occ), "amax")
        tot = t.tensor([n, srays.shape[0]], dtype=t.int64, device=rays.device)
        C.all_reduce(tot, C.op("SUM"))
        return {"samid": rsam[win].long(), "hits": out_hits,
                "shadow_samid": rsam.index_select(0, src).long(), "shadow_occ": socc,
                "n_rays": int(tot[0]), "n_shadow": int(tot[1])}
