"""In-situ (domain-sharded) frames across ranks, one rank per GPU: a thin
caller of the engine's in-situ tracer (spray_rt_insitu_*, insitu.cpp).

The reference's in-situ mode (src/insitu/) keeps every domain resident on
exactly one MPI rank and moves rays to the data:

* ``InsituPartition::partition`` (src/render/data_partition.h:59-137): domain
  centroids Morton-coded, sorted, dealt out in contiguous shares
  (``morton_partition`` -> spray_rt_insitu_partition);
* ``TileList`` / ``makeHorizontalStripe`` (src/render/tile.cc:159-212): each
  rank generates the eye rays of one horizontal stripe of every blocking
  tile (``horizontal_stripe``, spray_rt_eye_rays_insitu);
* the per-bounce exchange, compositing, shading and film run inside the
  engine (``InsituEngine.trace``): route, count exchange, ray exchange
  (grouped ncclSend / ncclRecv), keyed closest hit, key minimum, winner
  shading, shadow exchange and occlusion OR, film; one reduce composites the
  ranks' images (``InsituEngine.composite``).

Collectives go through RCCL directly from the engine; the communicator's id
is created on rank 0 and broadcast over ``torch.distributed`` once.  For tests
a host transport drives the same protocol over any ``torch.distributed``
group (e.g. "gloo" processes sharing one GPU), staging through host memory.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import SHADER_AO, SprayRtError, lib

__all__ = ["morton_partition", "view_partition", "partition", "PARTITION_GROUP_CLOSE",
           "PARTITION_ROUND_ROBIN", "PARTITION_VIEW", "horizontal_stripe", "setup_rank_context",
           "InsituEngine", "InsituRecords", "MISS_KEY", "box_rows", "shadow_boxes"]

MISS_KEY = 0x7FFFFFFFFFFFFFFF


PARTITION_GROUP_CLOSE = 0
PARTITION_ROUND_ROBIN = 1
PARTITION_VIEW = 2  # spray_rt_insitu_partition_view (needs the camera)


def view_partition(boxes, cam, nranks):
    """Owner rank per domain, view-aligned (spray_rt_insitu_partition_view):
    the box centres projected by camera record `cam` (camera_init, 14
    floats), dealt by recursive median splits into groups of equal count."""
    b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    c = np.ascontiguousarray(cam, np.float32).reshape(14)
    if nranks <= 0:
        raise ValueError("nranks must be > 0")
    owner = np.zeros(len(b), np.int32)
    rc = lib().spray_rt_insitu_partition_view(b.ctypes.data, len(b), c.ctypes.data, int(nranks),
                                              owner.ctypes.data)
    if rc:
        raise RuntimeError("spray_rt_insitu_partition_view failed (%d)" % rc)
    return owner


def partition(boxes, scene_bound, nranks, mode, cam=None):
    """morton_partition (GROUP_CLOSE / ROUND_ROBIN) or view_partition (VIEW)"""
    if mode == PARTITION_VIEW:
        return view_partition(boxes, cam, nranks)
    return morton_partition(boxes, scene_bound, nranks, mode)


def box_rows(cam, image_w, image_h, box):
    """(kind, x0[h], x1[h]) of spray_rt_camera_box_rows: per image row the
    pixel range whose eye rays may enter the box (x0 > x1: none); kind 0 =
    none, 1 = rows, 2 = the whole image"""
    c = np.ascontiguousarray(cam, np.float32).reshape(14)
    b = np.ascontiguousarray(box, np.float32).reshape(6)
    x0 = np.zeros(int(image_h), np.int32)
    x1 = np.zeros(int(image_h), np.int32)
    k = lib().spray_rt_camera_box_rows(c.ctypes.data, int(image_w), int(image_h), b.ctypes.data,
                                       x0.ctypes.data, x1.ctypes.data)
    if k < 0:
        raise ValueError("bad camera or box")
    return k, x0, x1


def shadow_boxes(box, scene, light, k=16):
    """spray_rt_camera_shadow_boxes: the slice boxes [n, 6] whose union holds
    the hit points whose shadow ray toward `light` may cross `box` (None:
    everywhere)"""
    out = np.zeros((k, 6), np.float32)
    n = lib().spray_rt_camera_shadow_boxes(
        np.ascontiguousarray(box, np.float32).ctypes.data,
        np.ascontiguousarray(scene, np.float32).ctypes.data,
        np.ascontiguousarray(light, np.float32).ctypes.data, int(k), out.ctypes.data)
    if n < -1:
        raise ValueError("bad arguments")
    return None if n < 0 else out[:n]


def morton_partition(boxes, scene_bound, nranks, mode=PARTITION_GROUP_CLOSE):
    """Owner rank per domain (InsituPartition::partition,
    src/render/data_partition.h:59-155): spray_rt_insitu_partition_mode.
    mode GROUP_CLOSE (contiguous shares of the sorted Morton order, the
    reference's compiled mode) or ROUND_ROBIN (the sorted order dealt out one
    domain per rank in turn).  boxes [n, 6] (lo, hi) world bounds in
    domain-id order, scene_bound [6]."""
    b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    sb = np.ascontiguousarray(scene_bound, np.float32).reshape(6)
    if nranks <= 0:
        raise ValueError("nranks must be > 0")
    owner = np.zeros(len(b), np.int32)
    rc = lib().spray_rt_insitu_partition_mode(b.ctypes.data, len(b), sb.ctypes.data,
                                              int(nranks), int(mode), owner.ctypes.data)
    if rc != 0:
        raise SprayRtError("insitu_partition failed (%d)" % rc)
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
# engine bindings
# ---------------------------------------------------------------------------
_A2A = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                   C.POINTER(C.c_size_t))
_AR = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)
_RED = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int)


class Transport(C.Structure):
    _fields_ = [("struct_size", C.c_size_t), ("user", C.c_void_p), ("alltoallv", _A2A),
                ("allreduce_u64", _AR),
                ("reduce_f32", _RED), ("allreduce_min_u64", _AR), ("allreduce_sum_u8", _AR)]


class RecStruct(C.Structure):
    _fields_ = [("samid", C.c_void_p), ("bounce", C.c_void_p), ("hits", C.c_void_p),
                ("svalid", C.c_void_p), ("occluded", C.c_void_p), ("cap", C.c_size_t),
                ("d_count", C.c_void_p)]


def _host_view(ptr, nbytes):
    if nbytes == 0:
        return np.zeros(0, np.uint8)
    return np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr))


class _HostCollectives:
    """spray_rt_transport over a torch.distributed group (host tensors)."""

    def __init__(self, dist, group=None):
        import torch
        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)

        def a2a(user, send, sb, recv, rb):
            try:
                s = [int(sb[r]) for r in range(self.world)]
                r = [int(rb[k]) for k in range(self.world)]
                src = torch.from_numpy(_host_view(send, sum(s)).copy())
                dst = torch.empty(sum(r), dtype=torch.uint8)
                self.dist.all_to_all_single(dst, src, r, s, group=self.group)
                if sum(r):
                    _host_view(recv, sum(r))[:] = dst.numpy()
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the status
                print("insitu host all-to-all failed:", e)
                return 1

        def ar(user, data, n):
            try:
                a = _host_view(data, 8 * n).view(np.int64)
                t = torch.from_numpy(a.copy())
                self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
                a[:] = t.numpy()
                return 0
            except Exception as e:  # noqa: BLE001
                print("insitu host all-reduce failed:", e)
                return 1

        def red(user, data, n, root):
            try:
                a = _host_view(data, 4 * n).view(np.float32)
                t = torch.from_numpy(a.copy())
                self.dist.reduce(t, dst=root, op=self.dist.ReduceOp.SUM, group=self.group)
                a[:] = t.numpy()
                return 0
            except Exception as e:  # noqa: BLE001
                print("insitu host reduce failed:", e)
                return 1

        def armin(user, data, n):
            try:  # keys are < 2^63: int64 MIN is their u64 MIN
                a = _host_view(data, 8 * n).view(np.int64)
                t = torch.from_numpy(a.copy())
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
                a[:] = t.numpy()
                return 0
            except Exception as e:  # noqa: BLE001
                print("insitu host min all-reduce failed:", e)
                return 1

        def arsum8(user, data, n):
            try:  # each byte sums at most `world` ones
                a = _host_view(data, n)
                t = torch.from_numpy(a.astype(np.int32))
                self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
                a[:] = t.numpy().astype(np.uint8)
                return 0
            except Exception as e:  # noqa: BLE001
                print("insitu host byte all-reduce failed:", e)
                return 1

        self._cbs = (_A2A(a2a), _AR(ar), _RED(red), _AR(armin), _AR(arsum8))  # kept alive
        self.struct = Transport(C.sizeof(Transport), None, *self._cbs)


class InsituRecords:
    """Device buffers of spray_rt_insitu_rec: per shaded copy its sample id,
    bounce, winning hit (float32 [cap, 12]) and shadow-slot bits."""

    def __init__(self, cap, device="cuda"):
        import torch
        self.cap = int(cap)
        self.samid = torch.zeros(cap, dtype=torch.int32, device=device)
        self.bounce = torch.zeros(cap, dtype=torch.int32, device=device)
        self.hits = torch.zeros((cap, 12), dtype=torch.float32, device=device)
        self.svalid = torch.zeros(cap, dtype=torch.int64, device=device)
        self.occluded = torch.zeros(cap, dtype=torch.int64, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.struct = RecStruct(self.samid.data_ptr(), self.bounce.data_ptr(),
                                self.hits.data_ptr(), self.svalid.data_ptr(),
                                self.occluded.data_ptr(), self.cap, self.count.data_ptr())

    def numpy(self):
        """Host copies of the written records, sorted by (bounce, samid)."""
        n = int(self.count.item())
        if n > self.cap:
            raise SprayRtError("record buffer overflow: %d > %d" % (n, self.cap))
        s = self.samid[:n].cpu().numpy()
        b = self.bounce[:n].cpu().numpy()
        o = np.lexsort((s, b))
        return {"samid": s[o], "bounce": b[o], "hits": self.hits[:n].cpu().numpy()[o],
                "svalid": self.svalid[:n].cpu().numpy().view(np.uint64)[o],
                "occluded": self.occluded[:n].cpu().numpy().view(np.uint64)[o]}


class InsituEngine:
    """spray_rt_insitu_t of one rank.

    transport="rccl" (the product): RCCL communicator from an id made on
    rank 0 and broadcast over ``dist`` (world 1 needs no ``dist``).
    transport="host": host-staged collectives over ``dist`` (tests).
    transport="replay": no collectives -- the group results of a camera
    frame replayed from replay_set (measurement of one rank alone)."""

    def __init__(self, rt, world=1, rank=0, dist=None, transport="rccl", group=None):
        import torch
        self.rt, self.world, self.rank = rt, int(world), int(rank)
        self._host = None
        h = C.c_void_p()
        L = lib()
        if transport == "rccl":
            uid = np.zeros(128, np.uint8)
            if self.rank == 0:
                rc = L.spray_rt_insitu_unique_id(uid.ctypes.data, 128)
                if rc != 0:
                    raise SprayRtError("spray_rt_insitu_unique_id failed (%d)" % rc)
            if self.world > 1:
                t = torch.from_numpy(uid)
                if dist.get_backend(group) == "nccl":
                    t = t.cuda()
                dist.broadcast(t, src=0, group=group)
                uid = np.ascontiguousarray(t.cpu().numpy())
            rc = L.spray_rt_insitu_create(rt.h, self.world, self.rank, uid.ctypes.data, None,
                                          C.byref(h))
        elif transport == "host":
            if self.world > 1 and dist is None:
                raise ValueError("host transport needs a torch.distributed group")
            self._host = _HostCollectives(dist, group) if dist is not None else None
            if self._host is None:  # world 1 without a group: local no-op collectives
                self._host = _LocalCollectives()
            rc = L.spray_rt_insitu_create(rt.h, self.world, self.rank, None,
                                          C.byref(self._host.struct), C.byref(h))
        elif transport == "replay":
            rc = L.spray_rt_insitu_create_replay(rt.h, self.world, self.rank, C.byref(h))
        else:
            raise ValueError("transport must be 'rccl', 'host' or 'replay'")
        rt._check(rc, "insitu_create")
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib().spray_rt_insitu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trace(self, shader, rays, pixid, samid, spp, image, records=None):
        """This rank's eye rays (device: rays [n, 8] float32 or 32-B rows,
        pixid / samid int32 [n]) through shader.bounces bounces; the shaded
        samples' contributions go to image (device float32 [w*h*4]).
        Returns the group's (radiance rays, shadow rays)."""
        from .engine import _addr, _nbytes
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        p, k2 = _addr(pixid)
        s, k3 = _addr(samid)
        im, k4 = _addr(image)
        tot = (C.c_ulonglong * 3)()
        rec = C.byref(records.struct) if records is not None else None
        rc = lib().spray_rt_insitu_trace(self.h, C.byref(shader), a, p, s, n, int(spp), im, rec,
                                         C.byref(tot))
        self.rt._check(rc, "insitu_trace")
        return int(tot[0]), int(tot[1])

    def trace_frame(self, shader, rays, pixid, samid, spp, image, records=None):
        """The whole frame with replicated eye rays (spray_rt_insitu_trace_frame):
        rays / pixid / samid are EVERY eye ray of the frame, the same on every
        rank.  Returns the group's (radiance rays, shadow rays)."""
        from .engine import _addr, _nbytes
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        p, k2 = _addr(pixid)
        s, k3 = _addr(samid)
        im, k4 = _addr(image)
        tot = (C.c_ulonglong * 3)()
        rec = C.byref(records.struct) if records is not None else None
        rc = lib().spray_rt_insitu_trace_frame(self.h, C.byref(shader), a, p, s, n, int(spp), im,
                                               rec, C.byref(tot))
        self.rt._check(rc, "insitu_trace_frame")
        self._rep_kind = "ao" if shader.shader == SHADER_AO else "pt"
        return int(tot[0]), int(tot[1])

    def trace_camera(self, shader, cam, image_w, image_h, spp, image, records=None):
        """The whole frame of camera record `cam` (spray_rt_insitu_trace_camera):
        the eye rays generated in the lanes, each rank's work bounded by its
        domains' screen footprints.  Returns the group's (radiance rays,
        shadow rays)."""
        from .engine import _addr
        c = np.ascontiguousarray(cam, np.float32).reshape(14)
        im, k4 = _addr(image)
        tot = (C.c_ulonglong * 3)()
        rec = C.byref(records.struct) if records is not None else None
        rc = lib().spray_rt_insitu_trace_camera(self.h, C.byref(shader), c.ctypes.data,
                                                int(image_w), int(image_h), int(spp), im, rec,
                                                C.byref(tot))
        self.rt._check(rc, "insitu_trace_camera")
        self._rep_kind = "ao" if shader.shader == SHADER_AO else "pt"
        return int(tot[0]), int(tot[1])

    def trace_image(self, shader, cam, image_w, image_h, spp, image, bands=1, records=None):
        """The image-parallel frame (spray_rt_insitu_trace_image): every domain
        resident on every rank, this rank's row bands traced with the
        all-local frame, the rows gathered into rank 0's image.  Returns the
        group's (radiance rays, shadow rays)."""
        from .engine import _addr
        c = np.ascontiguousarray(cam, np.float32).reshape(14)
        im, k4 = _addr(image)
        tot = (C.c_ulonglong * 3)()
        rec = C.byref(records.struct) if records is not None else None
        rc = lib().spray_rt_insitu_trace_image(self.h, C.byref(shader), c.ctypes.data,
                                               int(image_w), int(image_h), int(spp), int(bands),
                                               im, rec, C.byref(tot))
        self.rt._check(rc, "insitu_trace_image")
        return int(tot[0]), int(tot[1])

    def replay_capture(self):
        """(tmin u32, lpmin u8) device tensors of the last camera PT frame's
        group minima over U (spray_rt_insitu_replay_capture)."""
        import torch
        n = C.c_size_t(0)
        self.rt._check(lib().spray_rt_insitu_replay_capture(self.h, None, None, 0, C.byref(n)),
                       "replay_capture")
        t = torch.empty(max(n.value, 1), dtype=torch.int32, device="cuda")[:n.value]
        lp = torch.empty(max(n.value, 1), dtype=torch.uint8, device="cuda")[:n.value]
        self.rt._check(lib().spray_rt_insitu_replay_capture(self.h, t.data_ptr(), lp.data_ptr(),
                                                            n.value, C.byref(n)),
                       "replay_capture")
        return t, lp

    def replay_capture_ao(self):
        """(kmin u64, pub u64 [2 n]) device tensors of the last AO camera
        frame's key minima and published normals over U
        (spray_rt_insitu_replay_capture_ao)."""
        import torch
        n = C.c_size_t(0)
        self.rt._check(lib().spray_rt_insitu_replay_capture_ao(self.h, None, None, 0,
                                                               C.byref(n)), "replay_capture_ao")
        k = torch.empty(max(n.value, 1), dtype=torch.int64, device="cuda")[:n.value]
        pub = torch.empty(max(2 * n.value, 1), dtype=torch.int64, device="cuda")[:2 * n.value]
        self.rt._check(lib().spray_rt_insitu_replay_capture_ao(self.h, k.data_ptr(), pub.data_ptr(),
                                                               n.value, C.byref(n)),
                       "replay_capture_ao")
        return k, pub

    def replay_set_ao(self, kmin, pub):
        """The AO frame's group results a replay context hands back."""
        self._replay_ao = (kmin, pub)
        self.rt._check(lib().spray_rt_insitu_replay_set_ao(self.h, kmin.data_ptr(), pub.data_ptr(),
                                                           kmin.numel()), "replay_set_ao")

    def replay_bits_ao(self, bits=None):
        """Without bits: the last AO frame's own first-round occlusion bits
        (uint8 device tensor); with bits: the group's OR, handed back by that
        SUM in the following frames (spray_rt_insitu_replay_bits_ao)."""
        import torch
        n = C.c_size_t(0)
        if bits is None:
            self.rt._check(lib().spray_rt_insitu_replay_bits_ao(self.h, None, None, 0, C.byref(n)),
                           "replay_bits_ao")
            out = torch.empty(max(n.value, 1), dtype=torch.uint8, device="cuda")[:n.value]
            self.rt._check(lib().spray_rt_insitu_replay_bits_ao(self.h, None, out.data_ptr(),
                                                                n.value, C.byref(n)),
                           "replay_bits_ao")
            return out
        self._replay_bits = bits
        self.rt._check(lib().spray_rt_insitu_replay_bits_ao(self.h, bits.data_ptr(), None,
                                                            bits.numel(), C.byref(n)),
                       "replay_bits_ao")
        return None

    def replay_set(self, tmin, lpmin):
        """The group results a replay context's collectives hand back."""
        self._replay = (tmin, lpmin)  # keep the tensors alive
        self.rt._check(lib().spray_rt_insitu_replay_set(self.h, tmin.data_ptr(), lpmin.data_ptr(),
                                                        tmin.numel()), "replay_set")

    def set_timing(self, on=True):
        """Per-phase HIP-event timing of the traces (phase_times)."""
        self.rt._check(lib().spray_rt_insitu_set_timing(self.h, 1 if on else 0), "set_timing")

    # replicated-ray frames (insitu.cpp trace_replicated / trace_replicated_ao)
    # phase 0: C' (trace_frame) or the footprint tables and prefills
    # (trace_camera; its film needs no slots)
    REP_PHASES = ("prepare", "film_slots", "keyed_shade", "list_pos", "shadow_trace",
                  "winners", "film_totals")
    REP_AO_PHASES = ("prepare", "unused", "keyed_closest_hit", "publish", "ao_spawn",
                     "ao_own_trace", "film_totals")
    _rep_kind = "pt"
    PROTOCOL_PHASES = ("route_plan", "ray_pack_unpack", "keyed_closest_hit", "key_composite",
                       "shading", "shadow_route_pack", "shadow_any_hit_return",
                       "film_totals")

    def phase_times(self):
        """{phase: ms} accumulated since the last call (then reset); "collectives":
        the stream time inside the collectives and their count reads."""
        out = (C.c_double * 9)()
        n = C.c_int(0)
        lib().spray_rt_insitu_phase_times(self.h, C.byref(out), C.byref(n))
        rep = self.REP_AO_PHASES if self._rep_kind == "ao" else self.REP_PHASES
        names = {7: rep, 8: self.PROTOCOL_PHASES, 1: ("frame",)}.get(
            n.value, tuple("phase%d" % k for k in range(n.value)))
        d = {names[k]: float(out[k]) for k in range(n.value) if names[k] != "unused"}
        d["collectives"] = float(out[8])
        return d

    def composite(self, image):
        """HdrImage::composite: SUM of the ranks' images at rank 0."""
        from .engine import _addr
        im, k = _addr(image)
        rc = lib().spray_rt_insitu_composite(self.h, im, image.numel())
        self.rt._check(rc, "insitu_composite")
        return image

    COLL_OPS = {1: "counts_a2a_i64", 2: "alltoallv_u8", 3: "allreduce_sum_u64",
                4: "reduce_sum_f32", 5: "allreduce_min_u64", 6: "allreduce_sum_u8",
                7: "allreduce_min_u32", 8: "allreduce_min_u8"}

    def collective_log(self, clear=True):
        """The collectives this rank issued since the last read, in call order
        (spray_rt_insitu_collective_log): [(op, count, stream)] with stream
        "main" or "side".  Every rank of a group must issue the same list."""
        n = C.c_size_t(0)
        lib().spray_rt_insitu_collective_log(self.h, None, 0, C.byref(n), 0)
        buf = (C.c_uint64 * max(n.value, 1))()
        self.rt._check(lib().spray_rt_insitu_collective_log(self.h, buf, n.value, C.byref(n),
                                                            1 if clear else 0),
                       "collective_log")
        out = []
        for k in range(min(n.value, 1 << 16)):
            e = int(buf[k])
            out.append((self.COLL_OPS.get(e >> 56, "op%d" % (e >> 56)), e & ((1 << 48) - 1),
                        "side" if (e >> 51) & 1 else "main"))
        return out

    def stats(self):
        out = (C.c_ulonglong * 6)()
        lib().spray_rt_insitu_stats(self.h, C.byref(out))
        keys = ("bytes_sent", "bytes_received", "exchanges", "host_count_reads",
                "collectives", "traces")
        return dict(zip(keys, (int(x) for x in out)))


class _LocalCollectives:
    """A one-rank group's collectives (identity), for the host transport."""

    def __init__(self):
        def a2a(user, send, sb, recv, rb):
            n = int(sb[0])
            if n:
                C.memmove(recv, send, n)
            return 0

        self._cbs = (_A2A(a2a), _AR(lambda u, d, n: 0), _RED(lambda u, d, n, r: 0),
                     _AR(lambda u, d, n: 0), _AR(lambda u, d, n: 0))
        self.struct = Transport(C.sizeof(Transport), None, *self._cbs)
