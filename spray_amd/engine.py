"""Python front-end of the engine: RtContext (spray_rt.h) and Scene
(spray_scene.h).

Buffers may be numpy arrays (host: the call is synchronous, like Embree's)
or torch tensors on the GPU (device: enqueued on the context's stream; call
``sync()``).  The method names follow the reference's scene surface
(src/render/scene.h:153-205): load, intersect, occluded, intersectDomains.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import (HIT_DTYPE, INVALID_ID, RAY_DTYPE, RTC_ISECT_DTYPE, BsdfRec,
                      SprayRtError, lib)

__all__ = ["RtContext", "Scene", "OocCache", "ooc_scene", "camera_init", "make_rays",
           "host_parse_scene", "host_scene_bsdfs",
           "host_domain_mesh", "RAY_DTYPE",
           "HIT_DTYPE", "RTC_ISECT_DTYPE", "INVALID_ID", "SprayRtError"]


def _addr(x):
    """(address, keepalive) of a numpy array / torch tensor / int / None."""
    if x is None:
        return None, None
    if isinstance(x, int):
        return x, None
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("arrays must be C-contiguous")
        return x.ctypes.data, x
    if hasattr(x, "data_ptr"):
        if hasattr(x, "is_contiguous") and not x.is_contiguous():
            raise ValueError("tensors must be contiguous")
        return x.data_ptr(), x
    raise TypeError("unsupported buffer type %r" % type(x))


def _nbytes(x):
    if isinstance(x, np.ndarray):
        return x.nbytes
    return x.numel() * x.element_size()


def _lv_pixels(lv, nsamples):
    """Pixels the (pixel, sample) table lv holds (float4 per entry): the
    engine's bound on the pixel ids of an AO pairs spawn."""
    return _nbytes(lv) // (16 * int(nsamples))


def camera_init(pos, lookat, up, vfov, w, h):
    """Camera::init (src/render/camera.h:128-166) -> float32[14]."""
    cam = np.zeros(14, np.float32)
    p = np.asarray(pos, np.float32)
    la = np.asarray(lookat, np.float32)
    u = np.asarray(up, np.float32)
    lib().spray_camera_init(p.ctypes.data, la.ctypes.data, u.ctypes.data,
                            float(vfov), int(w), int(h), cam.ctypes.data)
    return cam


def make_rays(org, dir, tnear=0.001, tfar=np.inf):
    """Packs org/dir [n,3] into the 32-B ray records of the scene path."""
    org = np.asarray(org, np.float32).reshape(-1, 3)
    r = np.zeros(len(org), RAY_DTYPE)
    r["org"] = org
    r["dir"] = np.asarray(dir, np.float32).reshape(-1, 3)
    r["tnear"] = tnear
    r["tfar"] = tfar
    return r


def host_parse_scene(desc, ply_path=""):
    """Scene file -> (boxes [n,6], lights [nl,7]) without touching the GPU
    (spray_host_parse_scene)."""
    nd, nl = C.c_int(), C.c_int()
    err = C.create_string_buffer(1024)
    if lib().spray_host_parse_scene(desc.encode(), (ply_path or "").encode(), C.byref(nd),
                                    C.byref(nl), None, None, None, err, 1024) != 0:
        raise SprayRtError("parse %s: %s" % (desc, err.value.decode()))
    boxes = np.zeros((nd.value, 6), np.float32)
    xf = np.zeros((nd.value, 16), np.float32)
    lights = np.zeros((nl.value, 7), np.float32)
    if lib().spray_host_parse_scene(desc.encode(), (ply_path or "").encode(), C.byref(nd),
                                    C.byref(nl), boxes.ctypes.data, xf.ctypes.data,
                                    lights.ctypes.data, err, 1024) != 0:
        raise SprayRtError("parse %s: %s" % (desc, err.value.decode()))
    return boxes, lights


def host_scene_bsdfs(desc):
    """Scene file -> [(type, p0, p1, p2)] per domain (SceneLoader::parseMaterial)."""
    nd = C.c_int()
    err = C.create_string_buffer(1024)
    L = lib()
    if L.spray_host_scene_bsdfs(desc.encode(), C.byref(nd), None, err, 1024) != 0:
        raise SprayRtError("parse %s: %s" % (desc, err.value.decode()))
    arr = (BsdfRec * max(nd.value, 1))()
    if L.spray_host_scene_bsdfs(desc.encode(), C.byref(nd), C.addressof(arr), err, 1024) != 0:
        raise SprayRtError("materials of %s: %s" % (desc, err.value.decode()))
    return [(arr[i].type, arr[i].p[0], arr[i].p[1], arr[i].p[2]) for i in range(nd.value)]


def host_domain_mesh(desc, ply_path, domain_id):
    """TriMeshBuffer::load of one domain on the host -> (verts, faces,
    colors, normals)."""
    nv, nf = C.c_size_t(), C.c_size_t()
    L = lib()
    if L.spray_host_domain_mesh(desc.encode(), (ply_path or "").encode(), int(domain_id),
                                C.byref(nv), C.byref(nf), None, None, None, None) != 0:
        raise SprayRtError("domain %d of %s failed to load" % (domain_id, desc))
    v = np.zeros((nv.value, 3), np.float32)
    f = np.zeros((nf.value, 3), np.uint32)
    c = np.zeros(nv.value, np.uint32)
    n = np.zeros((nv.value, 3), np.float32)
    if L.spray_host_domain_mesh(desc.encode(), (ply_path or "").encode(), int(domain_id),
                                C.byref(nv), C.byref(nf), v.ctypes.data, f.ctypes.data,
                                c.ctypes.data, n.ctypes.data) != 0:
        raise SprayRtError("domain %d of %s failed to load" % (domain_id, desc))
    return v, f, c, n


class RtContext:
    """One engine context (one GPU).  ``owner=False`` wraps a context owned
    by a Scene."""

    def __init__(self, device=0, handle=None):
        self._own = handle is None
        if handle is None:
            h = C.c_void_p()
            rc = lib().spray_rt_create(int(device), C.byref(h))
            if rc != 0:
                raise SprayRtError("spray_rt_create(%d) failed: %d" % (device, rc))
            handle = h.value
        self.h = handle

    def close(self):
        if getattr(self, "h", None) and self._own:
            lib().spray_rt_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().spray_rt_last_error(self.h)
            raise SprayRtError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    # ---- context ----
    def set_stream(self, stream):
        """stream: torch.cuda.Stream, raw hipStream_t int, or None."""
        if stream is not None and hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        self._check(lib().spray_rt_set_stream(self.h, stream), "set_stream")

    def sync(self):
        self._check(lib().spray_rt_sync(self.h), "sync")

    RAYS_ADAPTIVE, RAYS_COHERENT, RAYS_INCOHERENT = 0, 1, 2

    def set_coherence(self, mode):
        """Traversal form of the any-hit launches (results are identical)."""
        self._check(lib().spray_rt_set_coherence(self.h, int(mode)), "set_coherence")

    # ---- domains ----
    def upload_domain(self, slot, verts, faces, colors=None, normals=None, async_=False):
        v = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
        f = np.ascontiguousarray(faces, np.uint32).reshape(-1, 3)
        c = None if colors is None else np.ascontiguousarray(colors, np.uint32)
        n = None if normals is None else np.ascontiguousarray(normals, np.float32)
        self._check(lib().spray_rt_domain_upload(
            self.h, int(slot), v.ctypes.data, len(v), f.ctypes.data, len(f),
            None if c is None else c.ctypes.data, None if n is None else n.ctypes.data,
            1 if async_ else 0), "domain_upload")

    def release_domain(self, slot):
        self._check(lib().spray_rt_domain_release(self.h, int(slot)), "domain_release")

    def domain_bounds(self, boxes):
        b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
        self._check(lib().spray_rt_domain_bounds(self.h, len(b), b.ctypes.data),
                    "domain_bounds")

    def map_domain(self, domain_id, slot):
        self._check(lib().spray_rt_map_domain(self.h, int(domain_id), int(slot)),
                    "map_domain")

    def slot_info(self, slot):
        nn, nt = C.c_size_t(), C.c_size_t()
        d = C.c_int()
        self._check(lib().spray_rt_slot_info(self.h, int(slot), C.byref(nn), C.byref(d),
                                             C.byref(nt)), "slot_info")
        return {"nodes": nn.value, "depth": d.value, "tris": nt.value}

    # ---- Embree-1M streams ----
    def intersect1M(self, slot, rays, stride=96):
        a, keep = _addr(rays)
        n = _nbytes(rays) // stride
        self._check(lib().spray_rt_intersect1M(self.h, int(slot), a, n, stride),
                    "intersect1M")

    def occluded1M(self, slot, rays, stride=96):
        a, keep = _addr(rays)
        n = _nbytes(rays) // stride
        self._check(lib().spray_rt_occluded1M(self.h, int(slot), a, n, stride),
                    "occluded1M")

    def _segments(self, fn, slots, offsets, rays, stride, what):
        s = np.ascontiguousarray(slots, np.int32)
        o = np.ascontiguousarray(offsets, np.uint64)
        assert len(o) == len(s) + 1
        a, keep = _addr(rays)
        self._check(fn(self.h, s.ctypes.data, o.ctypes.data, len(s), a, stride), what)

    def intersect_segments(self, slots, offsets, rays, stride=96):
        self._segments(lib().spray_rt_intersect_segments, slots, offsets, rays, stride,
                       "intersect_segments")

    def occluded_segments(self, slots, offsets, rays, stride=96):
        self._segments(lib().spray_rt_occluded_segments, slots, offsets, rays, stride,
                       "occluded_segments")

    def domains1M(self, org, dir, maxhits):
        org = np.ascontiguousarray(org, np.float32).reshape(-1, 3)
        dir = np.ascontiguousarray(dir, np.float32).reshape(-1, 3)
        n = len(org)
        ids = np.zeros((n, maxhits), np.int32)
        ts = np.zeros((n, maxhits), np.float32)
        cnt = np.zeros(n, np.int32)
        self._check(lib().spray_rt_domains1M(self.h, org.ctypes.data, dir.ctypes.data, n,
                                             ids.ctypes.data, ts.ctypes.data,
                                             cnt.ctypes.data, int(maxhits)), "domains1M")
        return ids, ts, cnt

    # ---- fused scene path ----
    def intersect_scene(self, rays, hits=None, counters=None):
        """rays: RAY_DTYPE numpy array or uint8/float torch tensor on the GPU
        (32 B per ray); hits: HIT_DTYPE array / 48-B-per-ray tensor."""
        n = _nbytes(rays) // 32
        if hits is None:
            hits = np.zeros(n, HIT_DTYPE)
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        c, k3 = _addr(counters)
        self._check(lib().spray_rt_intersect_scene_counted(self.h, a, n, b, c),
                    "intersect_scene")
        return hits

    def occluded_scene(self, rays, occ=None, counters=None):
        n = _nbytes(rays) // 32
        if occ is None:
            occ = np.zeros(n, np.uint8)
        a, k1 = _addr(rays)
        b, k2 = _addr(occ)
        c, k3 = _addr(counters)
        self._check(lib().spray_rt_occluded_scene_counted(self.h, a, n, b, c),
                    "occluded_scene")
        return occ

    def occluded_scene_masked(self, rays, valid, occ):
        """Any hit over the rays with valid[i] != 0 (device buffers)."""
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(valid)
        c, k3 = _addr(occ)
        self._check(lib().spray_rt_occluded_scene_masked(self.h, a, n, b, c),
                    "occluded_scene_masked")

    def intersect_scene_spawn_pt(self, rays, hits, shade, out_rays, out_valid, d_count=None):
        """Closest hit + fused positional PT shadow spawn (device buffers)."""
        n = _nbytes(rays) // 32
        shade = np.ascontiguousarray(shade, np.float32)
        assert shade.size == 10
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        c, k3 = _addr(out_rays)
        d, k4 = _addr(out_valid)
        e, k5 = _addr(d_count)
        self._check(lib().spray_rt_intersect_scene_spawn_pt(self.h, a, n, b, shade.ctypes.data,
                                                            c, d, e), "intersect_scene_spawn_pt")

    def intersect_scene_shadow_pt(self, rays, hits, shade, occ, sh_valid, d_count=None):
        """Closest hit + PT shadow spawn + the shadows' any hit, one launch
        (device buffers): sh_valid[i], occ[i] positional by source ray."""
        n = _nbytes(rays) // 32
        shade = np.ascontiguousarray(shade, np.float32)
        assert shade.size == 10
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        c, k3 = _addr(occ)
        d, k4 = _addr(sh_valid)
        e, k5 = _addr(d_count)
        self._check(lib().spray_rt_intersect_scene_shadow_pt(self.h, a, n, b, shade.ctypes.data,
                                                             c, d, e),
                    "intersect_scene_shadow_pt")

    def occluded_scene_devcount(self, rays, max_rays, d_count, occ, counters=None):
        a, k1 = _addr(rays)
        b, k2 = _addr(d_count)
        c, k3 = _addr(occ)
        e, k4 = _addr(counters)
        self._check(lib().spray_rt_occluded_scene_devcount(self.h, a, int(max_rays), b, c, e),
                    "occluded_scene_devcount")

    # ---- in-situ (domain-sharded) ----
    def set_owners(self, owner):
        """Domain -> rank map (InsituPartition::rank), host int array."""
        o = np.ascontiguousarray(owner, np.int32)
        self._check(lib().spray_rt_set_owners(self.h, o.ctypes.data), "set_owners")

    def route(self, rays, rank_mask):
        """rank_mask[i] (uint64 / int64 device tensor) = ranks owning a domain
        on ray i's list."""
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(rank_mask)
        self._check(lib().spray_rt_route(self.h, a, n, b), "route")

    def exchange_plan(self, rank_mask, world, idx, starts):
        """idx = per destination rank the ascending ray indices (device int64;
        None: bounds only); starts [world + 1] int64."""
        n = rank_mask.numel()
        a, k1 = _addr(rank_mask)
        b, k2 = _addr(idx)
        c, k3 = _addr(starts)
        self._check(lib().spray_rt_exchange_plan(self.h, a, n, int(world), b, c),
                    "exchange_plan")

    def gather_rows(self, src, idx, dst):
        """dst[j] = src[idx[j]] (device tensors, rows of 4/8/16/32/48 B)."""
        n = idx.numel()
        row = _nbytes(src) // src.shape[0] if src.shape[0] else 4
        a, k1 = _addr(src)
        b, k2 = _addr(idx)
        c, k3 = _addr(dst)
        self._check(lib().spray_rt_gather_rows(self.h, a, row, b, n, c), "gather_rows")

    def intersect_scene_keyed(self, rays, hits, keys):
        """Closest hit over the resident domains + composite key (device)."""
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        c, k3 = _addr(keys)
        self._check(lib().spray_rt_intersect_scene_keyed(self.h, a, n, b, c),
                    "intersect_scene_keyed")

    def eye_rays_insitu(self, cam, image_w, spp, block, stripe, rays, pixid=None,
                        samid=None):
        cam = np.ascontiguousarray(cam, np.float32)
        bx, by, bw, bh = block
        tx, ty, tw, th = stripe
        a, k1 = _addr(rays)
        b, k2 = _addr(pixid)
        c, k3 = _addr(samid)
        self._check(lib().spray_rt_eye_rays_insitu(self.h, cam.ctypes.data, int(image_w),
                                                   int(spp), bx, by, bw, bh, tx, ty, tw, th,
                                                   a, b, c), "eye_rays_insitu")

    # ---- device ray sources ----
    def eye_rays_ooc(self, cam, image_w, spp, tile, rays, pixid=None, samid=None):
        cam = np.ascontiguousarray(cam, np.float32)
        tx, ty, tw, th = tile
        a, k1 = _addr(rays)
        b, k2 = _addr(pixid)
        c, k3 = _addr(samid)
        self._check(lib().spray_rt_eye_rays_ooc(self.h, cam.ctypes.data, int(image_w),
                                                int(spp), tx, ty, tw, th, a, b, c),
                    "eye_rays_ooc")

    def spawn_shadows_ao(self, rays, hits, pixid, n, nsamples, out_rays, out_src, d_count,
                         order=None, traced=False):
        """ooc::ShaderAo rays (nsamples per hit), compacted (device); order
        (optional, uint32/int32 device tensor): their sample-major trace order;
        traced: the rays written in that trace order instead."""
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        p, k3 = _addr(pixid)
        c, k4 = _addr(out_rays)
        d, k5 = _addr(out_src)
        e, k6 = _addr(d_count)
        if traced:
            if order is not None:
                raise ValueError("traced spawn writes no order")
            self._check(lib().spray_rt_spawn_shadows_ao_traced(self.h, a, b, p, int(n),
                                                               int(nsamples), c, d, e),
                        "spawn_shadows_ao_traced")
            return
        if order is None:
            self._check(lib().spray_rt_spawn_shadows_ao(self.h, a, b, p, int(n), int(nsamples),
                                                        c, d, e), "spawn_shadows_ao")
            return
        o, k7 = _addr(order)
        self._check(lib().spray_rt_spawn_shadows_ao_ordered(self.h, a, b, p, int(n),
                                                            int(nsamples), c, d, e, o),
                    "spawn_shadows_ao_ordered")

    def occluded_scene_order(self, rays, max_rays, order, d_count, occ):
        """Any hit of rays order[j], j < *d_count; occ[order[j]] written (device;
        order None: rays 0 .. *d_count - 1)."""
        a, k1 = _addr(rays)
        o, k2 = _addr(order) if order is not None else (None, None)
        b, k3 = _addr(d_count)
        c, k4 = _addr(occ)
        self._check(lib().spray_rt_occluded_scene_order(self.h, a, int(max_rays), o, b, c),
                    "occluded_scene_order")

    def occluded_ao(self, rays, hits, pixid, n, nsamples, out_pairs, lv, rec, d_count, occ,
                    counters=None):
        """ooc::ShaderAo's spawn fused into the any hit (device): AO ray k of
        the sample-major trace order is sample out_pairs[k] & 31 of source ray
        out_pairs[k] >> 5; occ[k] its occlusion; *d_count rays.  The rays are
        made in the any-hit lanes, never stored; lv (float32, npix * nsamples
        * 4) holds the (pixel, sample) local hemisphere samples, rec (float32,
        n * 16) the source rays' origins and frames."""
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        p, k3 = _addr(pixid)
        c, k4 = _addr(out_pairs)
        d, k5 = _addr(lv)
        r, k9 = _addr(rec)
        e, k6 = _addr(d_count)
        f, k7 = _addr(occ)
        g, k8 = _addr(counters) if counters is not None else (None, None)
        self._check(lib().spray_rt_occluded_ao(self.h, a, b, p, int(n), int(nsamples),
                                               _lv_pixels(lv, nsamples), c, d, r, e, f, g),
                    "occluded_ao")

    def spawn_shadows_ao_pairs(self, rays, hits, pixid, n, nsamples, out_pairs, lv, rec,
                               d_count):
        """The traced AO spawn as (source << 5 | sample) pairs plus the
        (pixel, sample) local hemisphere samples lv and the source rays'
        origins / frames rec (device)."""
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        p, k3 = _addr(pixid)
        c, k4 = _addr(out_pairs)
        d, k5 = _addr(lv)
        r, k7 = _addr(rec)
        e, k6 = _addr(d_count)
        self._check(lib().spray_rt_spawn_shadows_ao_pairs(self.h, a, b, p, int(n), int(nsamples),
                                                          _lv_pixels(lv, nsamples), c, d, r, e),
                    "spawn_shadows_ao_pairs")

    def occluded_ao_pairs(self, max_n, pairs, rec, lv, nsamples, d_count, occ, counters=None):
        """Any hit of the AO rays of (source << 5 | sample) pairs, each
        generated in its lane from rec / lv (device); occ[k], k < *d_count."""
        c, k4 = _addr(pairs)
        r, k9 = _addr(rec)
        d, k5 = _addr(lv)
        e, k6 = _addr(d_count)
        f, k7 = _addr(occ)
        g, k8 = _addr(counters) if counters is not None else (None, None)
        self._check(lib().spray_rt_occluded_ao_pairs(self.h, int(max_n), c, r, d, int(nsamples),
                                                     e, f, g), "occluded_ao_pairs")

    # ---- frame layer (shading, film, tiles) ----
    def set_bsdfs(self, bsdfs):
        """Per-domain BSDFs: a sequence of (type, p0, p1, p2) (Scene::getBsdf)."""
        n = len(bsdfs)
        arr = (BsdfRec * max(n, 1))()
        for i, b in enumerate(bsdfs):
            arr[i].type = int(b[0])
            for k in range(3):
                arr[i].p[k] = float(b[1 + k])
        self._check(lib().spray_rt_set_bsdfs(self.h, n, C.addressof(arr) if n else None),
                    "set_bsdfs")

    def intersect_scene_masked(self, rays, valid, hits):
        """Closest hit of the rays with valid[i] != 0 (device buffers)."""
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(valid)
        c, k3 = _addr(hits)
        self._check(lib().spray_rt_intersect_scene_masked(self.h, a, n, b, c),
                    "intersect_scene_masked")

    def shade(self, shader, bounce, rays, hits, w, valid, pixid, samid, shadows, sw, svalid,
              stats=None):
        """One ShaderPt / ShaderAo pass over positional path slots (device)."""
        n = _nbytes(rays) // 32
        ptrs = [_addr(x) for x in (rays, hits, w, valid, pixid, samid, shadows, sw, svalid,
                                   stats)]
        a = [p[0] for p in ptrs]
        self._check(lib().spray_rt_shade(self.h, C.byref(shader), int(bounce), a[0], a[1], a[2],
                                         a[3], a[4], a[5], n, a[6], a[7], a[8], a[9]), "shade")

    def film(self, image, pixid, n, spp, ns, sw, svalid, occ, scale):
        """image[pixid] += scale * unoccluded shadow weights (device)."""
        ptrs = [_addr(x) for x in (image, pixid, sw, svalid, occ)]
        a = [p[0] for p in ptrs]
        self._check(lib().spray_rt_film(self.h, a[0], a[1], int(n), int(spp), int(ns), a[2],
                                        a[3], a[4], float(scale)), "film")

    def render_tile(self, shader, cam, image_w, spp, tile, image):
        """One tile of an ooc-mode frame, enqueued on the context's stream."""
        cam = np.ascontiguousarray(cam, np.float32)
        tx, ty, tw, th = (int(v) for v in tile)
        a, k1 = _addr(image)
        self._check(lib().spray_rt_render_tile(self.h, C.byref(shader), cam.ctypes.data,
                                               int(image_w), int(spp), tx, ty, tw, th, a),
                    "render_tile")

    def render_tiles(self, shader, cam, image_w, spp, tiles, image):
        """Tiles [(x, y, w, h)] of an ooc-mode frame as one device batch
        (the same image as render_tile per tile), enqueued on the stream."""
        cam = np.ascontiguousarray(cam, np.float32)
        t = np.ascontiguousarray(np.asarray(tiles, np.int32).reshape(-1, 4))
        a, k1 = _addr(image)
        self._check(lib().spray_rt_render_tiles(self.h, C.byref(shader), cam.ctypes.data,
                                                int(image_w), int(spp), t.ctypes.data,
                                                len(t), a), "render_tiles")

    def frame_stats(self, reset=True):
        """(radiance rays, shadow rays) traced by render_tile since the last
        reset (synchronises); raises on shading cases the reference aborts on."""
        out = (C.c_ulonglong * 3)()
        self._check(lib().spray_rt_frame_stats(self.h, out, int(bool(reset))), "frame_stats")
        return int(out[0]), int(out[1])

    def spawn_shadows_pt(self, rays, hits, n, shade, out_rays, out_src, d_count):
        shade = np.ascontiguousarray(shade, np.float32)
        assert shade.size == 10
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        c, k3 = _addr(out_rays)
        d, k4 = _addr(out_src)
        e, k5 = _addr(d_count)
        self._check(lib().spray_rt_spawn_shadows_pt(self.h, a, b, int(n), shade.ctypes.data,
                                                    c, d, e), "spawn_shadows_pt")


class OocCache:
    """Out-of-core domains (spray_rt_ooc_*): every domain image in pinned host
    memory, ``cache_slots`` of them resident in HBM at a time (LruCache)."""

    def __init__(self, rt, cache_slots):
        self.rt = rt
        h = C.c_void_p()
        rt._check(lib().spray_rt_ooc_create(rt.h, int(cache_slots), C.byref(h)), "ooc_create")
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib().spray_rt_ooc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_domain(self, domain_id, verts, faces, colors=None, normals=None):
        v = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
        f = np.ascontiguousarray(faces, np.uint32).reshape(-1, 3)
        c = None if colors is None else np.ascontiguousarray(colors, np.uint32)
        n = None if normals is None else np.ascontiguousarray(normals, np.float32)
        self.rt._check(lib().spray_rt_ooc_set_domain(
            self.h, int(domain_id), v.ctypes.data, len(v), f.ctypes.data, len(f),
            None if c is None else c.ctypes.data, None if n is None else n.ctypes.data),
            "ooc_set_domain")

    def intersect(self, rays, hits):
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(hits)
        self.rt._check(lib().spray_rt_ooc_intersect(self.h, a, n, b), "ooc_intersect")

    def occluded(self, rays, valid, occ):
        n = _nbytes(rays) // 32
        a, k1 = _addr(rays)
        b, k2 = _addr(valid)
        c, k3 = _addr(occ)
        self.rt._check(lib().spray_rt_ooc_occluded(self.h, a, n, b, c), "ooc_occluded")

    def stats(self):
        out = (C.c_ulonglong * 4)()
        self.rt._check(lib().spray_rt_ooc_stats(self.h, out), "ooc_stats")
        return {"loads": out[0], "hits": out[1], "bytes": out[2], "drains": out[3]}


def ooc_scene(desc, ply_path, cache_slots, device=0):
    """RtContext + OocCache over every domain of a scene file."""
    rt = RtContext(device)
    boxes, _ = host_parse_scene(desc, ply_path)
    rt.domain_bounds(boxes)
    oc = OocCache(rt, cache_slots)
    for d in range(len(boxes)):
        oc.set_domain(d, *host_domain_mesh(desc, ply_path, d))
    return rt, oc


class Scene:
    """GPU-backed scene (src/render/scene.h:62-251 surface)."""

    def __init__(self, desc, ply_path="", cache_size=-1, device=0):
        h = C.c_void_p()
        err = C.create_string_buffer(1024)
        rc = lib().spray_scene_create(desc.encode(), (ply_path or "").encode(),
                                      int(cache_size), int(device), C.byref(h), err, 1024)
        if rc != 0:
            raise SprayRtError("Scene(%s) failed (%d): %s" % (desc, rc, err.value.decode()))
        self.h = h.value
        self.rt = RtContext(handle=lib().spray_scene_rt(self.h))

    def close(self):
        if getattr(self, "h", None):
            lib().spray_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().spray_scene_last_error(self.h)
            raise SprayRtError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def getNumDomains(self):
        return lib().spray_scene_num_domains(self.h)

    def cache_capacity(self):
        return lib().spray_scene_cache_capacity(self.h)

    def domain_bounds(self):
        n = self.getNumDomains()
        boxes = np.zeros((n, 6), np.float32)
        bound = np.zeros(6, np.float32)
        lib().spray_scene_bounds(self.h, boxes.ctypes.data, bound.ctypes.data)
        return boxes, bound

    def getLights(self):
        out = []
        for i in range(lib().spray_scene_num_lights(self.h)):
            b = np.zeros(7, np.float32)
            lib().spray_scene_light(self.h, i, b.ctypes.data)
            out.append({"type": "point" if b[0] == 0 else "diffuse", "pos": b[1:4].copy(),
                        "rad": b[4:7].copy()})
        return out

    def load(self, domain_id):
        """Scene::load(id, SceneInfo*) -> cache block."""
        blk = C.c_int()
        self._check(lib().spray_scene_load(self.h, int(domain_id), C.byref(blk)), "load")
        return blk.value

    def intersect(self, cache_block, org, dir):
        """Scene::intersect for one ray -> (hit, RTC_ISECT_DTYPE record)."""
        rec = np.zeros(1, RTC_ISECT_DTYPE)
        o = np.asarray(org, np.float32)
        d = np.asarray(dir, np.float32)
        hit = lib().spray_scene_intersect1(self.h, int(cache_block), o.ctypes.data,
                                           d.ctypes.data, rec.ctypes.data)
        return bool(hit), rec[0]

    def occluded(self, cache_block, org, dir):
        rec = np.zeros(1, RTC_ISECT_DTYPE)
        o = np.asarray(org, np.float32)
        d = np.asarray(dir, np.float32)
        return bool(lib().spray_scene_occluded1(self.h, int(cache_block), o.ctypes.data,
                                                d.ctypes.data, rec.ctypes.data))

    def intersectDomains(self, org, dir, maxhits=None):
        """Sorted (ids, ts) per ray; org/dir [n,3]."""
        n = self.getNumDomains()
        ids, ts, cnt = self.rt.domains1M(org, dir, maxhits or n)
        return ids, ts, cnt

    def domain_mesh(self, domain_id):
        nv, nf = C.c_size_t(), C.c_size_t()
        self._check(lib().spray_scene_domain_mesh(self.h, int(domain_id), C.byref(nv),
                                                  C.byref(nf), None, None, None, None),
                    "domain_mesh")
        v = np.zeros((nv.value, 3), np.float32)
        f = np.zeros((nf.value, 3), np.uint32)
        c = np.zeros(nv.value, np.uint32)
        n = np.zeros((nv.value, 3), np.float32)
        self._check(lib().spray_scene_domain_mesh(self.h, int(domain_id), C.byref(nv),
                                                  C.byref(nf), v.ctypes.data, f.ctypes.data,
                                                  c.ctypes.data, n.ctypes.data),
                    "domain_mesh")
        return v, f, c, n
