"""Whole ooc-mode frames on the device: the film-mode render loop of
``SprayRenderer`` (src/render/spray_renderer.inl:352-380) over
``ooc::Tracer::trace`` (src/ooc/ooc_tracer.inl:184-234).

Per rank: the ooc tile schedule (``ImageScheduleTileList``, tile.cc:317-391:
the rank's vertical stripe cut into horizontal tiles); per tile, on the device
(``spray_rt_render_tile``, or all of them as one batch, ``spray_rt_render_tiles``): eye rays, then per bounce closest hit -> shading
(``ooc::ShaderPt`` / ``ooc::ShaderAo``) -> any hit of the shadow rays ->
film.  The ranks' images hold disjoint pixels, so the composite
(``HdrImage::composite``, image.h:170-186, an MPI_Reduce SUM) is one
``torch.distributed.reduce`` and exact.  ``write_ppm`` is
``HdrImage::writePpm`` (image.h:188-204).

Everything here runs through libspray_rt.so; the oracle restates it in
oracle/ for the tests only.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import (LIGHT_HEMISPHERE, LIGHT_POINT, MAX_LIGHTS, SHADER_AO, SHADER_PT,
                      ShaderRec, SprayRtError, lib)

__all__ = ["make_shader", "shadow_slots", "tile_list", "render_frame", "composite",
           "write_ppm", "SHADER_PT", "SHADER_AO", "LIGHT_POINT", "LIGHT_HEMISPHERE"]

# Config::maximum_num_screen_space_samples_per_rank (src/render/config.cc:66)
MAX_SAMPLES_PER_RANK = 1024 * 1024


def make_shader(kind="pt", bounces=1, samples=1, ks=(0.4, 0.4, 0.4), shininess=10.0,
                lights=()):
    """spray::Config shading fields + the scene's lights.  lights: rows of
    (type, x, y, z, r, g, b) as host_parse_scene returns them."""
    s = ShaderRec()
    s.shader = SHADER_AO if kind == "ao" else SHADER_PT
    s.bounces = int(bounces)
    s.samples = int(samples)
    lights = [tuple(l) for l in lights]
    if len(lights) > MAX_LIGHTS:
        raise ValueError("at most %d lights" % MAX_LIGHTS)
    s.nlights = len(lights)
    for k in range(3):
        s.ks[k] = float(ks[k])
    s.shininess = float(shininess)
    for i, l in enumerate(lights):
        s.lights[i].type = int(l[0])
        for k in range(3):
            s.lights[i].pos[k] = float(l[1 + k])
            s.lights[i].radiance[k] = float(l[4 + k])
    return s


def shadow_slots(shader):
    n = lib().spray_rt_shadow_slots(C.byref(shader))
    if n < 0:
        raise SprayRtError("bad shader configuration")
    return n


TILES = {"image": 0, "blocking": 1}


def tile_list(image_w, image_h, spp, nranks=1, rank=0, max_samples_per_rank=None,
              schedule="image"):
    """This rank's tiles [(x, y, w, h)]: "image" = ooc mode
    (ImageScheduleTileList), "blocking" = in-situ mode (TileList)."""
    ms = MAX_SAMPLES_PER_RANK if max_samples_per_rank is None else int(max_samples_per_rank)
    n = C.c_int()
    L = lib()
    sch = TILES[schedule]
    rc = L.spray_rt_tile_list(sch, int(image_w), int(image_h), int(spp), int(nranks), int(rank),
                              ms, None, 0, C.byref(n))
    if rc != 0:
        raise SprayRtError("tile_list failed (%d)" % rc)
    t = np.zeros((max(n.value, 1), 4), np.int32)
    rc = L.spray_rt_tile_list(sch, int(image_w), int(image_h), int(spp), int(nranks), int(rank),
                              ms, t.ctypes.data, n.value, C.byref(n))
    if rc != 0:
        raise SprayRtError("tile_list failed (%d)" % rc)
    return [tuple(int(v) for v in r) for r in t[:n.value]]


def render_frame(rt, shader, cam, image_w, image_h, spp, nranks=1, rank=0,
                 max_samples_per_rank=None, image=None, device="cuda", stats=True, batch=True):
    """One frame of this rank's tiles into a device float32 [h*w*4] image
    (cleared first, HdrImage::clear), enqueued on the context's stream.
    batch: all tiles as one device batch (spray_rt_render_tiles), else one
    render_tile per tile -- the same image.
    Returns (image, (radiance rays, shadow rays)) -- with stats=False the
    call does not synchronise and the counts are None."""
    import torch
    if image is None:
        image = torch.zeros(image_w * image_h * 4, dtype=torch.float32, device=device)
    else:
        image.zero_()
    tiles = [t for t in tile_list(image_w, image_h, spp, nranks, rank, max_samples_per_rank,
                                  "image") if t[2] * t[3]]
    if batch:
        rt.render_tiles(shader, cam, image_w, spp, tiles, image)
    else:
        for t in tiles:
            rt.render_tile(shader, cam, image_w, spp, t, image)
    return image, (rt.frame_stats() if stats else None)


def composite(image, dist=None):
    """HdrImage::composite: SUM of the ranks' images at rank 0."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(image, dst=0, op=dist.ReduceOp.SUM)
    return image


def write_ppm(path, rgba, w, h):
    """HdrImage::writePpm: P3, max 1023, bottom row first (host array)."""
    a = np.ascontiguousarray(np.asarray(rgba, np.float32).reshape(-1))
    if a.size != w * h * 4:
        raise ValueError("image must hold w*h*4 floats")
    if lib().spray_rt_write_ppm(str(path).encode(), a.ctypes.data, int(w), int(h)) != 0:
        raise SprayRtError("write_ppm(%s) failed" % path)
