"""ctypes binding of libspray_rt.so (include/spray_rt.h, include/spray_scene.h).

The library is the product: gfx950 kernels + C ABI + host scene layer.  There
is no fallback -- if the shared object is missing or fails to load, import of
the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SPRAY_RT_LIB selects another build of the engine (A/B runs of
# spray_amd.build.build(defines=..., out=...)); the default is the in-tree
# engine.
LIB_PATH = os.environ.get("SPRAY_RT_LIB") or os.path.join(HERE, "lib", "libspray_rt.so")

# record layouts (include/spray_rt.h)
RAY_DTYPE = np.dtype([("org", "<f4", 3), ("tnear", "<f4"), ("dir", "<f4", 3),
                      ("tfar", "<f4")])
HIT_DTYPE = np.dtype([("t", "<f4"), ("u", "<f4"), ("v", "<f4"), ("prim", "<u4"),
                      ("ng", "<f4", 3), ("color", "<u4"), ("ns", "<f4", 3),
                      ("domain", "<i4")])
RTC_ISECT_DTYPE = np.dtype([("org", "<f4", 3), ("align0", "<f4"), ("dir", "<f4", 3),
                            ("align1", "<f4"), ("tnear", "<f4"), ("tfar", "<f4"),
                            ("time", "<f4"), ("mask", "<u4"), ("Ng", "<f4", 3),
                            ("color", "<u4"), ("u", "<f4"), ("v", "<f4"),
                            ("geomID", "<u4"), ("primID", "<u4"), ("instID", "<u4"),
                            ("Ns", "<f4", 3)])
assert RAY_DTYPE.itemsize == 32 and HIT_DTYPE.itemsize == 48
assert RTC_ISECT_DTYPE.itemsize == 96

INVALID_ID = 0xFFFFFFFF

# frame-layer records (include/spray_rt.h)
SHADER_PT, SHADER_AO = 0, 1
LIGHT_POINT, LIGHT_HEMISPHERE = 0, 1
BSDF_DIFFUSE, BSDF_MIRROR, BSDF_GLASS, BSDF_TRANSMISSION = 0, 1, 2, 3
MAX_LIGHTS = 8


class LightRec(C.Structure):
    _fields_ = [("type", C.c_int32), ("pos", C.c_float * 3), ("radiance", C.c_float * 3)]


class BsdfRec(C.Structure):
    _fields_ = [("type", C.c_int32), ("p", C.c_float * 3)]


class ShaderRec(C.Structure):
    _fields_ = [("shader", C.c_int32), ("bounces", C.c_int32), ("samples", C.c_int32),
                ("nlights", C.c_int32), ("ks", C.c_float * 3), ("shininess", C.c_float),
                ("lights", LightRec * MAX_LIGHTS)]


assert C.sizeof(LightRec) == 28 and C.sizeof(BsdfRec) == 16
assert C.sizeof(ShaderRec) == 32 + 28 * MAX_LIGHTS

# every symbol the public headers declare: (restype, argtypes)
P = C.c_void_p
SZ = C.c_size_t
I = C.c_int
SIGNATURES = {
    # spray_rt.h
    "spray_rt_create": (I, [I, P]),
    "spray_rt_destroy": (I, [P]),
    "spray_rt_last_error": (C.c_char_p, [P]),
    "spray_rt_set_stream": (I, [P, P]),
    "spray_rt_sync": (I, [P]),
    "spray_rt_domain_upload": (I, [P, I, P, SZ, P, SZ, P, P, I]),
    "spray_rt_domain_release": (I, [P, I]),
    "spray_rt_domain_bounds": (I, [P, I, P]),
    "spray_rt_map_domain": (I, [P, I, I]),
    "spray_rt_slot_info": (I, [P, I, P, P, P]),
    "spray_rt_bvh_build_host": (I, [P, SZ, P, SZ, P, P, P, P, P]),
    "spray_rt_qnodes_host": (I, [P, SZ, P, SZ, P, P, P]),
    "spray_rt_qnodes4_host": (I, [P, SZ, P, SZ, P, P, P, P]),
    "spray_rt_intersect1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_occluded1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_intersect_segments": (I, [P, P, P, I, P, SZ]),
    "spray_rt_occluded_segments": (I, [P, P, P, I, P, SZ]),
    "spray_rt_domains1M": (I, [P, P, P, SZ, P, P, P, I]),
    "spray_rt_intersect_scene": (I, [P, P, SZ, P]),
    "spray_rt_occluded_scene": (I, [P, P, SZ, P]),
    "spray_rt_intersect_scene_counted": (I, [P, P, SZ, P, P]),
    "spray_rt_occluded_scene_counted": (I, [P, P, SZ, P, P]),
    "spray_rt_occluded_scene_devcount": (I, [P, P, SZ, P, P, P]),
    "spray_rt_intersect_scene_spawn_pt": (I, [P, P, SZ, P, P, P, P, P]),
    "spray_rt_occluded_scene_masked": (I, [P, P, SZ, P, P]),
    "spray_rt_intersect_scene_shadow_pt": (I, [P, P, SZ, P, P, P, P, P]),
    "spray_rt_eye_rays_ooc": (I, [P, P, I, I, I, I, I, I, P, P, P]),
    "spray_rt_eye_rays_insitu": (I, [P, P, I, I, I, I, I, I, I, I, I, I, P, P, P]),
    "spray_rt_set_owners": (I, [P, P]),
    "spray_rt_gather_rows": (I, [P, P, SZ, P, SZ, P]),
    "spray_rt_exchange_plan": (I, [P, P, SZ, I, P, P]),
    "spray_rt_set_coherence": (I, [P, I]),
    "spray_rt_spawn_shadows_ao": (I, [P, P, P, P, SZ, I, P, P, P]),
    "spray_rt_spawn_shadows_ao_ordered": (I, [P, P, P, P, SZ, I, P, P, P, P]),
    "spray_rt_spawn_shadows_ao_traced": (I, [P, P, P, P, SZ, I, P, P, P]),
    "spray_rt_occluded_scene_order": (I, [P, P, SZ, P, P, P]),
    "spray_rt_occluded_ao": (I, [P, P, P, P, SZ, I, SZ, P, P, P, P, P, P]),
    "spray_rt_spawn_shadows_ao_pairs": (I, [P, P, P, P, SZ, I, SZ, P, P, P, P]),
    "spray_rt_occluded_ao_pairs": (I, [P, SZ, P, P, P, I, P, P, P]),
    "spray_rt_ooc_create": (I, [P, I, P]),
    "spray_rt_ooc_destroy": (I, [P]),
    "spray_rt_ooc_set_domain": (I, [P, I, P, SZ, P, SZ, P, P]),
    "spray_rt_ooc_intersect": (I, [P, P, SZ, P]),
    "spray_rt_ooc_occluded": (I, [P, P, SZ, P, P]),
    "spray_rt_ooc_stats": (I, [P, P]),
    "spray_rt_route": (I, [P, P, SZ, P]),
    "spray_rt_intersect_scene_keyed": (I, [P, P, SZ, P, P]),
    "spray_rt_spawn_shadows_pt": (I, [P, P, P, SZ, P, P, P, P]),
    "spray_rt_set_bsdfs": (I, [P, I, P]),
    "spray_rt_shadow_slots": (I, [P]),
    "spray_rt_intersect_scene_masked": (I, [P, P, SZ, P, P]),
    "spray_rt_shade": (I, [P, P, I, P, P, P, P, P, P, SZ, P, P, P, P]),
    "spray_rt_film": (I, [P, P, P, SZ, I, I, P, P, P, C.c_double]),
    "spray_rt_render_tile": (I, [P, P, P, I, I, I, I, I, I, P]),
    "spray_rt_render_tiles": (I, [P, P, P, I, I, P, I, P]),
    "spray_rt_frame_stats": (I, [P, P, I]),
    "spray_rt_tile_list": (I, [I, I, I, I, I, I, C.c_longlong, P, I, P]),
    "spray_rt_write_ppm": (I, [C.c_char_p, P, I, I]),
    "spray_rt_lane_create": (I, [P, P]),
    "spray_rt_lane_create_error": (C.c_char_p, []),
    "spray_rt_lane_update_intersection1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_update_intersection1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_lane_destroy": (I, [P]),
    "spray_rt_lane_last_error": (C.c_char_p, [P]),
    "spray_rt_lane_intersect1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_lane_occluded1M": (I, [P, I, P, SZ, SZ]),
    "spray_rt_lane_domains1M": (I, [P, P, P, SZ, P, P, P, I]),
    "spray_rt_insitu_unique_id": (I, [P, SZ]),
    "spray_rt_insitu_create": (I, [P, I, I, P, P, P]),
    "spray_rt_insitu_destroy": (I, [P]),
    "spray_rt_insitu_partition": (I, [P, I, P, I, P]),
    "spray_rt_insitu_partition_mode": (I, [P, I, P, I, I, P]),
    "spray_rt_insitu_trace": (I, [P, P, P, P, P, SZ, I, P, P, P]),
    "spray_rt_insitu_trace_frame": (I, [P, P, P, P, P, SZ, I, P, P, P]),
    "spray_rt_insitu_trace_camera": (I, [P, P, P, I, I, I, P, P, P]),
    "spray_rt_insitu_trace_image": (I, [P, P, P, I, I, I, I, P, P, P]),
    "spray_rt_insitu_partition_view": (I, [P, I, P, I, P]),
    "spray_rt_insitu_create_replay": (I, [P, I, I, P]),
    "spray_rt_insitu_replay_set": (I, [P, P, P, SZ]),
    "spray_rt_insitu_replay_capture": (I, [P, P, P, SZ, P]),
    "spray_rt_insitu_replay_set_ao": (I, [P, P, P, SZ]),
    "spray_rt_insitu_replay_capture_ao": (I, [P, P, P, SZ, P]),
    "spray_rt_insitu_replay_bits_ao": (I, [P, P, P, SZ, P]),
    "spray_rt_camera_box_rows": (I, [P, I, I, P, P, P]),
    "spray_rt_camera_shadow_boxes": (I, [P, P, P, I, P]),
    "spray_rt_insitu_set_timing": (I, [P, I]),
    "spray_rt_insitu_phase_times": (I, [P, P, P]),
    "spray_rt_insitu_composite": (I, [P, P, SZ]),
    "spray_rt_insitu_stats": (I, [P, P]),
    "spray_rt_insitu_collective_log": (I, [P, P, SZ, P, I]),
    # spray_scene.h
    "spray_scene_create": (I, [C.c_char_p, C.c_char_p, I, I, P, C.c_char_p, SZ]),
    "spray_scene_destroy": (I, [P]),
    "spray_scene_last_error": (C.c_char_p, [P]),
    "spray_scene_rt": (P, [P]),
    "spray_scene_num_domains": (I, [P]),
    "spray_scene_cache_capacity": (I, [P]),
    "spray_scene_bounds": (I, [P, P, P]),
    "spray_scene_num_lights": (I, [P]),
    "spray_scene_light": (I, [P, I, P]),
    "spray_scene_load": (I, [P, I, P]),
    "spray_scene_intersect1": (I, [P, I, P, P, P]),
    "spray_scene_occluded1": (I, [P, I, P, P, P]),
    "spray_camera_init": (I, [P, P, P, C.c_float, I, I, P]),
    "spray_scene_domain_mesh": (I, [P, I, P, P, P, P, P, P]),
    "spray_host_parse_scene": (I, [C.c_char_p, C.c_char_p, P, P, P, P, P, C.c_char_p, SZ]),
    "spray_host_scene_bsdfs": (I, [C.c_char_p, P, P, C.c_char_p, SZ]),
    "spray_host_domain_mesh": (I, [C.c_char_p, C.c_char_p, I, P, P, P, P, P, P]),
}

_lib = None


class SprayRtError(RuntimeError):
    pass


def lib():
    """Loads libspray_rt.so; raises if it is absent (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "spray_amd: %s is missing -- build it with `python -m spray_amd.build` "
                "(there is no CPU fallback)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("SPRAY_RT_LIB") and not hasattr(L, name):
                continue  # an A/B build that predates the symbol (never the in-tree library)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib
