"""spray_amd -- MI355X-native BVH traversal + ray/triangle intersection engine
behind SpRay's scene intersect/occluded surface.

The engine is libspray_rt.so (hand-written gfx950 HIP kernels + C ABI, see
include/spray_rt.h and include/spray_scene.h); this package is its Python
binding.  There is no CPU fallback.
"""
from .engine import (HIT_DTYPE, INVALID_ID, RAY_DTYPE, RTC_ISECT_DTYPE, OocCache,
                     RtContext, Scene, SprayRtError, camera_init, make_rays, ooc_scene)
from . import frame

__all__ = ["RtContext", "Scene", "OocCache", "ooc_scene", "SprayRtError", "camera_init",
           "make_rays", "RAY_DTYPE", "HIT_DTYPE", "RTC_ISECT_DTYPE", "INVALID_ID", "frame"]
