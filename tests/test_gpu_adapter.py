"""The SceneT drop-in (include/spray_scene.hpp) driven the way the
reference's tracers drive Scene: a C++ mock ooc drain (tests/cpp/
scene_adapter_test.cpp, built by __graft_entry__.build()) with domain loads in
`omp single` and intersect / occluded / intersectDomains from every OpenMP
thread at once, each result bit-exact against the CPU oracle -- with every
domain resident and with a 4-block LRU cache that evicts while the threads
drain; the baseline tracers' scene-less forms (load(id), intersect(org, dir,
isect), occluded(org, dir, ray), updateIntersection); and the batched drain
(gather -> intersect1M / occluded1M -> scatter per thread and domain), whose
rate the test prints beside the per-ray form's."""
import os
import re
import subprocess

import pytest

from conftest import ROOT, SCENES, WAVELETS64

WAVELET2 = os.path.join(SCENES, "wavelet2.spray")

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "scene_adapter_test")


def _run(*args, timeout=240, scene=WAVELETS64):
    assert os.path.exists(BIN), "build it with __graft_entry__.build()"
    r = subprocess.run([BIN, scene, SCENES, *[str(a) for a in args]], capture_output=True,
                       text=True, timeout=timeout)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert " mismatches 0" in r.stdout
    return r.stdout


@pytest.mark.parametrize("threads,cache", [(8, -1), (16, 4), (1, 2)])
def test_scene_adapter_concurrent_drain(threads, cache):
    assert "domain-list mismatches 0" in _run(threads, cache)


@pytest.mark.parametrize("threads,cache", [(8, -1), (4, 4)])
def test_scene_adapter_current_domain_forms(threads, cache):
    """load(id) + the scene-less intersect / occluded and updateIntersection
    of the baseline tracers (scene.h:169-189, 203)."""
    _run(threads, cache, "current")


@pytest.mark.parametrize("threads,cache,img", [(1, -1, 512), (8, -1, 1024), (16, 4, 1024)])
def test_scene_adapter_batched_drain(threads, cache, img):
    """The batched drain from 1, 8 and 16 threads (1024x1024 camera rays at
    8 and 16), bit-exact against the oracle.  Prints its Mrays/s beside the
    per-ray form's and the CPU baseline of the same drain (the oracle's BVH
    over the same queues and shadow rays with the same thread count); at 8
    and 16 threads the GPU drain must beat that baseline."""
    out = _run(threads, cache, "batched", img, timeout=400)
    assert "domain-list mismatches 0" in out
    m = re.search(r"batched_Mrays_s ([\d.]+) per_ray_Mrays_s ([\d.]+).*oracle_Mrays_s ([\d.]+)",
                  out)
    assert m
    batched, per_ray, cpu = float(m.group(1)), float(m.group(2)), float(m.group(3))
    assert batched > per_ray
    if threads >= 8:
        assert batched > cpu, (batched, cpu)


@pytest.mark.parametrize("scene,threads,cache", [(WAVELETS64, 8, -1), (WAVELETS64, 16, 4),
                                                 (WAVELET2, 1, -1), (WAVELET2, 8, 1)])
def test_scene_adapter_app_types_shade(scene, threads, cache):
    """spray_amd::Scene<AppTypes> with the application's own Light / Bsdf /
    Aabb classes (tests/cpp/ref_mock.h): getLights() as std::vector<Light*>,
    getBsdf() as const Bsdf*, getBound() as Aabb, buildWbvh(), the in-situ
    partition's getDomains(rank) -- driven by a ShaderPt written with the
    reference's expressions inside the batched drain; every spawned shadow
    and continuation ray bit-exact against the oracle's ShaderPt, every
    shadow's occlusion against the oracle's BVH (wavelet2: a point light and
    a hemisphere area light)."""
    out = _run(threads, cache, "shade", 256, scene=scene)
    assert "scene-interface mismatches 0" in out
