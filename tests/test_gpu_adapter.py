"""The SceneT drop-in (include/spray_scene.hpp) driven the way the
reference's tracers drive Scene: a C++ mock ooc drain (tests/cpp/
scene_adapter_test.cpp, built by __graft_entry__.build()) with domain loads in
`omp single` and intersect / occluded / intersectDomains from every OpenMP
thread at once, each result bit-exact against the CPU oracle -- with every
domain resident and with a 4-block LRU cache that evicts while the threads
drain."""
import os
import subprocess

import pytest

from conftest import ROOT, SCENES, WAVELETS64

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "scene_adapter_test")


@pytest.mark.parametrize("threads,cache", [(8, -1), (16, 4), (1, 2)])
def test_scene_adapter_concurrent_drain(threads, cache):
    assert os.path.exists(BIN), "build it with __graft_entry__.build()"
    r = subprocess.run([BIN, WAVELETS64, SCENES, str(threads), str(cache)], capture_output=True,
                       text=True, timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    assert "mismatches 0" in r.stdout and "domain-list mismatches 0" in r.stdout
