"""Profile provenance of the bench line (no GPU): the committed PMC profile
names the library build it measured, and bench.roofline attaches its
traffic and ceilings only to a run of that very build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from spray_amd import build as spray_build  # noqa: E402

FUSED = "k_scene<1, false, false, 3, 16, 1>"


def _profile():
    with open(os.path.join(ROOT, "profiles", "pmc_counters.json")) as fh:
        return json.load(fh)


def test_profile_names_its_build_and_the_headline_kernel():
    pm = _profile()
    assert pm.get("build_id") and len(pm["build_id"]) == 16
    dv = pm["kernels"][FUSED]["derived"]
    # traffic from separate FETCH_SIZE / WRITE_SIZE passes, plus the launch's
    # occupancy over time (persistent waves)
    assert dv["traffic_bytes"] > 0
    assert 0.0 < dv["wave_life_frac"] <= 1.0
    assert summary_mentions(pm["round"], pm["build_id"])


def summary_mentions(tag, build_id):
    path = os.path.join(ROOT, "profiles", "%s_summary.md" % tag)
    with open(path) as fh:
        return build_id in fh.readline()


def test_roofline_attaches_traffic_only_for_the_profiled_build(monkeypatch):
    pm = _profile()
    args = (FUSED, 0.75e-3, 720347136, 8669238680, "index")
    monkeypatch.setattr(spray_build, "build_id", lambda: pm["build_id"])
    same = bench.roofline(*args)
    assert same["traffic"] and same["traffic"] > 0
    assert "ceilings" in same and same["bound"] == "latency"
    monkeypatch.setattr(spray_build, "build_id", lambda: "0" * 16)
    other = bench.roofline(*args)
    assert other["traffic"] is None
    assert other["traffic_source"].startswith("not attached")
