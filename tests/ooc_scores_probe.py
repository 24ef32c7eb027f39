"""Subprocess of tests/test_gpu_ooc.py::test_ooc_queue_scores_match_domain_stats:
one closest-hit pass of the out-of-core path with SPRAY_OOC_TRACE=1 (the
drain schedule, with each queue's length and DomainStats score, on stderr;
the switch is read once per process, hence the subprocess).

    python tests/ooc_scores_probe.py case.npz slots

case.npz: org / dir (float32 [n, 3]) and either `desc` (a scene file) or
`v`, `f`, `c`, `shifts` (one mesh placed once per shift, overlapping)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import spray_amd
    from conftest import SCENES
    import insitu_helpers as H
    z = np.load(sys.argv[1])
    slots = int(sys.argv[2])
    if "desc" in z.files:
        rt, oc = spray_amd.engine.ooc_scene(str(z["desc"]), SCENES, slots)
    else:
        v, f, c, n, shifts = z["v"], z["f"], z["c"], z["n"], z["shifts"]
        boxes = np.stack([np.concatenate([(v + s).min(0), (v + s).max(0)]) for s in shifts])
        rt = spray_amd.RtContext(0)
        rt.domain_bounds(boxes.astype(np.float32))
        oc = spray_amd.OocCache(rt, slots)
        for k, s in enumerate(shifts):
            oc.set_domain(k, (v + s).astype(np.float32), f, c, n)
    rays = H.rays_tensor(z["org"], z["dir"]).cuda()
    hits = torch.empty((len(z["org"]), 12), dtype=torch.float32, device="cuda")
    oc.intersect(rays, hits)
    rt.sync()
    oc.close()
    rt.close()
    print("probe done")


if __name__ == "__main__":
    main()
