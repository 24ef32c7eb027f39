"""Where a small closest-hit launch's time goes (research tool, GPU): the
keyed closest hit of a rank's own eye rays (N = 8 partition, rank r, its 8
domains resident) over the first K packets, K from 1 to all -- the fixed
cost of a persistent launch vs. the latency of its heaviest packet walk vs.
throughput -- and the same over the whole-scene context.

    python scripts/launch_floor.py [rank] [close|rr]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from insitu_rank_kernels import CAM, H, SCENE, SCENES, SPP, W, timed  # noqa: E402


def main():
    rank = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    mode = sys.argv[2] if len(sys.argv) > 2 else "close"
    import torch
    import spray_amd
    from spray_amd import insitu
    from spray_amd.engine import host_parse_scene
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    boxes, _ = host_parse_scene(SCENE, SCENES)
    bound = np.concatenate([boxes[:, :3].min(0), boxes[:, 3:].max(0)])
    cam = spray_amd.camera_init(CAM["pos"], CAM["lookat"], CAM["up"], CAM["fov"], W, H)
    n = W * H * SPP
    rays = torch.empty((n, 8), dtype=torch.float32, device="cuda")
    pix = torch.empty(n, dtype=torch.int32, device="cuda")
    sam = torch.empty(n, dtype=torch.int32, device="cuda")
    sc = spray_amd.Scene(SCENE, SCENES, cache_size=-1)
    full = sc.rt
    full.set_stream(stream)
    full.eye_rays_insitu(cam, W, SPP, (0, 0, W, H), (0, 0, W, H), rays, pix, sam)
    full.set_coherence(full.RAYS_COHERENT)
    pm = insitu.PARTITION_ROUND_ROBIN if mode == "rr" else insitu.PARTITION_GROUP_CLOSE
    owner = insitu.morton_partition(boxes, bound, 8, pm)
    rt = spray_amd.RtContext(0)
    insitu.setup_rank_context(rt, SCENE, SCENES, owner, rank)
    rt.set_stream(stream)
    rt.set_coherence(rt.RAYS_COHERENT)
    m = torch.empty(n, dtype=torch.int64, device="cuda")
    rt.route(rays, m)
    lr = rays[((m >> rank) & 1).bool()].contiguous()
    nl = lr.shape[0]
    lh = torch.empty((nl, 12), dtype=torch.float32, device="cuda")
    lk = torch.empty(nl, dtype=torch.int64, device="cuda")
    print("rank %d (%s): %d own rays" % (rank, mode, nl), flush=True)
    for k in [64, 640, 6400, 64000, nl // 4, nl // 2, nl]:
        k = min(k, nl)
        t_own = timed(lambda: rt.intersect_scene_keyed(lr[:k], lh[:k], lk[:k]), reps=9)
        t_all = timed(lambda: full.intersect_scene_keyed(lr[:k], lh[:k], lk[:k]), reps=9)
        t_ch = timed(lambda: rt.intersect_scene(lr[:k], lh[:k]), reps=9)
        print("K %8d rays: own-domain keyed %.4f ms, all-domain keyed %.4f ms, own plain CH %.4f ms"
              % (k, t_own, t_all, t_ch), flush=True)
    # an empty index: the launch alone
    z = lr[:0]
    print("K 0: %.4f ms" % timed(lambda: rt.intersect_scene(lr[:1], lh[:1]), reps=9))
    rt.close()
    sc.close()


if __name__ == "__main__":
    main()
