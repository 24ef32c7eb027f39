"""Per-rank kernel times of a camera-frame replay rehearsal from its
rocprofv3 kernel trace (rocpd database), for profiles/:

    rocprofv3 --kernel-trace -d <dir> -o run -- python3 scripts/camera_rehearse.py \
        --worlds 8 --modes view --frames F [--shader ao] ...
    python scripts/rank_kernel_table.py <dir>/run_results.db <F> <pt|ao> <world> > out.json

Each rank of the rehearsal runs 3 warm-up frames and 2 x F timed frames back
to back (camera_rehearse.py); frames are cut at their first kernel (the
keyed closest hit for PT, the eye-ray pass for AO) and a rank's kernels are
averaged over its last F frames (the ones timed without phase events)."""
import json
import sqlite3
import sys
from collections import OrderedDict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("spray_rt::", "")
    return n.split("(")[0].replace("void ", "")


def main(db, frames, kind, world):
    rows = sqlite3.connect(db).execute(
        "select name, start, end from kernels order by start").fetchall()
    anchor = "k_cam_eye_rays" if kind == "ao" else "k_scene<1, false, false, 6"
    idx = [i for i, r in enumerate(rows) if anchor in r[0]]
    per_rank = 3 + 2 * frames
    idx = idx[len(idx) - world * per_rank:]  # the ranks' frames (after the capture)
    out = []
    for rank in range(world):
        starts = idx[rank * per_rank:(rank + 1) * per_rank]
        ends = starts[1:] + [idx[(rank + 1) * per_rank] if rank + 1 < world else len(rows)]
        acc = OrderedDict()
        for a, b in list(zip(starts, ends))[-frames:]:
            for r in rows[a:b]:
                k = short(r[0])
                acc.setdefault(k, []).append((r[2] - r[1]) / 1000.0)
        out.append({"rank": rank,
                    "kernels_us": {k: [round(sum(v) / frames, 1), len(v) // frames]
                                   for k, v in acc.items()}})
    json.dump({"kind": kind, "world": world, "frames_averaged": frames,
               "note": "per rank: kernel -> [us per frame (summed over its calls), calls per frame]",
               "ranks": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]))
