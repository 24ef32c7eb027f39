"""Per-rank kernel breakdown of an image-parallel rehearsal trace
(scripts/trace_image_ranks.sh): the dispatches after the scene setup are cut
into ranks by the eye-ray kernel that opens each frame, the last 10 frames of
each rank kept, and the average duration per kernel and frame printed."""
import collections
import csv
import glob
import sys

out, world = sys.argv[1], int(sys.argv[2])
f = glob.glob(out + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
frames = []  # list of frames: [(name, dur_us)]
cur = None
for r in rows:
    name = r["Kernel_Name"]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_cam_eye_rays" in name or "k_eye_rays_insitu" in name:
        cur = []
        frames.append((int(r["Start_Timestamp"]), cur))
    if cur is not None:
        short = name.replace("void ", "").replace("(anonymous namespace)::", "")
        short = short.replace("spray_rt::", "").split("(")[0][:60]
        cur.append((short, dur, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
per = 13  # 3 warmup + 10 timed frames per rank
assert len(frames) >= world * per, (len(frames), world * per)
frames = frames[-world * per:]
for rank in range(world):
    fr = frames[rank * per + 3:(rank + 1) * per]
    acc = collections.defaultdict(float)
    span = 0.0
    for _, ks in fr:
        for name, d, _, _ in ks:
            acc[name] += d / len(fr)
        span += (ks[-1][3] - ks[0][2]) / 1e3 / len(fr)
    tot = sum(acc.values())
    print("rank %d: kernels %.1f us, first start -> last end %.1f us" % (rank, tot, span))
    for name, d in sorted(acc.items(), key=lambda kv: -kv[1]):
        print("   %-60s %8.1f us" % (name, d))
