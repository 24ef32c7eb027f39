"""Per-rank device time of the replicated frames' segments from the
rehearsal's rocprofv3 kernel traces (one CSV per process):

    rocprofv3 --kernel-trace --output-format csv -d DIR -o "%pid%/run" -- \
        python scripts/insitu_rep_rehearse.py --worlds 2 4 8 --kinds pt ao \
        --out R.json ...
    python scripts/rehearse_kernel_segments.py DIR R.json [--out seg.json]

Why not the rehearsal's HIP-event phases: the N processes' host-staged
collectives (gloo over tens of MB) leave the GPU idle for ~100 ms between a
rank's segments; its clocks drop, and the first launches after such a gap
run up to 4x slower (k_rep_cull 0.06 -> 1.7 ms, the AO any hit 3.8 -> 15.8
ms in the same process, with no other process's kernel overlapping them in
the trace).  A multi-GPU frame has gaps of tens of microseconds.  Here a
segment's time is the sum of its launches' durations (one stream: they
never overlap), each launch taken at its MINIMUM over the timed frames (a
frame issues the same launches in the same order on the same data), and
the launches whose work is identical on every rank (RANK_INDEPENDENT) at
their minimum over the ranks too.

Segments (the device work between two of the frame's collectives):
  pt: [cull + select + film slots + keyed closest hit & shading]
      [list positions + shadow any hit + winners + totals] [film]
  ao: [cull + select + keyed closest hit] [publish]
      [AO hits + spawn + own-pair select + any hit + count fields] [film]
A frame starts at k_rep_cull; a segment ends with its last launch (the
keyed k_scene launch, k_rep_totals, k_rep_ao_publish, k_rep_ao_scatter).
The host transport's staging copies (__amd_rocclr_copyBuffer; an RCCL
frame has none) and the harness's torch kernels are left out; the first
(warm-up) frame of each process is dropped.
"""
import argparse
import csv
import glob
import json
import os
import re

ENDS = {
    "pt": [lambda k: _epi(k) == 6, lambda k: "k_rep_totals" in k],
    "ao": [lambda k: _epi(k) == 6, lambda k: "k_rep_ao_publish" in k,
           lambda k: "k_rep_ao_scatter" in k],
}
NAMES = {"pt": ["cull_select_keyed", "shadow_winners", "film"],
         "ao": ["cull_select_keyed", "publish", "ao_spawn_trace", "film"]}


def _epi(name):
    m = re.search(r"k_scene<(\d+), (\w+), (\w+), (\d+),", name)
    return int(m.group(4)) if m else -1


# launches whose work is the same on every rank (the eye rays, C' and the
# published hits are identical everywhere): taken at their minimum over the
# ranks as well -- a rank that always resumes after the longest idle gap
# otherwise carries a clock-ramp artifact in every frame (k_rep_cull 0.06 vs
# 1.4 ms on one rank of a run)
RANK_INDEPENDENT = ("k_rep_cull", "k_select_count", "k_scan_blocks", "k_select_write",
                    "k_rep_heads", "k_rep_slot_pix", "init_lookback_scan_state",
                    "trampoline_kernel", "k_pix_bmax", "k_max_u32", "k_fill_u64",
                    "__amd_rocclr_fillBuffer", "k_rep_ao_hits", "k_spawn_ao_hitmask",
                    "k_spawn_ao_index")


def process(path, kind):
    """Per launch (segment, name, occurrence) of one rank: the minimum over
    the timed frames; and the number of timed frames."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    frames = []
    for r in rows:
        k = r["Kernel_Name"]
        if "k_rep_cull" in k:
            frames.append([])
        if not frames or "__amd_rocclr_copyBuffer" in k or "at::native" in k:
            continue
        frames[-1].append((k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    timed = frames[1:]
    if not timed:
        return None
    nl = min(len(f) for f in timed)
    seg, best, seen = 0, {}, {}
    for q in range(nl):
        k = timed[0][q][0]
        key = (min(seg, len(NAMES[kind]) - 1), k, seen.get((seg, k), 0))
        seen[(seg, k)] = key[2] + 1
        best[key] = min(f[q][1] for f in timed)
        if seg < len(ENDS[kind]) and ENDS[kind][seg](k):
            seg += 1
    return best, len(timed)


def segments(best, kind, floor):
    out = [0.0] * len(NAMES[kind])
    for key, dt in best.items():
        if any(p in key[1] for p in RANK_INDEPENDENT):
            dt = min(dt, floor.get(key, dt))
        out[key[0]] += dt
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("rehearse")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rep = json.load(open(args.rehearse))
    by_pid = {}
    for f in glob.glob(os.path.join(args.dir, "*", "*kernel_trace.csv")):
        by_pid[int(os.path.basename(os.path.dirname(f)))] = f
    runs = []
    for run in rep["runs"]:
        kind = run.get("kind", "pt")
        if kind not in NAMES:
            continue
        per = []
        for r in run["ranks"]:
            f = by_pid.get(r.get("pid"))
            res = process(f, kind) if f else None
            if res is None:
                per = None
                break
            per.append((r["rank"], res))
        if not per:
            continue
        floor = {}
        for _, (best, _) in per:
            for key, dt in best.items():
                floor[key] = min(dt, floor.get(key, dt))
        ranks = [{"rank": rk, "segments_ms": [round(x, 4) for x in segments(best, kind, floor)],
                  "frames": nf} for rk, (best, nf) in per]
        busiest = [round(max(x["segments_ms"][k] for x in ranks), 4)
                   for k in range(len(NAMES[kind]))]
        runs.append({"world": run["world"], "partition": run["partition"], "kind": kind,
                     "segments": NAMES[kind], "ranks": ranks,
                     "busiest_per_segment_ms": busiest, "device_ms": round(sum(busiest), 4)})
        print("%s N=%d %s: busiest %s = %.3f ms; per rank %s" % (
            kind, run["world"], run["partition"], " + ".join("%.3f" % x for x in busiest),
            sum(busiest), [round(sum(x["segments_ms"]), 3) for x in ranks]))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump({"method": __doc__.strip().split("\n\n")[2], "runs": runs}, fh, indent=1)


if __name__ == "__main__":
    main()
