"""Condenses a gpurun profiling directory into committed evidence.

    python scripts/summarize_profiles.py gpurun_out/r1k r1

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats
summary, verbatim), profiles/<round>_summary.md (per-kernel average duration,
PMC traffic per launch) and profiles/pmc_traffic.json (read by bench.py as
roofline.traffic).

HBM traffic per launch follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the bytes of wide
coalesced reads, so the corrected read bytes are 2 x FETCH_SIZE x 1024 (an
upper bound for this kernel's mix of 16-B and narrower loads; the raw value
is the lower bound, both are reported).  Infinity-Cache hits are counted in
FETCH_SIZE (the guide's caveat), so this is traffic beyond L2, not strictly
DRAM.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("spray_rt::(anonymous namespace)::", "").replace("void ", "")
    if "k_scene<" in name:
        return name[name.index("k_scene<"):name.index(">") + 1]
    return name.split("(")[0][:60]


def pmc(path):
    agg = defaultdict(list)
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return {}
    for r in csv.DictReader(open(f)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(src, tag):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", "%s_kernel_stats.csv" % tag))
    rows = list(csv.DictReader(open(stats)))
    fetch = pmc(os.path.join(src, "pmc_fetch"))
    write = pmc(os.path.join(src, "pmc_write"))
    l2 = pmc(os.path.join(src, "pmc_l2"))
    lines = ["# rocprofv3 summary, %s" % tag, "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 "
             "--warmup 3 --cpu-baseline 0` (trace), and separate `--pmc FETCH_SIZE`, "
             "`--pmc WRITE_SIZE`, `--pmc TCC_HIT_sum TCC_MISS_sum` passes of "
             "`bench.py --steps 3 --warmup 1 --cpu-baseline 0 --ao 0 --ooc 0` (scripts/gpu_profile.sh).", "",
             "| kernel | calls | avg us | FETCH_SIZE KiB | read bytes (x2 corr.) | "
             "WRITE_SIZE KiB | L2 hit |", "|---|---|---|---|---|---|---|"]
    traffic = {}
    for r in rows:
        k = short(r["Name"])
        fs = fetch.get((k, "FETCH_SIZE"))
        ws = write.get((k, "WRITE_SIZE"))
        h, m = l2.get((k, "TCC_HIT_sum")), l2.get((k, "TCC_MISS_sum"))
        hit = "%.3f" % (h / (h + m)) if h is not None and (h + m) > 0 else "-"
        rd = 2 * fs * 1024 if fs is not None else None
        lines.append("| `%s` | %s | %.2f | %s | %s | %s | %s |" % (
            k, r["Calls"], float(r["AverageNs"]) / 1e3,
            "%.0f" % fs if fs is not None else "-", "%.3e" % rd if rd else "-",
            "%.0f" % ws if ws is not None else "-", hit))
        if fs is not None and ws is not None:
            traffic[k] = {"fetch_kib": fs, "write_kib": ws,
                          "bytes_lower": fs * 1024 + ws * 1024,
                          "bytes_corrected": 2 * fs * 1024 + ws * 1024,
                          "avg_us": float(r["AverageNs"]) / 1e3}
    # the bench step's launch: the fused closest hit + shadow any hit (EPI 3),
    # else (older profiles) the closest hit with the fused spawn (EPI 1)
    ch = [v for k, v in traffic.items() if k.startswith("k_scene<1, false, false, 3,")]
    ch = ch or [v for k, v in traffic.items() if k.startswith("k_scene<1, false, false, 1,")]
    out = {"source": src, "round": tag, "per_kernel": traffic}
    if ch:
        out["scene_intersect_bytes_per_launch"] = ch[0]["bytes_corrected"]
        out["scene_intersect_bytes_per_launch_lower"] = ch[0]["bytes_lower"]
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        js = [l for l in open(bench) if l.startswith("{")]
        if js:
            lines += ["", "bench line of the same run:", "", "```", js[-1].strip(), "```"]
            shutil.copy(bench, os.path.join(ROOT, "profiles", "%s_bench.log" % tag))
    open(os.path.join(ROOT, "profiles", "%s_summary.md" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
