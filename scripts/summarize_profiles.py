"""Condenses a scripts/gpu_profile.sh run into committed evidence.

    python scripts/summarize_profiles.py gpurun_out/<TAG> <round-tag>

Writes
* profiles/<tag>_kernel_stats.csv -- the rocprofv3 --kernel-trace --stats
  summary, verbatim;
* profiles/<tag>_pmc.csv -- every PMC counter, per kernel, averaged over its
  dispatches (raw rocprofv3 values);
* profiles/<tag>_summary.md -- per-kernel duration, HBM traffic and the
  derived ceilings below;
* profiles/pmc_counters.json -- the same per kernel, read by bench.py for the
  roofline's measured traffic and ceilings (labelled with <tag>).

Derived metrics (MI355X_MICROARCH.md):
* traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950 FETCH_SIZE
  counts half the bytes of wide reads: "HBM" section); Infinity-Cache hits
  are counted in FETCH_SIZE, so this is traffic beyond L2;
* cycles = GRBM_GUI_ACTIVE / 8 (one GRBM per XCD);
* VALU issue = SQ_INSTS_VALU x 2 / (cycles x 1024 SIMDs) (a wave64 VALU
  instruction issues over 2 cycles); SALU issue = SQ_INSTS_SALU / (cycles x
  256 CUs);
* L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS); L2 request bytes = TCC_REQ x 128 B
  (the L2 line; an upper bound of the bytes the L2 served);
* scalar-cache hit = SQC_DCACHE_HITS / SQC_DCACHE_REQ; TA busy =
  TA_BUSY_avr / cycles; VALU lane utilisation = SQ_THREAD_CYCLES_VALU /
  (64 x SQ_ACTIVE_INST_VALU); memory wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES;
  wave life = 4 x SQ_WAVE_CYCLES / SQ_WAVES / cycles (quad-cycle units; for
  a persistent launch the share of the launch its waves are alive).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK = 8.0e12
L2_PEAK = 34.5e12


def short(name):
    name = name.replace("spray_rt::(anonymous namespace)::", "").replace("void ", "")
    if "k_scene<" in name:
        return name[name.index("k_scene<"):name.index(">") + 1]
    return name.split("(")[0][:60]


def counters(src):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def derive(c, dur_s):
    d = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["traffic_bytes"] = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        if dur_s:
            d["hbm_frac"] = d["traffic_bytes"] / dur_s / HBM_PEAK
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
        d["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCC_REQ_sum" in c:
        d["l2_request_bytes"] = c["TCC_REQ_sum"] * 128
        if dur_s:
            d["l2_frac"] = d["l2_request_bytes"] / dur_s / L2_PEAK
    if cyc:
        d["cycles_per_xcd"] = cyc
        if "SQ_INSTS_VALU" in c:
            d["valu_issue"] = c["SQ_INSTS_VALU"] * 2 / (cyc * 1024)
        if "SQ_INSTS_SALU" in c:
            d["salu_issue"] = c["SQ_INSTS_SALU"] / (cyc * 256)
        if "TA_BUSY_avr" in c:
            d["ta_busy"] = c["TA_BUSY_avr"] / cyc
    if c.get("SQC_DCACHE_REQ"):
        d["scalar_cache_hit"] = c.get("SQC_DCACHE_HITS", 0) / c["SQC_DCACHE_REQ"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        d["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    if c.get("SQ_WAVE_CYCLES") and c.get("SQ_WAVES") and cyc:
        # mean wave lifetime over the launch (SQ_WAVE_CYCLES counts quad-cycles);
        # for the persistent launches, the share of the launch a wave is alive
        d["wave_life_frac"] = c["SQ_WAVE_CYCLES"] * 4 / c["SQ_WAVES"] / cyc
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                d[k.lower().replace("sq_", "") + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    return d


def main(src, tag):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats))) if os.path.exists(stats) else []
    if rows:
        shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    dur = {short(r["Name"]): float(r["AverageNs"]) * 1e-9 for r in rows}
    calls = {short(r["Name"]): r["Calls"] for r in rows}
    ctr = counters(src)
    names = sorted(set(ctr), key=lambda k: -dur.get(k, 0) * float(calls.get(k, 1) or 1))
    with open(os.path.join(prof, "%s_pmc.csv" % tag), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "value_per_dispatch"])
        for k in names:
            for c, v in sorted(ctr[k].items()):
                w.writerow([k, c, "%.6g" % v])
    # the build the profile measured (scripts/gpu_profile.sh copies the
    # library's build info next to the traces); bench.py attaches these
    # counters only to a library with the same build id
    binfo = os.path.join(src, "build.json")
    build_id = json.load(open(binfo)).get("build_id") if os.path.exists(binfo) else None
    out = {"round": tag, "source": src, "build_id": build_id, "kernels": {}}
    lines = ["# rocprofv3 summary, %s (library build %s)" % (tag, build_id), "",
             "Kernel trace: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 "
             "--warmup 5 --cpu-baseline 0`.  PMC: one `rocprofv3 --pmc <set>` pass per counter "
             "set of `bench.py --steps 2 --warmup 1 --cpu-baseline 0 --ooc 0 --frame 0 "
             "--insitu 0` (scripts/gpu_profile.sh); raw counters in `%s_pmc.csv`; derivations "
             "in scripts/summarize_profiles.py." % tag, "",
             "| kernel | calls | avg us | traffic B | HBM frac | L2 hit | L2 req frac | "
             "VALU issue | SALU issue | lane util | scalar hit | TA busy | mem wait | wave life |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]

    def f(x, fmt="%.3f"):
        return fmt % x if x is not None else "-"

    for k in names:
        dv = derive(ctr[k], dur.get(k))
        out["kernels"][k] = {"avg_us": dur.get(k, 0) * 1e6, "counters": ctr[k], "derived": dv}
        if not k.startswith("k_") or k not in dur:
            continue
        lines.append("| `%s` | %s | %.2f | %s | %s | %s | %s | %s | %s | %s | %s | %s | %s | %s |" % (
            k, calls.get(k, "-"), dur[k] * 1e6, f(dv.get("traffic_bytes"), "%.3e"),
            f(dv.get("hbm_frac")), f(dv.get("l2_hit")), f(dv.get("l2_frac")),
            f(dv.get("valu_issue")), f(dv.get("salu_issue")), f(dv.get("valu_lane_util")),
            f(dv.get("scalar_cache_hit")), f(dv.get("ta_busy")), f(dv.get("wait_any_frac")),
            f(dv.get("wave_life_frac"))))
    json.dump(out, open(os.path.join(prof, "pmc_counters.json"), "w"), indent=1)
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        js = [l for l in open(bench) if l.startswith("{")]
        if js:
            lines += ["", "bench line of the same run:", "", "```", js[-1].strip(), "```"]
            shutil.copy(bench, os.path.join(prof, "%s_bench.log" % tag))
    open(os.path.join(prof, "%s_summary.md" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
