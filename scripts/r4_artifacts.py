"""Round-4 evidence from one final GPU call (gpurun_out/<tag>: gpu_profile.sh
+ the REHKT rehearsal + rehearse_multi.sh N=8) into profiles/: the rocprof
summary, bench logs, the rehearsal JSON, per-rank segments, the projection
and the N = 8 ranks' trimmed kernel traces.

    python scripts/r4_artifacts.py r4i
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    py = sys.executable
    subprocess.run([py, os.path.join(ROOT, "scripts", "summarize_profiles.py"), src, tag],
                   check=True, stdout=subprocess.DEVNULL)
    shutil.copy(os.path.join(src, "bench.log"), os.path.join(prof, "%s_bench.log" % tag))
    shutil.copy(os.path.join(src, "bench_n8.log"), os.path.join(prof, "%s_rehearse_n8.log" % tag))
    rep = os.path.join(prof, "r4_rehearse.json")
    shutil.copy(os.path.join(src, "rehearse.json"), rep)
    seg = os.path.join(prof, "r4_rehearse_segments.json")
    subprocess.run([py, os.path.join(ROOT, "scripts", "rehearse_kernel_segments.py"),
                    os.path.join(src, "rehkt"), rep, "--out", seg], check=True,
                   stdout=subprocess.DEVNULL)
    out = subprocess.run([py, os.path.join(ROOT, "scripts", "insitu_rep_projection.py"), rep,
                          "--n1-ms", "0.770", "--n1-ao-ms", "4.70", "--kernels", seg, "--out",
                          os.path.join(prof, "r4_insitu_projection.json")],
                         check=True, capture_output=True, text=True).stdout
    with open(os.path.join(ROOT, "gpurun_out", "projection_%s.md" % tag), "w") as fh:
        fh.write(out)
    kd = os.path.join(prof, "r4_rehearse_kernels")
    shutil.rmtree(kd, ignore_errors=True)
    os.makedirs(kd)
    for run in json.load(open(rep))["runs"]:
        if run["world"] != 8:
            continue
        for r in run["ranks"]:
            f = glob.glob(os.path.join(src, "rehkt", str(r["pid"]), "*kernel_trace.csv"))[0]
            rows = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
            name = "%s_n8_%s_rank%d.csv" % (run["kind"], run["partition"], r["rank"])
            with open(os.path.join(kd, name), "w", newline="") as fh:
                w = csv.writer(fh)
                w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Duration_ns"])
                for x in rows:
                    w.writerow([x["Kernel_Name"][:120], x["Start_Timestamp"], x["End_Timestamp"],
                                int(x["End_Timestamp"]) - int(x["Start_Timestamp"])])
    print(out)


if __name__ == "__main__":
    main()
