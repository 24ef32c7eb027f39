"""Per-kernel SQ/TCP/TCC counter table from a scripts/gpu_counters.sh run.

    python scripts/counter_table.py gpurun_out/<TAG>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    if "k_scene<" in name:
        return name[name.index("k_scene<"):name.index(">") + 1]
    return name.split("(")[0].replace("void ", "")[-50:]


def main(d):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, ctr in sorted(agg.items()):
        if not k.startswith("k_scene"):
            continue
        print(k)
        for c, v in sorted(ctr.items()):
            print("   %-28s %14.4g" % (c, sum(v) / len(v)))
        g = {c: sum(v) / len(v) for c, v in ctr.items()}
        if "SQ_INSTS_VALU" in g and "SQ_WAVES" in g:
            print("   valu insts / wave           %14.1f" % (g["SQ_INSTS_VALU"] / g["SQ_WAVES"]))
        if "SQ_THREAD_CYCLES_VALU" in g and "SQ_ACTIVE_INST_VALU" in g:
            print("   lane utilisation (VALU)     %14.3f" %
                  (g["SQ_THREAD_CYCLES_VALU"] / (64 * g["SQ_ACTIVE_INST_VALU"])))
        if "SQ_WAIT_ANY" in g and "SQ_WAVE_CYCLES" in g:
            print("   wait_any / wave_cycles      %14.3f" % (g["SQ_WAIT_ANY"] / g["SQ_WAVE_CYCLES"]))


if __name__ == "__main__":
    main(sys.argv[1])
