# One PMC pass over a bench leg (ARGS: bench flags, KEYS: kernel-name filters;
# default the ooc leg), counters averaged per kernel and grid.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-oocpmc}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE} -d "$OUT/pmc" -o run --output-format csv -- python3 bench.py ${ARGS:---steps 1 --warmup 1 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0} > "$OUT/bench.log" 2>&1
rc=$?; echo "rc=$rc"
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("spray_rt::(anonymous namespace)::", "")[:40]
        if any(k in n for k in os.environ.get("KEYS", "ooc").split(",")):
            agg[(n, r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (n, g), d in sorted(agg.items()):
    print(n, g, " ".join("%s=%.3g" % (c, sum(v) / len(v)) for c, v in sorted(d.items())))
PY
