# PMC A/B of one bench leg: for each library (LIBS: name=path ... ; "default"
# = the shipped one) the counter passes below, one rocprofv3 run each, then
# per-kernel averages of the kernels matching KEYS.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcab}
mkdir -p "$OUT"
ARGS=${ARGS:-"--steps 2 --warmup 1 --cpu-baseline 0 --ooc 0 --frame 0 --insitu 0"}
PASSES=${PASSES:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS;GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"}
IFS=';' read -ra ALL <<< "$PASSES"
for spec in ${LIBS:-default=}; do
  name=${spec%%=*}; path=${spec#*=}
  i=0
  for set in "${ALL[@]}"; do
    i=$((i+1))
    if [ -n "$path" ]; then export SPRAY_RT_LIB="$GRAFT_REPO_ROOT/$path"; else unset SPRAY_RT_LIB; fi
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d "$OUT/$name/p$i" -o run -- python3 bench.py $ARGS > "$OUT/$name.p$i.log" 2>&1
    rc=$?; echo "$name pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.p$i.log"; exit $rc; fi
  done
done
unset SPRAY_RT_LIB
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
keys = os.environ.get("KEYS", "k_scene<1, true, false, 5").split(",")
for d in sorted(glob.glob(root + "/*/")):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("void ", "").replace("spray_rt::(anonymous namespace)::", "")
            if any(k in n for k in keys):
                agg[n[:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, c in agg.items():
        a = {k: sum(v) / len(v) for k, v in c.items()}
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8.0
        out = {}
        if cyc:
            out["valu_issue"] = a.get("SQ_INSTS_VALU", 0) * 2 / (cyc * 1024)
            out["salu_issue"] = a.get("SQ_INSTS_SALU", 0) / (cyc * 256)
            out["ta_busy"] = a.get("TA_BUSY_avr", 0) / cyc
        if a.get("SQ_ACTIVE_INST_VALU"):
            out["lane_util"] = a.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * a["SQ_ACTIVE_INST_VALU"])
        if a.get("SQ_WAVE_CYCLES"):
            out["wait_any"] = a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"]
            out["active_any"] = a.get("SQ_ACTIVE_INST_ANY", 0) / a["SQ_WAVE_CYCLES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "TCP_TOTAL_CACHE_ACCESSES_sum", "GRBM_GUI_ACTIVE"):
            if k in a: out[k] = a[k]
        print(os.path.basename(d.rstrip("/")), n, " ".join("%s=%.4g" % kv for kv in out.items()))
PY
