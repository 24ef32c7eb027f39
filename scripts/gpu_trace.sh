# Kernel-trace summary of one bench run: TAG=<name> ARGS="<bench args>" bash scripts/gpu_trace.sh
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 bench.py ${ARGS:---steps 5 --warmup 2 --cpu-baseline 0} > "$OUT/bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 "$OUT/bench.log"
python3 - "$OUT" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:25]:
    print("%-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
