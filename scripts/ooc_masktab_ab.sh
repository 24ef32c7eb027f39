# k_ooc_masks A/B: the shipped weight-table form against the LDS entry lists
# (SPRAY_OOC_MASK_TAB=0): per-pass kernel times (rocprofv3) and the drain
# schedule with its DomainStats scores (SPRAY_OOC_TRACE), which must match.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-masktab}
mkdir -p "$OUT"
for v in shipped ${VARS:-ooc_masktab0}; do
  L=""; [ "$v" != shipped ] && L="spray_amd/lib/diag/libspray_rt_$v.so"
  SPRAY_RT_LIB="$L" SPRAY_OOC_TRACE=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --frame 0 --ao 0 --insitu 0 --ooc 1 > "$OUT/${v}_trace.out" 2> "$OUT/${v}_trace.err"
  rc=$?; echo "$v trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/${v}_trace.err"; exit $rc; }
  grep -E "^ooc pass|^  launch" "$OUT/${v}_trace.err" > "$OUT/${v}_sched.txt" || true
  SPRAY_RT_LIB="$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --frame 0 --ao 0 --insitu 0 --ooc 1 > "$OUT/$v.log" 2>&1
  rc=$?; echo "$v prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/$v.log"; exit $rc; }
  python3 - "$OUT/$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_ooc_masks" in r["Kernel_Name"]]
print("  k_ooc_masks us: eye", [round(x) for x in d[0::2]], "shadow", [round(x) for x in d[1::2]])
PY
  grep '^{' "$OUT/$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('  ooc ms', d['ooc']['ms_per_step'])"
done
if cmp -s "$OUT/shipped_sched.txt" "$OUT/ooc_masktab0_sched.txt"; then echo "schedules identical ($(wc -l < $OUT/shipped_sched.txt) lines)"; else echo "SCHEDULES DIFFER"; diff "$OUT/shipped_sched.txt" "$OUT/ooc_masktab0_sched.txt" | head -20; fi
