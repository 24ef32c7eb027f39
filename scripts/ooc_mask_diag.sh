# k_ooc_masks part timings: the shipped library and the SPRAY_OOC_MASK_DIAG
# builds (1 no confirmation, 2 no per-block counts, 3 top-level walk only),
# each under a rocprofv3 kernel trace of the OOC bench leg.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-oocmask}
mkdir -p "$OUT"
for v in shipped ${VARS:-ooc_mask1 ooc_mask2 ooc_mask3}; do
  L=""; [ "$v" != shipped ] && L="spray_amd/lib/diag/libspray_rt_$v.so"
  SPRAY_RT_LIB="$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --frame 0 --ao 0 --insitu 0 --ooc 1 > "$OUT/$v.log" 2>&1
  rc=$?; echo "$v rc=$rc"
  [ $rc -ne 0 ] && { tail -20 "$OUT/$v.log"; exit $rc; }
  python3 - "$OUT/$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "ooc" in r["Name"]:
        print("  %-50s calls %5s avg %8.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
