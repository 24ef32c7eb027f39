# Round-4 GPU call: optional pytest files (TESTS), the bench (BENCH args),
# A/B of diagnostic libraries (AB="name ..." from spray_amd/lib/diag), the
# replicated in-situ rehearsal (REHEARSE="worlds"), a rocprof kernel trace
# (PROF=1).  Every step under its own time limit; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4}
mkdir -p "$OUT"
fail() { echo "STOP: $1 rc=$2"; tail -40 "$3"; exit "$2"; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread $TESTS > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3
  [ $rc -ne 0 ] && fail tests $rc "$OUT/tests.log"
fi
summ() {
  python - "$1" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("headline %.1f Mrays/s %.4f ms fused %.4f" % (d["value"], d["ms_per_step"], d["kernels_ms"]["intersect_scene_shadow_pt"]))
for k in ("insitu", "insitu_protocol", "ao", "frame", "ooc"):
    if k in d:
        e = d[k]
        extra = (" any-hit %.4f ms" % e["roofline"]["avg_launch_ms"]) if "roofline" in e else ""
        ph = (" phases %s" % e["rank0_phases_ms"]) if "rank0_phases_ms" in e else ""
        print("%s %.1f Mrays/s %.4f ms%s%s" % (k, e["value"], e["ms_per_step"], extra, ph))
PY
}
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 ${BTIME:-400} python bench.py $BENCH > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"
  [ $rc -ne 0 ] && fail bench $rc "$OUT/bench.log"
  summ "$OUT/bench.log"
fi
for v in ${AB:-}; do
  for rep in 1 2; do
    for lib in shipped "$v"; do
      if [ "$lib" = shipped ]; then L=""; else L="spray_amd/lib/diag/libspray_rt_$lib.so"; fi
      SPRAY_RT_LIB="$L" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --frame 0 --ooc ${ABOOC:-0} --ao ${ABAO:-0} --insitu 0 > "$OUT/ab_${lib}_$rep.log" 2>&1
      rc=$?
      [ $rc -ne 0 ] && fail "ab $lib" $rc "$OUT/ab_${lib}_$rep.log"
      echo -n "ab $lib #$rep: "; summ "$OUT/ab_${lib}_$rep.log" | tr '\n' ' '; echo
    done
  done
done
if [ -n "${REHEARSE:-}" ]; then
  # REHKT=1: under a per-process rocprofv3 kernel trace (rehearse_kernel_segments.py)
  PRE=""
  [ "${REHKT:-0}" = 1 ] && PRE="rocprofv3 --kernel-trace --output-format csv -d $OUT/rehkt -o %pid%/run --"
  timeout -k 10 ${RTIME:-600} $PRE python -u scripts/insitu_rep_rehearse.py --worlds $REHEARSE --modes ${MODES:-close rr} --kinds ${KINDS:-pt} --frames ${FRAMES:-3} --out "$OUT/rehearse.json" > "$OUT/rehearse.log" 2>&1
  rc=$?; echo "rehearse rc=$rc"; tail -12 "$OUT/rehearse.log"
  [ $rc -ne 0 ] && fail rehearse $rc "$OUT/rehearse.log"
fi
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > "$OUT/prof.log" 2>&1
  rc=$?; echo "prof rc=$rc"
  [ $rc -ne 0 ] && fail prof $rc "$OUT/prof.log"
fi
echo done
# rocprof kernel trace of one rehearsal configuration (REHPROF="world mode kind")
if [ -n "${REHPROF:-}" ]; then
  set -- $REHPROF
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/rehprof" -o "%pid%/run" -- python -u scripts/insitu_rep_rehearse.py --worlds $1 --modes $2 --kinds $3 --frames 3 --rccl-floor 0 --out "$OUT/rehprof.json" > "$OUT/rehprof.log" 2>&1
  rc=$?; echo "rehprof rc=$rc"
  [ $rc -ne 0 ] && fail rehprof $rc "$OUT/rehprof.log"
fi
echo done2
