# Round-3 GPU check: the given pytest files (TESTS), then the bench (BENCH
# args), each step under its own time limit; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread $TESTS > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3
  [ $rc -ne 0 ] && { tail -40 "$OUT/tests.log"; exit $rc; }
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 ${BTIME:-400} python bench.py $BENCH > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"
  [ $rc -ne 0 ] && { tail -30 "$OUT/bench.log"; exit $rc; }
  python - "$OUT/bench.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("headline %.1f Mrays/s %.4f ms fused %.4f" % (d["value"], d["ms_per_step"], d["kernels_ms"]["intersect_scene_shadow_pt"]))
for k in ("insitu", "ao", "frame", "ooc"):
    if k in d:
        e = d[k]
        extra = (" any-hit %.4f ms" % e["roofline"]["avg_launch_ms"]) if "roofline" in e else ""
        print("%s %.1f Mrays/s %.4f ms%s" % (k, e["value"], e["ms_per_step"], extra))
PY
fi
