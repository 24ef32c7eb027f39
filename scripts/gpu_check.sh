# GPU tests of the given files + the default bench + the image rehearsal:
#   TAG=<name> TESTS="tests/a.py tests/b.py" bash scripts/gpu_check.sh
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-check}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests} -m gpu > "$OUT/test.log" 2>&1 || { tail -30 "$OUT/test.log"; exit 1; }
tail -2 "$OUT/test.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])
for k in ("insitu", "insitu_protocol", "image_parallel", "frame", "ao", "ooc"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, v.get("value"), v.get("ms_per_step"))
PY
[ "${REH:-1}" = 1 ] || exit 0
timeout -k 10 300 python -u scripts/image_rehearse.py --worlds 1 2 4 8 --bands ${BANDS:-1 4} --out "$OUT/rehearse.json" > "$OUT/rehearse.txt" 2>&1 || { tail -20 "$OUT/rehearse.txt"; exit 1; }
cat "$OUT/rehearse.txt"
