# The headline step timed in R separate bench.py processes (box variance):
#   R=3 TAG=<name> bash scripts/bench_repeats.sh
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-rep}; mkdir -p "$OUT"
for k in $(seq 1 ${R:-3}); do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --insitu 0 --ao 0 --frame 0 \
    --image 0 --ooc 0 --cpu-baseline 0 > "$OUT/b$k.json" 2>/dev/null || exit 1
  python3 - "$OUT/b$k.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], r["avg_launch_ms"], r["traffic"], r.get("traffic_source"))
PY
done
