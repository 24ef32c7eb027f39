# OOC drain lag A/B (SPRAY_OOC_LAG = launches between a batch's launch and the counts it waits for)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ooclag}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ooc.py -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for lag in 1 2 3; do
  SPRAY_OOC_LAG=$lag timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_$lag.log" 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('$OUT/bench_$lag.log') if x.startswith('{')][-1]; d=json.loads(l)['ooc']; print('lag $lag', d['ms_per_step'], d['loads_per_step'])"
done
done
