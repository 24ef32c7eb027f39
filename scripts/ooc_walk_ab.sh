# OOC any-hit drain walk A/B: packets vs the per-wave choice (id span + direction)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-oocwalk}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ooc.py -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
SPRAY_OOC_AH_ADAPTIVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ooc.py -q --timeout 120 --timeout-method thread > "$OUT/pytest_ad.log" 2>&1
rc=$?; echo "pytest adaptive rc=$rc"; tail -1 "$OUT/pytest_ad.log"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for ad in 0 1; do
  SPRAY_OOC_AH_ADAPTIVE=$ad timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_$ad.log" 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('$OUT/bench_$ad.log') if x.startswith('{')][-1]; d=json.loads(l)['ooc']; print('adaptive $ad', d['ms_per_step'])"
done
done
