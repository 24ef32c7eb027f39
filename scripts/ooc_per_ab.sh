# OOC domains-per-launch A/B (SPRAY_OOC_PER): bench's ooc line only.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ooc_per}
mkdir -p "$OUT"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ooc.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
for rep in 1 2; do
  for p in ${PERS:-0 4}; do
    SPRAY_OOC_PER=$p timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_${p}_$rep.log" 2>&1 || { tail -5 "$OUT/bench_${p}_$rep.log"; exit 1; }
    python -c "
import json; l=[x for x in open('$OUT/bench_${p}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); o=d['ooc']; print('per=$p', o['ms_per_step'], o['loads_per_step'])"
  done
done
