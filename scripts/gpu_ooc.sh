# OOC check: parity tests, then the bench's ooc line only.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ooc}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ooc.py -v -rA --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json; l=[x for x in open('$OUT/bench.log') if x.startswith('{')][-1]; d=json.loads(l); print(d['ms_per_step'], json.dumps(d.get('ooc')))"
if [ "${AB:-0}" = 1 ]; then
  for w in lane packet; do
    SPRAY_BENCH_OOC_WALK=$w timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_$w.log" 2>&1 || exit $?
    python -c "
import json; l=[x for x in open('$OUT/bench_$w.log') if x.startswith('{')][-1]; d=json.loads(l); print('$w', json.dumps(d.get('ooc'))[:160])"
  done
fi
if [ "${TRACE:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 5 --warmup 2 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/trace.log" 2>&1
  echo "trace rc=$?"
fi
