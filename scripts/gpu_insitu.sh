# GPU check of the engine's in-situ tracer: tests, then a short bench of the insitu line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-insitu}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_insitu.py -v -rA --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --ao 0 --frame 0 --ooc 0 --cpu-baseline 0 > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench.log"
if [ "${TRACE:-0}" = 1 ] && [ $rc -eq 0 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 5 --warmup 2 --ao 0 --frame 0 --ooc 0 --cpu-baseline 0 > "$OUT/trace.log" 2>&1
  echo "trace rc=$?"
fi
