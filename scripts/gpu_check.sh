# GPU check: parity tests, smoke, short bench (one call, each step time-limited).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-6} "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
  return 0
}
step pytest_gpu ${PYT_TO:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v -rA --timeout 180 --timeout-method thread
[ "${SMOKE:-1}" = 1 ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${BENCH:-1}" = 1 ] && step bench 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 5
echo done
