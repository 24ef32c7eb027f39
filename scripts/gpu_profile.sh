# GPU round check: parity tests, smoke, bench, rocprofv3 kernel trace + PMC passes.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r1}
mkdir -p "$OUT"
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -rA
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3
step prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0
step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --ao 0 --ooc 0
step prof_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --ao 0 --ooc 0
step prof_l2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_l2" -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --ao 0 --ooc 0
echo done
