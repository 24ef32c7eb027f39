# SQ counters of the scene kernels (one pass per counter group).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sq}; mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
grep -o "SQ_[A-Z_0-9]*" "$OUT/avail.txt" | sort -u > "$OUT/sq_names.txt"; wc -l "$OUT/sq_names.txt"
BENCH="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --ao ${AO:-0} --ooc 0 --frame 0"
i=0
for G in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- $BENCH > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($G) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
