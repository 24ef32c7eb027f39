# OOC-only kernel + copy trace of the bench's ooc leg.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-oocprof}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench.log" 2>&1
rc=$?; echo "rc=$rc"; find "$OUT/trace" -name "*stats.csv" | head
