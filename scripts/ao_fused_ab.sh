# AO: parity tests, then the fused (pairs + in-lane generation) vs written-ray step, then a kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aofused}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ao.py -v -rA --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for f in 1 0 1; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --frame 0 --insitu 0 --ooc 0 --cpu-baseline 0 --ao-fused $f > "$OUT/bench_$f.log" 2>&1 || exit $?
  python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_$f.log').read().strip().splitlines()[-1])
a=d['ao']; print('fused=$f ao ms', a['ms_per_step'], 'AH ms', a['roofline']['avg_launch_ms'], 'n_ao', a['ao_rays'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --frame 0 --insitu 0 --ooc 0 --cpu-baseline 0 > "$OUT/trace.log" 2>&1 || exit $?
python3 -c "
import csv,glob
for f in glob.glob('$OUT/trace/**/run_kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:12]:
        print('%10.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))
"
