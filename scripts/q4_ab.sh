# 4-wide any hit A/B: AO-16 leg of the bench for the shipped library and the
# diagnostic variants given in LIBS (spray_amd/lib/diag/*.so), alternated.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-q4ab}
mkdir -p "$OUT"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTFILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
for rep in 1 2; do
  for L in shipped ${LIBS:-}; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    n=$(basename $L .so)
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --ooc 0 --frame 0 --insitu 0 > "$OUT/bench_${n}_$rep.log" 2>&1 || { tail -5 "$OUT/bench_${n}_$rep.log"; exit 1; }
    python -c "
import json; l=[x for x in open('$OUT/bench_${n}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); a=d['ao']; print('$n', d['ms_per_step'], a['ms_per_step'], a['roofline']['avg_launch_ms'])"
  done
done
