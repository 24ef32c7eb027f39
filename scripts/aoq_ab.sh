# Variant A/B on the bench's headline and AO legs: optional parity of each
# variant in LIBS on the AO / quantized-node tests (PARITY=1), then the bench
# (no OOC / frame / in-situ legs) alternated with the shipped library.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aoq}; mkdir -p "$OUT"
LIBS=${LIBS:-$LIB}
if [ "${PARITY:-1}" = 1 ]; then
  for L in $LIBS; do
    SPRAY_RT_LIB=$PWD/$L timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_ao.py tests/test_gpu_qnodes.py > "$OUT/p.log" 2>&1
    rc=$?; echo "parity $L: $(tail -1 $OUT/p.log)"; [ $rc -ne 0 ] && { tail -30 "$OUT/p.log"; exit $rc; }
  done
fi
for rep in 1 2 3; do
  for L in shipped $LIBS; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --ooc 0 --frame 0 --insitu 0 > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
    python -c "
import json; l=[x for x in open('$OUT/b.log') if x.startswith('{')][-1]; d=json.loads(l); a=d['ao']; print('%-22s step %.4f fused %.4f ao %.4f ao any hit %.4f' % ('$(basename $L .so)', d['ms_per_step'], d['kernels_ms']['intersect_scene_shadow_pt'], a['ms_per_step'], a['roofline']['avg_launch_ms']))"
  done
done
