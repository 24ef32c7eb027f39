# A/B of packet-walk variants (spray_amd/lib/diag/*.so) against the shipped
# library: the fused bench launch and its two-launch form (scripts/
# fused_shadow.py, two passes in alternating order), then the parity tests
# that run the packet walks, per variant.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pkt_ab}; mkdir -p "$OUT"
LIBS="shipped $(ls spray_amd/lib/diag/*.so)"
for pass in 1 2; do
  for L in $LIBS; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    echo "== pass $pass $L"
    timeout -k 10 200 python -u scripts/fused_shadow.py > "$OUT/t.log" 2>&1
    rc=$?; grep -v amdgpu.ids "$OUT/t.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
for L in $LIBS; do
  [ "${SKIP_PARITY:-0}" = 1 ] && break
  if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
  echo "== parity $L"
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_configs.py::test_config1_full_frame_fused_launch \
    tests/test_gpu_parity.py tests/test_gpu_ooc.py ${EXTRA_TESTS:-} > "$OUT/p.log" 2>&1
  rc=$?; tail -2 "$OUT/p.log"
  if [ $rc -ne 0 ]; then cp "$OUT/p.log" "$OUT/fail_$(basename $L).log"; exit $rc; fi
done
unset SPRAY_RT_LIB
for L in spray_amd/lib/wt/*.so; do
  [ -e "$L" ] || continue
  echo "== wave times $L"
  SPRAY_RT_LIB=$PWD/$L timeout -k 10 200 python -u scripts/wave_times.py > "$OUT/wt.log" 2>&1
  rc=$?; grep -v amdgpu.ids "$OUT/wt.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
