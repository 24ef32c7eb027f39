# A/B of the current tree: AO + parity tests, traversal-variant timing, AO trace orders.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ao.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/diag_variants.py run > "$OUT/variants.log" 2>&1
rc=$?; echo "variants rc=$rc"; cat "$OUT/variants.log" | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/ao_modes.py > "$OUT/ao_modes.log" 2>&1
rc=$?; echo "ao_modes rc=$rc"; cat "$OUT/ao_modes.log"
exit $rc
