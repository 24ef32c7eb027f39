set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-diag}
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/${TAG:-diag}/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG:-diag}/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python scripts/diag_variants.py run 2>&1 | tee gpurun_out/${TAG:-diag}/diag.log
