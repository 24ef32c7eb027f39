#!/bin/bash
# GPU test suite on the box: pytest -m gpu (one process), a heartbeat file
# under gpurun_out/ while it runs (single full-size tests run for minutes
# without printing), then smoke().  Usage: scripts/gpu_suite.sh <tag> [pytest args]
tag=$1; shift
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/${tag}_heartbeat.txt; done ) &
hb=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 \
  --timeout-method thread "$@" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
kill $hb
tail -5 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
