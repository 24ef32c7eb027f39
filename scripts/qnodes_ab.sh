# Quantized-node per-lane any hit: GPU tests with the shipped library, then
# the AO any-hit forms (scripts/ao_modes.py) for shipped vs the fp32-node
# build (spray_amd/lib/diag/libspray_rt_fp32nodes.so), then the bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
for L in shipped spray_amd/lib/diag/libspray_rt_fp32nodes.so; do
  if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 200 python -u scripts/ao_modes.py || exit 1
done
unset SPRAY_RT_LIB
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_q.log 2>&1 || { tail -5 gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log
