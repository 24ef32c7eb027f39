# Quantized nodes in the packet walks: GPU tests with the shipped library
# (packets over QNode), then the bench for shipped vs the fp32-node packet
# build (spray_amd/lib/diag/libspray_rt_fp32packet.so).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qp.log 2>&1 || { tail -30 gpurun_out/pytest_qp.log; exit 1; }
tail -2 gpurun_out/pytest_qp.log
for L in shipped spray_amd/lib/diag/libspray_rt_fp32packet.so shipped spray_amd/lib/diag/libspray_rt_fp32packet.so; do
  if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_qp.log 2>&1 || { tail -5 gpurun_out/bench_qp.log; exit 1; }
  tail -1 gpurun_out/bench_qp.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['ms_per_step'], j['kernels_ms'], 'ao', j['ao']['ms_per_step'], 'frame', j['frame']['ms_per_step'], 'ooc', j['ooc']['ms_per_step'])"
done
