# AO A/B: bash scripts/_ab_ao.sh <tag> <variant>
set -e
export TMPDIR=/tmp
tag=$1; var=$2
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 tests/test_gpu_ao.py tests/test_gpu_qnodes.py "tests/test_gpu_fullsize.py::test_ao16_full_frame_vs_oracle" > gpurun_out/$tag/tests.log 2>&1
B="python -u bench.py --steps 10 --warmup 3 --insitu 0 --frame 0 --ooc 0 --cpu-baseline 0"
for k in 1 2; do
  timeout -k 10 300 $B > gpurun_out/$tag/new$k.log 2>&1
  SPRAY_RT_LIB=$PWD/_ab/$var/libspray_rt.so timeout -k 10 300 $B > gpurun_out/$tag/old$k.log 2>&1
done
