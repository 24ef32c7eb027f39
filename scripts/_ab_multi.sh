# headline A/B of the in-tree library against several _ab/<variant> builds:
#   bash scripts/_ab_multi.sh <tag> <variant>...
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/$tag/tests_$v.log 2>&1
done
B="python -u bench.py --steps 30 --warmup 10 --insitu 0 --ao 0 --frame 0 --ooc 0 --cpu-baseline 0"
for k in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/$tag/ship$k.log 2>&1
  for v in "$@"; do
    SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 200 $B > gpurun_out/$tag/${v}_$k.log 2>&1
  done
done
