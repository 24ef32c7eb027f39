# headline A/B of the in-tree library against _ab/<variant>: bash scripts/_ab_lib.sh <tag> <variant>
set -e
export TMPDIR=/tmp
tag=$1; var=$2
mkdir -p gpurun_out/$tag
SPRAY_RT_LIB=$PWD/_ab/$var/libspray_rt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/$tag/tests.log 2>&1
B="python -u bench.py --steps 30 --warmup 10 --insitu 0 --ao 0 --frame 0 --ooc 0 --cpu-baseline 0"
for k in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/$tag/ship$k.log 2>&1
  SPRAY_RT_LIB=$PWD/_ab/$var/libspray_rt.so timeout -k 10 200 $B > gpurun_out/$tag/var$k.log 2>&1
done
