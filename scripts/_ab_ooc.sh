# OOC A/B: bash scripts/_ab_ooc.sh <tag> <variant>...
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 tests/test_gpu_ooc.py > gpurun_out/$tag/tests.log 2>&1
for k in 1 2; do
  timeout -k 10 200 python -u scripts/ooc_only.py 20 > gpurun_out/$tag/new$k.log 2>&1
  for v in "$@"; do
    SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 200 python -u scripts/ooc_only.py 20 > gpurun_out/$tag/${v}_$k.log 2>&1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run -- python scripts/ooc_only.py 5 > gpurun_out/$tag/prof.log 2>&1
