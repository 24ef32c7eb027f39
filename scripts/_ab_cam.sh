# camera-frame rehearsal A/B (PT and AO, N = 2 / 8, view partition) of the
# in-tree library against _ab/<variant> builds: bash scripts/_ab_cam.sh <tag> <variant>...
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 tests/test_gpu_insitu.py -k "camera" > gpurun_out/$tag/tests_$v.log 2>&1
done
R="python -u scripts/camera_rehearse.py --worlds 2 8 --modes view --frames 10"
for k in 1 2; do
  timeout -k 10 300 $R --out gpurun_out/$tag/ship_pt$k.json > gpurun_out/$tag/ship_pt$k.log 2>&1
  for v in "$@"; do
    SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 300 $R --out gpurun_out/$tag/${v}_pt$k.json > gpurun_out/$tag/${v}_pt$k.log 2>&1
  done
done
timeout -k 10 300 $R --shader ao --out gpurun_out/$tag/ship_ao.json > gpurun_out/$tag/ship_ao.log 2>&1
for v in "$@"; do
  SPRAY_RT_LIB=$PWD/_ab/$v/libspray_rt.so timeout -k 10 300 $R --shader ao --out gpurun_out/$tag/${v}_ao.json > gpurun_out/$tag/${v}_ao.log 2>&1
done
