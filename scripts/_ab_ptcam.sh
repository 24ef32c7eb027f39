# PT camera-frame A/B: GPU camera tests of the in-tree library, the N = 2 / 8
# PT rehearsal of it and of _ab/old, alternated
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ptab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_insitu.py tests/test_gpu_fullsize.py -k "camera or replicated" > gpurun_out/ptab/tests.log 2>&1
R="python -u scripts/camera_rehearse.py --worlds 2 8 --modes view --frames 10"
for k in 1 2; do
  timeout -k 10 300 $R --out gpurun_out/ptab/new$k.json > gpurun_out/ptab/new$k.log 2>&1
  SPRAY_RT_LIB=$PWD/_ab/old/libspray_rt.so timeout -k 10 300 $R --out gpurun_out/ptab/old$k.json > gpurun_out/ptab/old$k.log 2>&1
done
