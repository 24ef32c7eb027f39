# AO camera-frame A/B: GPU tests of the in-tree library, the N = 2 / 8 AO
# rehearsal of it and of _ab/old, and a kernel trace of the new N = 8 rehearsal
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/aoab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_insitu.py tests/test_gpu_fullsize.py -k "ao or camera or replicated" > gpurun_out/aoab/tests.log 2>&1
R="python -u scripts/camera_rehearse.py --worlds 2 8 --modes view --frames 10 --shader ao"
for k in 1 2; do
  timeout -k 10 300 $R --out gpurun_out/aoab/new$k.json > gpurun_out/aoab/new$k.log 2>&1
  SPRAY_RT_LIB=$PWD/_ab/old/libspray_rt.so timeout -k 10 300 $R --out gpurun_out/aoab/old$k.json > gpurun_out/aoab/old$k.log 2>&1
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/aoab/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/camera_rehearse.py --worlds 8 --modes view --frames 5 --shader ao --out $GRAFT_REPO_ROOT/gpurun_out/aoab/k.json > $GRAFT_REPO_ROOT/gpurun_out/aoab/k.log 2>&1
