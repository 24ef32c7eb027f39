# Frame tests, then the bench "frame" line of the shipped library and the diag variants.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for rep in 1 2; do
  for L in shipped spray_amd/lib/diag/*.so; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --ao 0 --ooc 0 > gpurun_out/frame_ab.log 2>&1 || exit 1
    python3 -c "
import json; l=[x for x in open('gpurun_out/frame_ab.log') if x.startswith('{')][-1]; j=json.loads(l); f=j['frame']; print('$L', j['ms_per_step'], f['ms_per_step'], f['rays_per_step'], f['image_mean'])"
  done
done
