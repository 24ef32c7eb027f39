# A/B of library variants x one environment switch on the same box:
#   LIBS="spray_amd/lib/libspray_rt.so _ab/q8/libspray_rt.so" VAR=X VALS="0 1" bash scripts/ab_libs.sh
# per combination: scripts/launch_probe.py (fused launch over miss / mid / full
# ray sets), the bench's fused step, the image-parallel rehearsal (REH)
set -u
cd "$GRAFT_REPO_ROOT"
REH=${REH:---worlds 2 8 --bands 1 4 --frames 10}
for lib in $LIBS; do
  for v in $VALS; do
    echo "== $lib $VAR=$v"
    env SPRAY_RT_LIB=$lib "$VAR=$v" timeout -k 10 200 python3 scripts/launch_probe.py | grep -v amdgpu || exit 1
    env SPRAY_RT_LIB=$lib "$VAR=$v" timeout -k 10 200 python3 bench.py --steps 30 --warmup 10 --insitu 0 --ao 0 --frame 0 --image 0 --ooc 0 --cpu-baseline 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fused ms', d['kernels_ms']['intersect_scene_shadow_pt'])" || exit 1
    [ -n "$REH" ] && { env SPRAY_RT_LIB=$lib "$VAR=$v" timeout -k 10 200 python3 scripts/image_rehearse.py $REH | grep -v amdgpu || exit 1; }
  done
done
