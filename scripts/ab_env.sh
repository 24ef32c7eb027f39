# A/B of an environment switch on the same box: bench.py's fused step and
# the image-parallel rehearsal, alternating A and B runs.
#   VAR=SPRAY_STATIC_FIRST A=0 B=1 REPS=2 bash scripts/ab_env.sh > gpurun_out/ab.log
set -u
cd "$GRAFT_REPO_ROOT"
REPS=${REPS:-2}
BENCH=${BENCH:---steps 30 --warmup 10 --insitu 0 --ao 0 --frame 0 --image 0 --ooc 0 --cpu-baseline 0}
REH=${REH:---worlds 1 8 --bands 1 4 --frames 10}
for r in $(seq "$REPS"); do
  for v in "$A" "$B"; do
    echo "== $VAR=$v rep $r"
    env "$VAR=$v" timeout -k 10 200 python3 bench.py $BENCH | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fused ms', d['kernels_ms']['intersect_scene_shadow_pt'], 'step', d['ms_per_step'])" || exit 1
    [ -n "$REH" ] && { env "$VAR=$v" timeout -k 10 200 python3 scripts/image_rehearse.py $REH | grep -v amdgpu || exit 1; }
  done
done
