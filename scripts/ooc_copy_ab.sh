# OOC: copy blocks per launch (prefetch of the next batch's images) A/B
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ooccopy}; mkdir -p "$OUT"
for rep in 1 2; do
for nb in 4 16 64; do
  SPRAY_OOC_COPY_BLOCKS=$nb timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_$nb.log" 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('$OUT/bench_$nb.log') if x.startswith('{')][-1]; d=json.loads(l)['ooc']; print('copy blocks $nb', d['ms_per_step'], d['loads_per_step'])"
done
done
