# OOC A/B over environment settings (ENVS: ';'-separated "VAR=v VAR2=w" sets;
# "-" = defaults): bench's ooc line only, two rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ooc_env}
mkdir -p "$OUT"
IFS=';' read -ra SETS <<< "${ENVS:--}"
for rep in 1 2; do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1))
    if [ "$e" = "-" ]; then e=""; fi
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ao 0 --frame 0 --insitu 0 --cpu-baseline 0 > "$OUT/bench_${i}_$rep.log" 2>&1 || { tail -5 "$OUT/bench_${i}_$rep.log"; exit 1; }
    python -c "
import json; l=[x for x in open('$OUT/bench_${i}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); o=d['ooc']; print('[$e]', o['ms_per_step'], o['loads_per_step'])"
  done
done
