# OOC leg A/B: the bench's "ooc" line (and headline) for the shipped library
# and the variants in LIBS, alternated, three rounds.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-oocab}; mkdir -p "$OUT"
for rep in 1 2 3; do
  for L in shipped $LIBS; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --frame 0 --insitu 0 --ao 0 > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
    python -c "
import json; l=[x for x in open('$OUT/b.log') if x.startswith('{')][-1]; d=json.loads(l); o=d['ooc']; print('%-22s step %.4f ooc %.4f loads %s' % ('$(basename $L .so)', d['ms_per_step'], o['ms_per_step'], o['loads_per_step']))"
  done
done
