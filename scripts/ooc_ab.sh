# OOC bench line of the shipped library and the diag variants, twice each.
set -u
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for L in shipped spray_amd/lib/diag/*.so; do
    if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --ao 0 --frame 0 > gpurun_out/ooc_ab.log 2>&1 || exit 1
    python3 -c "
import json; l=[x for x in open('gpurun_out/ooc_ab.log') if x.startswith('{')][-1]; j=json.loads(l); print('$L', j['ms_per_step'], j['ooc']['ms_per_step'])"
  done
done
