# Profiling evidence for profiles/: rocprofv3 kernel trace + stats of the
# default bench, then separate --pmc passes (one counter block set each) of a
# short bench run with the AO leg (the dominant AO any-hit kernel) included.
# PASSES: ';'-separated counter sets (default below).  Each pass has its own
# time limit; a failing pass stops the script.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
# provenance: the build id of the profiled library (bench.py matches it)
cp spray_amd/lib/libspray_rt.build.json "$OUT/build.json" || exit 1
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-3} "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
  return 0
}
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1; echo "list rc=$?"
fi
if [ "${TRACE:-1}" = 1 ]; then
  step bench 400 python bench.py --steps 20 --warmup 5 --cpu-seconds 5
  step trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0
fi
BENCHARGS=${BENCHARGS:-"--steps 2 --warmup 1 --cpu-baseline 0 --ooc 0 --frame 0 --insitu 0"}
DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS;GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ"
PASSES=${PASSES:-$DEFAULT}
i=0
IFS=';' read -ra ALL <<< "$PASSES"
for set in "${ALL[@]}"; do
  i=$((i+1))
  step pmc$i 150 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o run -- python3 bench.py $BENCHARGS
done
echo done
