# PMC passes of the headline launch for the in-tree library and an A/B build:
#   bash scripts/_pmc_ab.sh <tag> <variant>   (variant: _ab/<variant>/libspray_rt.so)
set -u
export TMPDIR=/tmp
tag=$1; var=$2
OUT=gpurun_out/$tag
mkdir -p $OUT
B="bench.py --steps 3 --warmup 2 --cpu-baseline 0 --ooc 0 --frame 0 --insitu 0 --ao 0"
SETS=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ")
for v in ship $var; do
  if [ $v = ship ]; then L=""; else L=$PWD/_ab/$v/libspray_rt.so; fi
  SPRAY_RT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v/trace -o run -- python3 $B > $OUT/$v.trace.log 2>&1 || exit 1
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    SPRAY_RT_LIB=$L timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$v/pmc$i -o run -- python3 $B > $OUT/$v.pmc$i.log 2>&1 || exit 1
  done
done
echo done
