# SQ / TA / TD / TCP / TCC counters of the scene kernels, one --pmc pass per
# set (SETS: ';'-separated counter lists; default: the SQ issue/wait sets).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ctr}; mkdir -p "$OUT"
DEFAULT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum;GRBM_GUI_ACTIVE GRBM_COUNT"
SETS=${SETS:-$DEFAULT}
BENCH=${BENCH:-"--steps 2 --warmup 1 --cpu-baseline 0 --ao 0 --ooc 0"}
i=0
IFS=';' read -ra ALL <<< "$SETS"
for set in "${ALL[@]}"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $BENCH > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
