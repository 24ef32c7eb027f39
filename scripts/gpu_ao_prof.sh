# AO step: kernel trace + one PMC pass (spawn and any-hit kernels).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aoprof}
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --frame 0 --insitu 0 --ooc 0 --cpu-baseline 0 > "$OUT/bench.log" 2>&1 || exit $?
python3 -c "
import csv,glob
for f in glob.glob('$OUT/trace/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('%10.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))
"
PMC="${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}" TAG=${TAG:-aoprof}_pmc timeout -k 10 200 bash scripts/gpu_pmc.sh > /dev/null 2>&1 || true
