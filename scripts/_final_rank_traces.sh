# kernel traces of the N = 8 (view) PT and AO camera-frame rehearsals of the
# shipped build, for scripts/rank_kernel_table.py
set -e
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5r_rk
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/pt -o run -- python3 $GRAFT_REPO_ROOT/scripts/camera_rehearse.py --worlds 8 --modes view --frames 5 --out $O/pt.json > $O/pt.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/ao -o run -- python3 $GRAFT_REPO_ROOT/scripts/camera_rehearse.py --worlds 8 --modes view --frames 5 --shader ao --out $O/ao.json > $O/ao.log 2>&1
