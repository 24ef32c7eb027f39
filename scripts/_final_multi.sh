set -e
export TMPDIR=/tmp
TAG=r5r_multi N=2 bash scripts/rehearse_multi.sh
TAG=r5r_multi N=8 bash scripts/rehearse_multi.sh
mkdir -p gpurun_out/r5r_multi
timeout -k 10 400 python bench.py --steps 20 --warmup 10 --cpu-seconds 10 > gpurun_out/r5r_multi/bench_repeat.log 2>&1
