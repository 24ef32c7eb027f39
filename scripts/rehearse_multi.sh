# Rehearses bench.py's N > 1 path on a one-GPU box: N ranks share GPU 0 over
# "gloo", in-situ exchanges through the engine's host transport.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rehearse}
mkdir -p "$OUT"
N=${N:-4}
SPRAY_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --steps 3 --warmup 1 \
  --cpu-baseline 0 --frame 0 --ooc 0 > "$OUT/bench_n$N.log" 2>&1
rc=$?; echo "rehearse N=$N rc=$rc"; grep -v "amdgpu.ids\|socket.cpp" "$OUT/bench_n$N.log" | tail -c 2500
