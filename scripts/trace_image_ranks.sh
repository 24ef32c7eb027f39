# Kernel trace of the image-parallel rehearsal at one N: every dispatch of
# each rehearsed rank's frames, summarised per kernel name and rank.
#   W=8 B=4 TAG=<name> bash scripts/trace_image_ranks.sh
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-imgtrace}; mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 scripts/image_rehearse.py --worlds ${W:-8} --bands ${B:-4} --frames 10 --warmup 3 > "$OUT/rehearse.txt" 2>&1
rc=$?; echo "trace rc=$rc"; cat "$OUT/rehearse.txt"
[ $rc -eq 0 ] || exit $rc
python3 scripts/summarize_image_trace.py "$OUT" ${W:-8} > "$OUT/summary.txt"; cat "$OUT/summary.txt"
