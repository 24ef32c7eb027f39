# wave-time / packet-log diagnostics of the libraries in spray_amd/lib/wt
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wt}; mkdir -p "$OUT"
for L in spray_amd/lib/wt/*.so; do
  echo "== wave times $L"
  SPRAY_RT_LIB=$PWD/$L timeout -k 10 200 python -u scripts/wave_times.py > "$OUT/wt.log" 2>&1
  rc=$?; grep -v amdgpu.ids "$OUT/wt.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
