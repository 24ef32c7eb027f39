# AO tests with the shipped library, then scripts/ao_modes.py per library.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ao.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for L in shipped spray_amd/lib/diag/*.so; do
  if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 200 python -u scripts/ao_modes.py 2>&1 | grep "ordered\|output   lane" || exit 1
done
