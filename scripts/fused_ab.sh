# scripts/fused_shadow.py with the shipped library and each diag variant.
set -u
cd "$GRAFT_REPO_ROOT"
for L in shipped spray_amd/lib/diag/*.so; do
  if [ $L = shipped ]; then unset SPRAY_RT_LIB; else export SPRAY_RT_LIB=$PWD/$L; fi
  echo "== $L"
  timeout -k 10 200 python -u scripts/fused_shadow.py 2>&1 | grep -v amdgpu.ids || exit 1
done
