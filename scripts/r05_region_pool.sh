# Wave-level region breakdown of the pooled pair kernel (probe build libwk_prof.so), bench regime
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
REGIME_ITERS=8 timeout -k 10 300 python -u scripts/region_prof.py 65536 16 2 > gpurun_out/region_pool_65536.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/region_pool_65536.log; exit $rc
