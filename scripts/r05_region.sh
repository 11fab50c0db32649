# Region breakdown (s_memtime stamps, -DWK_REGION_PROF probe build libwk_prof.so) of the final
# build's split kernels in the bench regime: 65,536 walkers (pair) and 8,192 (quad)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
REGIME_ITERS=8 timeout -k 10 300 python -u scripts/region_prof.py 65536 16 2 > gpurun_out/region_65536.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/region_65536.log; [ $rc -eq 0 ] || exit $rc
REGIME_ITERS=8 timeout -k 10 300 python -u scripts/region_prof.py 8192 16 4 > gpurun_out/region_8192.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/region_8192.log; exit $rc
