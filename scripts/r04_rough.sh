set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
REGIME_ROUGH=1 timeout -k 10 500 python -u scripts/regime_ab.py 8192 WK_ORDER=1 WK_ORDER=0 WK_ORDER=1 WK_ORDER=0 > gpurun_out/rough_ab2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rough_ab2.log; [ $rc -eq 0 ] || exit $rc
REGIME_ROUGH=1 REGIME_UPDATES=0 timeout -k 10 500 python -u scripts/regime_ab.py 8192 WK_ORDER=1 WK_ORDER=0 > gpurun_out/rough_ab3.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rough_ab3.log; exit $rc
