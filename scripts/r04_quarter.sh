set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/regime_ab.py 8192,4096 WK_QUARTER=0 WK_QUARTER=1 WK_QUARTER=0 WK_QUARTER=1 > gpurun_out/quarter_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/quarter_ab.log; [ $rc -eq 0 ] || exit $rc
REGIME_ROUGH=1 timeout -k 10 400 python -u scripts/regime_ab.py 8192 WK_QUARTER=0 WK_QUARTER=1 > gpurun_out/quarter_rough.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/quarter_rough.log; exit $rc
