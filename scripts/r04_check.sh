# full GPU suite then regime timing (the current build)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/regime_ab.py ${AB_SIZES:-65536,8192} ${AB_VARIANTS:-WK_ORDER=1} > gpurun_out/regime.log 2>&1; rc=$?; cat gpurun_out/regime.log; exit $rc
