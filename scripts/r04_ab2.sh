set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ppo-bipedalwalker_amd
for rep in 1 2; do
  for lib in libwk.so libwk_noopq.so; do
    echo "== $lib (rep $rep)" >> gpurun_out/ab2.log
    WK_LIB=$L/$lib REPS=8 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 WK_ORDER=1 >> gpurun_out/ab2.log 2>&1 || exit $?
  done
done
cat gpurun_out/ab2.log | grep -v amdgpu.ids
REGIME_ROUGH=1 timeout -k 10 400 python -u scripts/regime_ab.py 8192,65536 WK_ORDER=0 WK_ORDER=1 > gpurun_out/rough_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rough_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest "tests/test_gpu_multirank.py::test_ipc_peer_never_publishes" tests/test_gpu_baseline_shapes.py -m gpu -s -v -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/tol.log 2>&1; rc=$?; grep -E "PASSED|FAILED|failing update|max|diag" gpurun_out/tol.log | head -40; exit $rc
