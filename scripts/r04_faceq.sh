set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ppo-bipedalwalker_amd
WK_LIB=$L/libwk_flq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_nonfinite.py tests/test_gpu_rough.py "tests/test_gpu_baseline_shapes.py::test_shard_8192_rollout_T64_bitexact" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/flq_tests.log 2>&1; rc=$?; tail -2 gpurun_out/flq_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk.so libwk_flq.so; do
  echo "== $lib" >> gpurun_out/flq_ab.log
  WK_LIB=$L/$lib REPS=6 timeout -k 10 300 python -u scripts/regime_ab.py 8192,4096 WK_ORDER=1 >> gpurun_out/flq_ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids gpurun_out/flq_ab.log
