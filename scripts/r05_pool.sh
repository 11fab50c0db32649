# Pooled contact stages (WK_POOL, default) vs the per-lane stages (libwk_nopool.so, -DWK_POOL=0):
# the bit-exact parity tests of the pair mapping on the default build, then rollout time in the
# bench regime (65,536 walkers, pair mapping; 8,192 quad as a control: unchanged code)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/pool; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_nonfinite.py "tests/test_gpu_baseline_shapes.py::test_headline_65536_rollout_T64_bitexact" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk.so libwk_nopool.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=5 timeout -k 10 300 python -u scripts/regime_ab.py 65536 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
