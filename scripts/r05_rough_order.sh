# Rough floor lane order by start offset (static, wk_api.cpp rough_order_upload) against the
# identity order: the order / rough / scene / io GPU tests, then the rough rollouts in the bench
# regime (WK_ORDER=1 vs 0 in the same build: 65,536 pair and 8,192 quad walkers).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rorder; mkdir -p $OUT; rm -f $OUT/ab.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_rough.py tests/test_gpu_scene.py tests/test_gpu_io.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  REGIME_ROUGH=1 REPS=3 timeout -k 10 400 python -u scripts/regime_ab.py 65536,8192 "WK_ORDER=0" "WK_ORDER=1" >> $OUT/ab.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/ab.log
