# Rough floor pair kernel: 16 of the legs' coordinates parked in a 4-record LDS column over the
# policy (WK_ROUGH_STASH, 56 -> 16 B scratch) vs the previous build (libwk_rs0.so): the rough-floor
# parity tests, then the rollout in the bench regime on the rough floor.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/rstash; mkdir -p $OUT; rm -f $OUT/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rough.py tests/test_gpu_scene.py tests/test_gpu_order.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_rs0.so libwk.so; do
  echo "== $lib" >> $OUT/ab.log
  REGIME_ROUGH=1 WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
