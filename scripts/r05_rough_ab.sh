# Rough floor: the segment loop with closed-form segment boxes and the polygon built only on an
# overlap (libwk.so) vs round 4's loop (libwk_rough0.so); parity first (every rough-floor test,
# incl. the scene props on the rough floor), then the rollout in the bench regime on the rough floor
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/rough; mkdir -p $OUT; rm -f $OUT/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rough.py tests/test_gpu_scene.py tests/test_gpu_order.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_rough0.so libwk.so; do
  echo "== $lib" >> $OUT/ab.log
  REGIME_ROUGH=1 WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
