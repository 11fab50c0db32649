# Rough floor: the segment loop restricted to the part's x-range (+1 segment each side, the full
# rest once the part moved) against visiting all ten (libwk_krange0.so): every rough-floor GPU
# test (all mappings, bench-size replays, scene props on the rough floor, lane order), then the
# rough rollouts in the bench regime.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/krange; mkdir -p $OUT; rm -f $OUT/ab.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_rough.py tests/test_gpu_scene.py tests/test_gpu_order.py tests/test_gpu_api2.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_krange0.so libwk.so; do
  echo "== $lib" >> $OUT/ab.log
  REGIME_ROUGH=1 WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
