# Round-5 A/B on one box: (1) the parity tests the changes touch (torso step moved next to the
# lower leg's integrate; fused minibatch tail; pooled stages build kept as an option), then
# (2) the rollout in the bench regime: libwk_nopool.so (round-4 kernel) vs libwk.so (torso
# early) vs libwk_pool3.so (torso early + pooled stages), 65,536 and 8,192 walkers, and (3) the
# PPO update with the fused tail (WK_GRAD_TAIL=1, default) vs the separate reduction launch
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/ab3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grad_scale.py tests/test_gpu_baseline_shapes.py tests/test_gpu_multirank.py tests/test_gpu_api2.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_nopool.so libwk.so libwk_pool3.so libwk_pool1.so libwk_pool2.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=5 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
for rep in 1 2; do for t in 0 1; do
  echo "== WK_GRAD_TAIL=$t" >> $OUT/upd.log
  WK_GRAD_TAIL=$t timeout -k 10 300 python -u scripts/update_ab.py 10 >> $OUT/upd.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/upd.log
bash scripts/r05_region_pool.sh
