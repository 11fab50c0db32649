# PPO update with the fused minibatch tail: WK_GRAD_TAIL=0 (separate reduction + Adam launch, the
# default), 1 (release / acquire hand-off), 2 (sc1 hand-off); parity of the tail modes first
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tail; mkdir -p $OUT; rm -f $OUT/upd.log
for t in 1 2; do
  WK_GRAD_TAIL=$t timeout -k 10 600 python -u -m pytest tests/test_gpu_grad_scale.py "tests/test_gpu_parity.py::test_collective_path_matches_single_gpu_path" "tests/test_gpu_parity.py::test_ppo_update_matches_oracle" "tests/test_gpu_baseline_shapes.py::test_shard_8192_update_minibatch_global_vs_oracle" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$t.log 2>&1; rc=$?; echo "tail $t tests:"; tail -1 $OUT/tests_$t.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do for t in 0 1 2; do
  echo "== WK_GRAD_TAIL=$t" >> $OUT/upd.log
  WK_GRAD_TAIL=$t timeout -k 10 300 python -u scripts/update_ab.py 10 >> $OUT/upd.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/upd.log
