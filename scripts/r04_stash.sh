# Legs parked in LDS across the policy section (WK_POLICY_STASH, default) vs the spill
# (libwk_nostash.so, -DWK_POLICY_STASH=0): parity tests on the default build, then rollout time
# in the bench regime (65,536 walkers, pair mapping) and WRITE_SIZE per rollout launch.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/stash; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_nonfinite.py "tests/test_gpu_baseline_shapes.py::test_headline_65536_rollout_T64_bitexact" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk.so libwk_nostash.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=5 timeout -k 10 300 python -u scripts/regime_ab.py 65536 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
for lib in libwk.so libwk_nostash.so; do
  WK_LIB=$L/$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/w_$lib -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/w_$lib.json 2> $OUT/w_$lib.err; rc=$?; echo "pmc $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
