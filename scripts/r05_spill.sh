# The rollout kernel without scratch (WK_OPQ_LOOP: loop-invariant addresses / Philox words / the
# template offset formed inside the env-step loop from opaque copies) vs the previous build
# (libwk_spill.so: 28 VGPRs, 112 B of scratch per lane): parity first, then rollout time in the
# bench regime (65,536 and the 8,192 shard) and FETCH_SIZE / WRITE_SIZE per rollout launch.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/spill; mkdir -p $OUT; rm -f $OUT/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_nonfinite.py tests/test_gpu_rough.py "tests/test_gpu_baseline_shapes.py::test_headline_65536_rollout_T64_bitexact" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_spill.so libwk.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
for lib in libwk.so libwk_spill.so; do for C in FETCH_SIZE WRITE_SIZE; do
  WK_LIB=$L/$lib timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_side" -d $OUT/p_${lib}_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/b_${lib}_$C.json 2> $OUT/b_${lib}_$C.err; rc=$?; echo "pmc $lib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/traffic_from_pmc.py $(find $OUT/p_${lib}_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $OUT/p_${lib}_WRITE_SIZE -name "*counter_collection.csv" | head -1) 65536 64 $OUT/traffic_$lib.json
done
