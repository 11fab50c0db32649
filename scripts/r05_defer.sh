# Done bytes deferred (WK_DONE_DEFER, default now: a lane's terminal flags of 32 env-steps in one
# register, written row by row at once) against the per-env-step byte (libwk_nodefer.so), and
# plain instead of non-temporal trajectory stores (libwk_plain.so): the whole GPU suite on the
# default build, rollout time in the bench regime, WRITE_SIZE per launch (rollouts only), then
# FETCH / WRITE of the bench's own launches for the default build (profiles/traffic_physics.json).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/defer; mkdir -p $OUT; rm -f $OUT/ab.log $OUT/series.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libwk_nodefer.so libwk.so libwk_plain.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
for lib in libwk_nodefer.so libwk.so libwk_plain.so; do for O in 1 0; do
  tag=${lib%.so}_o$O
  WK_ORDER=$O WK_LIB=$L/$lib REGIME_UPDATES=0 REPS=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/$tag -o run --output-format csv -- python3 scripts/regime_ab.py 65536 > $OUT/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "$tag $(python3 scripts/pmc_series.py $(find $OUT/$tag -name '*counter_collection.csv' | head -1) WRITE_SIZE)" >> $OUT/series.txt
done; done
cat $OUT/series.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_side" -d $OUT/bench_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/bench_$C.json 2> $OUT/bench_$C.err; rc=$?; echo "pmc bench $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/traffic_from_pmc.py $(find $OUT/bench_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $OUT/bench_WRITE_SIZE -name "*counter_collection.csv" | head -1) 65536 64 $OUT/traffic_physics.json
