# Plain trajectory stores with the done byte per env-step (libwk_plainnd.so) against plain stores
# with the deferred done bytes (libwk_plain.so) and the round-5 default (non-temporal rows,
# libwk_nodefer.so): WRITE_SIZE per launch (rollouts only, both lane orders), rollout time, then
# the bench's own launches under the plain + per-step build.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/plain; mkdir -p $OUT; rm -f $OUT/ab.log $OUT/series.txt
for lib in libwk_nodefer.so libwk_plain.so libwk_plainnd.so; do for O in 1 0; do
  tag=${lib%.so}_o$O
  WK_ORDER=$O WK_LIB=$L/$lib REGIME_UPDATES=0 REPS=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/$tag -o run --output-format csv -- python3 scripts/regime_ab.py 65536 > $OUT/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "$tag $(python3 scripts/pmc_series.py $(find $OUT/$tag -name '*counter_collection.csv' | head -1) WRITE_SIZE)" >> $OUT/series.txt
done; done
cat $OUT/series.txt
for rep in 1 2; do for lib in libwk_nodefer.so libwk_plainnd.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
for lib in libwk_plainnd.so libwk_plain.so; do for C in FETCH_SIZE WRITE_SIZE; do
  WK_LIB=$L/$lib timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_side" -d $OUT/bench_${lib}_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/bench_${lib}_$C.json 2> $OUT/bench_${lib}_$C.err; rc=$?; echo "pmc bench $lib $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/traffic_from_pmc.py $(find $OUT/bench_${lib}_FETCH_SIZE -name "*counter_collection.csv" | head -1) $(find $OUT/bench_${lib}_WRITE_SIZE -name "*counter_collection.csv" | head -1) 65536 64 $OUT/traffic_$lib.json
done
