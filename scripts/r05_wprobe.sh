# Where the rollout's written bytes above the algorithmic ones go: WRITE_SIZE per rollout launch
# (rollouts only, weights at init: REGIME_UPDATES=0, so nothing reads the trajectory and a probe
# build that skips a store changes nothing else) for the default build, the identity lane order,
# and probe builds without the s rows (1), the done bytes (2), the a / lp / v / r rows (4).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/wprobe; mkdir -p $OUT; rm -f $OUT/series.txt
run() {  # tag lib env...
  tag=$1; lib=$2; shift 2
  env "$@" WK_LIB=$L/$lib REGIME_UPDATES=0 REPS=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/$tag -o run --output-format csv -- python3 scripts/regime_ab.py 65536 > $OUT/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "$tag $(python3 scripts/pmc_series.py $(find $OUT/$tag -name '*counter_collection.csv' | head -1) WRITE_SIZE)" >> $OUT/series.txt
}
run default libwk.so WK_ORDER=1
run order0 libwk.so WK_ORDER=0
run skip_s libwk_probe1.so WK_ORDER=1
run skip_d libwk_probe2.so WK_ORDER=1
run skip_alpvr libwk_probe4.so WK_ORDER=1
cat $OUT/series.txt
