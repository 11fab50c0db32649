# Probe: trajectory rows written at the lane slot instead of the walker id (libwk_slotrows.so,
# -DWK_PROBE_SLOTROWS=1: wrong columns, timing only) against the default build, both with the
# lane order on: what the rows' scatter under a lane order costs (rough floor: static order by
# start offset; flat floor: the episode-0 swaps).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/slotrows; mkdir -p $OUT; rm -f $OUT/ab.log
for rep in 1 2; do for lib in libwk.so libwk_slotrows.so; do
  echo "== $lib rough" >> $OUT/ab.log
  REGIME_ROUGH=1 WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
  echo "== $lib flat" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
