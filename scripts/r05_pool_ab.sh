# Rollout A/B of the pooled-stage variants in the bench regime (65,536 walkers, pair mapping):
# libwk_nopool (per-lane stages), libwk_pool1 (leg-floor slots pooled), libwk_pool2 (leg-leg pairs
# pooled), libwk.so (both); then the wave-level breakdown of the pooled probe build
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/pool; mkdir -p $OUT; rm -f $OUT/ab2.log
for rep in 1 2; do for lib in libwk_nopool.so libwk_nopool_te.so libwk_pool1.so libwk_pool2.so libwk.so; do
  echo "== $lib" >> $OUT/ab2.log
  WK_LIB=$L/$lib REPS=5 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab2.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab2.log
bash scripts/r05_region_pool.sh
