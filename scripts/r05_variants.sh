# Rollout build variants on the scratch-free kernel (bench regime, 65,536 and the 8,192 shard):
# default (max-ILP scheduling, torso early, LDS faces, legs stashed over the policy) against the
# default scheduler (libwk_sdef.so), WK_TORSO_EARLY=0, WK_FACE_LDS=0, WK_POLICY_STASH=0.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/variants; mkdir -p $OUT; rm -f $OUT/ab.log
for rep in 1 2; do for lib in libwk.so libwk_sdef.so libwk_torso0.so libwk_face0.so libwk_stash0.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
