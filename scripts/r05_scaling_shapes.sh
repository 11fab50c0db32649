# Per-GPU shard times for the 1 -> 8 GPU strong-scaling projection (Multi-GPU):
# rollout in the bench regime at 32,768 / 16,384 walkers and the update at those shards'
# minibatches (M = walkers, M_global = 65,536), final round-5 build
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
REPS=5 timeout -k 10 300 python -u scripts/regime_ab.py 32768,16384 > gpurun_out/scaling_rollout.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/scaling_rollout.log; [ $rc -eq 0 ] || exit $rc
UPDATE_SHAPES="32768:32768:65536,16384:16384:65536" timeout -k 10 300 python -u scripts/update_ab.py 10 > gpurun_out/scaling_update.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/scaling_update.log; exit $rc
