#!/bin/bash
# GPU box: rollout A/B of the shared floor slot (wk_physics.hip substep_side) -- libwk_base.so (the
# four-slot kernel) against libwk.so, twice in alternating order, in the bench regime
# (scripts/regime_ab.py) at the headline size and the 8-GPU shard.
set -u
P=ppo-bipedalwalker_amd
for rep in 1 2; do
  for lib in libwk_base.so libwk.so; do
    echo "== $lib"
    WK_LIB=$P/$lib REPS=4 timeout -k 10 200 python -u scripts/regime_ab.py 65536,8192 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
