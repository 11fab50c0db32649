#!/bin/bash
# GPU box: the rough-floor side kernels (build part 5) with the default scheduler (libwk_r5.so) against
# max-ILP (libwk.so), bench regime on the rough floor.
set -u
P=ppo-bipedalwalker_amd
for rep in 1 2; do
  for lib in libwk.so libwk_r5.so; do
    echo "== $lib"; WK_LIB=$P/$lib REGIME_ROUGH=1 REPS=3 timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
