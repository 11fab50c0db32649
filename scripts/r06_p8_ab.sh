#!/bin/bash
# GPU box: the quad kernels in their own build part with the default scheduler (libwk.so) against the
# single side-kernel part built with max-ILP (libwk_base.so), bench regime, twice in alternating order.
set -u
P=ppo-bipedalwalker_amd
for rep in 1 2; do
  for lib in libwk_base.so libwk.so; do
    echo "== $lib"; WK_LIB=$P/$lib REPS=4 timeout -k 10 200 python -u scripts/regime_ab.py 65536,8192,4096 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
