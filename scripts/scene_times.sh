#!/bin/bash
# GPU-box: scene-kernel (one lane per walker, scene_a props) physics/rollout rates for each library in LIBS
set -u
for lib in ${LIBS:-libwk.so}; do
  echo "== $lib"
  WK_SCENE=1 WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 300 python scripts/phys_bench.py ${SCENE_N:-65536} ${SCENE_T:-16} 1 || exit $?
done
