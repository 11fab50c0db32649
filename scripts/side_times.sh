#!/bin/bash
# GPU-box: pair-mapping (L=2) rollout / physics rates at several walker counts for each library in LIBS
set -u
for lib in ${LIBS:-libwk.so}; do
  echo "== $lib"
  for n in ${SIZES:-8192 32768 65536}; do
    WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 200 python scripts/phys_bench.py $n 16 ${LANES:-2} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
