#!/bin/bash
# GPU-box: RoughFloor rollout / physics-only ms per 16 env-steps for each mapping (L = 1, 2, 4,
# 16) at the strong-scaling shard sizes
set -u
for n in ${SIZES:-8192 65536}; do
  WK_ROUGH=1 timeout -k 10 300 python scripts/phys_bench.py $n 16 ${LANES:-1 2 4 16} 2>&1 | grep -v amdgpu.ids || exit $?
done
