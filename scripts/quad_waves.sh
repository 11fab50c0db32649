#!/bin/bash
# GPU-box: the quad mapping built for one wave per SIMD (libwk.so) against a build for two
# (libwk_q2.so, -DWK_QUAD_WAVES=2), with the pair mapping as reference, at the strong-scaling
# shard sizes (65,536 / N walkers): rollout and physics-only ms per 16 env-steps.
set -u
for n in ${SIZES:-8192 16384 32768 65536}; do
  for cfg in "libwk.so 4" "libwk_q2.so 4" "libwk.so 2"; do
    set -- $cfg
    echo "== $1 L=$2 n=$n"
    WK_LIB=ppo-bipedalwalker_amd/$1 timeout -k 10 120 python scripts/phys_bench.py $n 16 $2 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
