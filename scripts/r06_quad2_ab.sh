#!/bin/bash
# GPU box: the quad mapping at two waves per SIMD (probe build libwk_q2.so: the quad kernel compiled for
# two waves per SIMD, paced; WK_Q2=1 halves the walkers per wave so the shard launches twice the waves)
# against the product build, bench regime (scripts/regime_ab.py) at the 8-GPU shard and config 2/3's size.
set -u
P=ppo-bipedalwalker_amd
for rep in 1 2; do
  echo "== libwk.so"; WK_LIB=$P/libwk.so REPS=4 timeout -k 10 200 python -u scripts/regime_ab.py 8192,4096 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== libwk_q2.so"; WK_LIB=$P/libwk_q2.so REPS=4 timeout -k 10 200 python -u scripts/regime_ab.py 8192,4096 "" "WK_Q2=1" 2>&1 | grep -v amdgpu.ids || exit 1
done
