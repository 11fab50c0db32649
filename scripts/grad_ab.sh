#!/bin/bash
# GPU-box: gradient-kernel A/B of libwk.so against LIBS (default libwk_base.so): bit-equality of
# gradients / update weights (scripts/grad_bitwise.py) and per-size timings (grad_scaling.py).
set -u
mkdir -p gpurun_out
timeout -k 10 180 python scripts/grad_bitwise.py gpurun_out/g_new.npz || exit $?
for lib in ${LIBS:-libwk_base.so}; do
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 180 python scripts/grad_bitwise.py gpurun_out/g_$lib.npz || exit $?
  python scripts/grad_bitwise.py compare gpurun_out/g_$lib.npz gpurun_out/g_new.npz
done
for lib in libwk.so ${LIBS:-libwk_base.so}; do
  echo "== $lib"
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 120 python scripts/grad_scaling.py || exit $?
done
