#!/bin/bash
# GPU box: gradient-kernel A/B of variant libraries against libwk_base.so (the round's product
# build): bit-equality of minibatch gradients and update weights (scripts/grad_bitwise.py), then
# PPO-update timings (scripts/update_ab.py), every library twice in alternating order.
#   LIBS="libwk_perm.so ..." bash scripts/r06_grad_ab.sh
set -u
mkdir -p gpurun_out
P=ppo-bipedalwalker_amd
LIBS=${LIBS:-libwk_perm.so}
WK_LIB=$P/libwk_base.so timeout -k 10 180 python scripts/grad_bitwise.py gpurun_out/g_base.npz || exit $?
for lib in $LIBS; do
  WK_LIB=$P/$lib timeout -k 10 180 python scripts/grad_bitwise.py gpurun_out/g_$lib.npz || exit $?
  echo "== bitwise $lib vs base"
  python scripts/grad_bitwise.py compare gpurun_out/g_base.npz gpurun_out/g_$lib.npz
done
for rep in 1 2; do
  for lib in libwk_base.so $LIBS; do
    WK_LIB=$P/$lib timeout -k 10 180 python scripts/update_ab.py ${REPS:-10} || exit $?
  done
done
