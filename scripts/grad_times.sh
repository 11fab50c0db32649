#!/bin/bash
# GPU-box: grad_scaling.py timings for each library in LIBS
set -u
for lib in ${LIBS:-libwk.so}; do
  echo "== $lib"
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 120 python scripts/grad_scaling.py || exit $?
done
