#!/bin/bash
# Build the differential-cost variants of libwk (region k executed twice) into
# ppo-bipedalwalker_amd/libwk_dup{k}.so:  bash scripts/dup_probe.sh build
# Time them on the GPU:                   bash scripts/dup_probe.sh run
set -eu
cd "$(dirname "$0")/../ppo-bipedalwalker_amd"
if [ "${1:-build}" = build ]; then
  for k in 1 2 3 4 5 6; do
    make -s -j2 BUILD=build_dup$k LIB=libwk_dup$k.so EXTRA=-DWK_DUP=$k &
  done
  wait
else
  cd ..
  for lib in libwk.so libwk_dup1.so libwk_dup2.so libwk_dup3.so libwk_dup4.so libwk_dup5.so libwk_dup6.so; do
    echo "== $lib"
    WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 120 python scripts/phys_bench.py 65536 64 2
  done
fi
