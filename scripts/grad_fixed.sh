#!/bin/bash
# grad-kernel fixed cost: kernel-trace durations of the main build, and the chunk-loop /
# epilogue probe builds (make BUILD=build_noloop LIB=libwk_noloop.so EXTRA=-DWK_GRAD_NOLOOP, ...)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in libwk.so libwk_noloop.so libwk_noepi.so; do
  echo "== $lib"
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 120 python scripts/grad_scaling.py || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gradprof -o run --output-format csv -- python3 scripts/grad_scaling.py > gpurun_out/gradprof.log 2>&1 || exit $?
find gpurun_out/gradprof -name "*kernel_stats.csv" -exec cat {} \;
