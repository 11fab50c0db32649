#!/bin/bash
# GPU-box: instruction-cache and SQ counters of the scene kernel (scene_a, 65,536 walkers) for LIBS
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/spmc
for lib in ${LIBS:-libwk.so}; do
  WK_SCENE=1 WK_LIB=ppo-bipedalwalker_amd/$lib timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex k_env_scene -d gpurun_out/spmc/$lib -o run --output-format csv -- python3 scripts/phys_bench.py 65536 4 1 > gpurun_out/spmc/$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_agg.py gpurun_out/spmc/$lib
done
