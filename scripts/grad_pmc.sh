#!/bin/bash
# GPU-box: SQ counters of k_ppo_grad_mfma (M = 65,536) for libwk.so and LIBS (A/B), one pass each.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gpmc
for lib in libwk.so ${LIBS:-libwk_base.so}; do
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_ppo_grad_mfma -d gpurun_out/gpmc/$lib -o run --output-format csv -- python3 scripts/grad_one.py > gpurun_out/gpmc/$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_agg.py gpurun_out/gpmc/$lib
done
