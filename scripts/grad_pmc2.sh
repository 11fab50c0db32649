#!/bin/bash
# GPU-box: two SQ counter passes over k_ppo_grad_mfma (M = 65,536) for each library in LIBS:
# issue / MFMA-busy / waits, then LDS instructions, bank conflicts and LDS waits.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gpmc2
for lib in ${LIBS:-libwk.so}; do
  i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i + 1))
    WK_LIB=ppo-bipedalwalker_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_ppo_grad_mfma -d gpurun_out/gpmc2/$lib.$i -o run --output-format csv -- python3 scripts/grad_one.py > gpurun_out/gpmc2/$lib.$i.log 2>&1
    rc=$?; echo "$lib pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 scripts/pmc_agg.py gpurun_out/gpmc2/$lib.$i
  done
done
