#!/bin/bash
# Counter passes (one rocprofv3 run per counter set) over one launch of the env-step kernel.
#   ARGS="65536 8 2 rollout" PMC_SETS="A B C;D E" bash scripts/pmc_physics.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
DEF="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES;SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEF}"
i=0
for CTRS in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "k_env_s(tep|ide)" -d $OUT/p$i -o run --output-format csv -- python3 scripts/phys_only.py ${ARGS:-65536 8 2} > $OUT/log$i.txt 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
