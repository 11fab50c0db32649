#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "k_env_step" -d $OUT/p$i -o run --output-format csv -- python3 scripts/phys_only.py ${ARGS:-8192 8} > $OUT/log$i.txt 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
