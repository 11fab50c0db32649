#!/bin/bash
# Counter passes over kernels matching $KREGEX while running $CMD (python3 script args).
#   KREGEX="k_ppo_grad_mfma" CMD="scripts/ppo_only.py 65536 64 1" PMC_SETS="A B;C D" bash scripts/pmc_generic.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
IFS=';' read -ra SETS <<< "$PMC_SETS"
i=0
for CTRS in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "$KREGEX" -d $OUT/p$i -o run --output-format csv -- python3 $CMD > $OUT/log$i.txt 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
