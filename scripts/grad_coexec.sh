#!/bin/bash
# GPU-box: do the producer's VALU and the consumer's MFMAs co-execute in
# k_ppo_grad_ws?  One SQ pass (<= 8 SQ counters) over a PPO update at M = 65,536 and one at the
# 8,192-sample shard minibatch (scripts/grad_one.py [walkers]).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/coexec
mkdir -p $OUT
for n in 65536 8192; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY --kernel-include-regex k_ppo_grad_ws -d $OUT/m$n -o run --output-format csv -- python3 scripts/grad_one.py $n > $OUT/m$n.log 2>&1
  rc=$?; echo "M=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_agg.py $OUT/m$n
done
