#!/bin/bash
# GPU-box: one SQ pass over the small-shard rollout kernel (quad mapping, L = 4) at WALKERS
# (default 8,192), T = 16: VALU instructions per wave-substep, active lanes per VALU
# instruction, issue vs wait cycles.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${WALKERS:-8192}; L=${LANES:-4}
OUT=gpurun_out/qpmc_${N}_$L
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex "k_env_side" -d $OUT -o run --output-format csv -- python3 scripts/phys_bench.py $N 16 $L > $OUT/log 2>&1
rc=$?; echo "quad pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_agg.py $OUT
