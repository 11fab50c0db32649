#!/bin/bash
# Round profiles (ROUND=r02): rocprofv3 kernel-trace stats of the default bench command, then
# separate PMC passes (no tracing) over the rollout kernel: HBM bytes (FETCH_SIZE, WRITE_SIZE)
# and one SQ pass (instruction mix, lane utilisation).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${ROUND:-r03}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_env_s(tep|ide)" -d $OUT/pmc_$tag -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/bench_pmc_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
find $OUT -name "*.csv" | head -20
