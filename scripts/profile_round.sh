#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then separate PMC passes
# (one counter each, no tracing) for the rollout kernel's HBM bytes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_env_s(tep|ide)" -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
find $OUT -name "*.csv" | head -20
