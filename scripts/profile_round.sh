#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench, then separate PMC passes for HBM bytes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_env_step" -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_step" -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
find $OUT -name "*.csv" | head -20
