#!/bin/bash
# GPU box: the exchange kernel A/B (xa: system-scope acquire polls + every thread's acquire fence +
# plain Adam stores; xb: relaxed polls, one acquire by the polling wave, written-through Adam /
# grad_out stores), each measured uncontended (scripts/r06_xch_own.py) after the IPC tests pass
# on it.
set -u
cd "$(dirname "$0")/.."
for v in xa xb; do
  export WK_LIB=$PWD/ppo-bipedalwalker_amd/libwk_$v.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_xch_ab_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/r06_xch_ab_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06_xch_ab_tests_$v.log
  timeout -k 10 300 python3 scripts/r06_xch_own.py 2 5 > gpurun_out/r06_xch_own_$v.log 2>&1 || { echo "own $v failed"; exit 1; }
  mkdir -p gpurun_out/r06_xch_own_$v && cp -r gpurun_out/r06_xch_own/n2_r0 gpurun_out/r06_xch_own_$v/
done
