#!/bin/bash
# round-4 first GPU pass: the new / changed GPU tests, smoke, then the default bench line
set -u
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_api2.py \
  "tests/test_gpu_baseline_shapes.py::test_headline_65536_rollout_T64_bitexact" \
  -m gpu -v -s -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|failing update" gpurun_out/t1.log | tail -30
stop_if_fatal $rc tests; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc smoke; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; exit $rc
