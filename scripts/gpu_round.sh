#!/bin/bash
# GPU-box driver: each GPU step has its own time limit; stop on timeout/abort/segfault.
set -u
mkdir -p gpurun_out
stop_if_fatal() {  # exit codes that mean the GPU step hung, aborted or faulted
  case "$1" in 124|134|137|139) echo "FATAL rc=$1 in $2 -- stopping"; exit "$1";; esac
}
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/gpu_tests.log; stop_if_fatal $rc tests;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_fatal $rc smoke;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; stop_if_fatal $rc bench;;
  esac
done
