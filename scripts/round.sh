#!/bin/bash
# Round GPU driver (ROUND=r06 STEPS="tests smoke bench trace pmc"): every GPU step has its own time limit,
# and a hang / abort / fault (124, 134, 137, 139) or a failure stops the call.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${ROUND:-r06}
fatal() { case "$1" in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit "$1";; esac; [ "$1" -eq 0 ] || exit "$1"; }
for s in ${STEPS:-tests smoke bench}; do
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log; fatal $rc tests;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; fatal $rc smoke;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} --detail-file gpurun_out/bench_detail_$R.json > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.err; fatal $rc bench;;
    trace)
      OUT=gpurun_out/prof_$R; mkdir -p $OUT
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_trace.json 2> $OUT/bench_trace.err
      rc=$?; echo "trace rc=$rc"; fatal $rc trace
      python3 scripts/trace_by_grid.py $(find $OUT/trace -name "*kernel_trace.csv" | head -1) > $OUT/kernel_stats_by_grid.csv
      cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
      gzip -f $(find $OUT/trace -name "*kernel_trace.csv" | head -1);;
    pmc)
      OUT=gpurun_out/prof_$R; mkdir -p $OUT
      for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES"; do
        tag=$(echo $C | cut -d' ' -f1)
        timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_env_s(tep|ide)" -d $OUT/pmc_$tag -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/bench_pmc_$tag.json 2> $OUT/bench_pmc_$tag.err
        rc=$?; echo "pmc $tag rc=$rc"; fatal $rc pmc
      done;;
  esac
done
