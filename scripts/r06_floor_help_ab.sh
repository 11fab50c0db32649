#!/bin/bash
# GPU box: the pair mapping's leg-floor pair with wave-level helper lanes
# (WK_FLOOR_HELP=1, libwk.so) against the per-lane pair (libwk_fh0.so): bench.py's headline
# (65,536 walkers, bench regime) alternated A B A B, after the bit-exact suites pass on libwk.so.
set -u
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_nonfinite.py tests/test_gpu_baseline_shapes.py tests/test_gpu_call_shape.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_fh_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_fh_tests.log; exit 1; }
tail -1 gpurun_out/r06_fh_tests.log
for rep in 1 2; do
  for v in fh0 help; do
    if [ $v = fh0 ]; then export WK_LIB=$PWD/ppo-bipedalwalker_amd/libwk_fh0.so; else export WK_LIB=$PWD/ppo-bipedalwalker_amd/libwk.so; fi
    timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --detail-file gpurun_out/r06_fh_${v}_$rep.json > gpurun_out/r06_fh_${v}_$rep.line 2> gpurun_out/r06_fh_${v}_$rep.err || { echo "bench $v failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06_fh_${v}_$rep.json'));print('$v', $rep, round(d['value']/1e6,2), 'M/s rollout_ms', round(d['roofline']['mean_launch_ms'],3), 'update_ms', round(d['ppo_update_ms'],3))"
  done
done
