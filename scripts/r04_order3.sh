set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/order_test.log 2>&1; rc=$?; tail -2 gpurun_out/order_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/regime_ab.py 65536,8192 WK_ORDER=0 WK_ORDER=1 > gpurun_out/order3_ab.log 2>&1; rc=$?; cat gpurun_out/order3_ab.log; [ $rc -eq 0 ] || exit $rc
REGIME_ROUGH=1 timeout -k 10 400 python -u scripts/regime_ab.py 8192 WK_ORDER=0 WK_ORDER=1 > gpurun_out/order3_rough.log 2>&1; rc=$?; cat gpurun_out/order3_rough.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_r04b; mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/pmc_WRITE_SIZE -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/w.json 2> $OUT/w.err; echo "pmc rc=$?"
