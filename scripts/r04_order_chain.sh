set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/order_test.log 2>&1; rc=$?; tail -3 gpurun_out/order_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/regime_ab.py 65536,8192,4096 WK_ORDER=0 WK_ORDER=1 > gpurun_out/order_ab.log 2>&1; rc=$?; cat gpurun_out/order_ab.log; [ $rc -eq 0 ] || exit $rc
REGIME_UPDATES=0 timeout -k 10 300 python -u scripts/regime_ab.py 1024 WK_QUAD_WPW=1 > gpurun_out/chain.log 2>&1 || exit $?
REGIME_UPDATES=0 timeout -k 10 300 python -u scripts/regime_ab.py 2048 WK_QUAD_WPW=2 >> gpurun_out/chain.log 2>&1 || exit $?
REGIME_UPDATES=0 timeout -k 10 300 python -u scripts/regime_ab.py 4096 WK_QUAD_WPW=4 >> gpurun_out/chain.log 2>&1 || exit $?
REGIME_UPDATES=0 timeout -k 10 300 python -u scripts/regime_ab.py 8192 WK_QUAD_WPW=8 >> gpurun_out/chain.log 2>&1 || exit $?
cat gpurun_out/chain.log
