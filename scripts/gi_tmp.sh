cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_bench_rehearsal.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/xch_tests.log 2>&1; rc=$?; tail -3 gpurun_out/xch_tests.log; exit $rc
