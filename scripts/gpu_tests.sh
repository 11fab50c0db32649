#!/bin/bash
# GPU-box: run selected GPU test files (TESTS="tests/a.py tests/b.py"), one pytest process,
# each test time-limited; stop on a fatal exit status.
set -u
mkdir -p gpurun_out
LOG=gpurun_out/${LOGNAME_:-gpu_sel}.log
timeout -k 10 ${TLIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v -s -x --timeout 300 --timeout-method thread -p no:cacheprovider > $LOG 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $LOG | tail -40
exit $rc
