set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=ppo-bipedalwalker_amd
for rep in 1 2; do for lib in libwk.so libwk_nosc1.so; do
  WK_LIB=$L/$lib timeout -k 10 300 python -u scripts/update_ab.py 10 >> gpurun_out/upd_ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids gpurun_out/upd_ab.log
mkdir -p gpurun_out/upd_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/upd_trace -o run --output-format csv -- python3 scripts/update_ab.py 3 > gpurun_out/upd_trace/log.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grad_scale.py tests/test_gpu_multirank.py tests/test_gpu_api2.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/upd_tests.log 2>&1; rc=$?; tail -2 gpurun_out/upd_tests.log; exit $rc
