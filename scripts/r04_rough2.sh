set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rough_trace
REGIME_ROUGH=1 timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/rough_trace -o run --output-format csv -- python3 scripts/regime_ab.py 8192 WK_ORDER=0 WK_ORDER=1 > gpurun_out/rough_trace/log.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rough_trace/log.txt | tail -3; exit $rc
