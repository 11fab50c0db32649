# regime timing, then the full GPU suite, smoke, bench, kernel trace and PMC passes
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/regime_ab.py 65536,8192 WK_ORDER=1 > gpurun_out/regime.log 2>&1; rc=$?; cat gpurun_out/regime.log; [ $rc -eq 0 ] || exit $rc
STEPS="${STEPS:-tests smoke bench trace pmc}" bash scripts/r04_round.sh
