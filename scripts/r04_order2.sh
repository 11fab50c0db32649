set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/regime_ab.py 65536,8192 WK_ORDER=1 WK_ORDER=2 > gpurun_out/order2_ab.log 2>&1; rc=$?; cat gpurun_out/order2_ab.log; [ $rc -eq 0 ] || exit $rc
for W in 1 8; do
  N=$((1024 * W))
  REPS=2 REGIME_UPDATES=0 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY --kernel-include-regex "k_env_side" -d gpurun_out/pmc_chain_$W -o run --output-format csv -- python3 scripts/regime_ab.py $N WK_QUAD_WPW=$W > gpurun_out/pmc_chain_$W.log 2>&1; rc=$?; echo "pmc $W rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
