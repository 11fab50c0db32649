#!/bin/bash
# kernel trace of one PPO update at a given shape: ARGS="8192 64 5"
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_ppo; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 scripts/ppo_only.py ${ARGS:-8192 64 5} > $OUT/log.txt 2>&1
rc=$?; echo "rc=$rc"; cat $OUT/log.txt | tail -3
find $OUT -name "*.csv" | head
