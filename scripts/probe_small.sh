#!/bin/bash
# rollout / PPO-update timings at the small per-GPU shapes (BASELINE configs 2-4: 4,096 and
# 8,192 walkers) for every physics mapping
set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/phys_bench.py 8192 64 1 2 16 > gpurun_out/probe_8192.log 2>&1 || exit $?
timeout -k 10 300 python scripts/phys_bench.py 4096 64 1 2 16 > gpurun_out/probe_4096.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_only.py 8192 64 5 > gpurun_out/probe_ppo8192.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_only.py 4096 64 5 > gpurun_out/probe_ppo4096.log 2>&1 || exit $?
cat gpurun_out/probe_*.log
