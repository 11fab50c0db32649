set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/phys_bench.py 32768 64 2 > gpurun_out/probe_32768.log 2>&1 || exit $?
timeout -k 10 300 python scripts/phys_bench.py 16384 64 2 > gpurun_out/probe_16384.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_only.py 32768 64 5 > gpurun_out/probe_ppo32768.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ppo_only.py 16384 64 5 > gpurun_out/probe_ppo16384.log 2>&1 || exit $?
cat gpurun_out/probe_32768.log gpurun_out/probe_16384.log gpurun_out/probe_ppo32768.log gpurun_out/probe_ppo16384.log
