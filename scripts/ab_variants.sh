#!/bin/bash
# A/B rollout throughput for libwk variants (WK_LIB), interleaved base/variant runs
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for round in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-base v1 v2}; do
    if [ $v = base ]; then L=ppo-bipedalwalker_amd/libwk.so; else L=ppo-bipedalwalker_amd/libwk_$v.so; fi
    WK_LIB=$L timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/$v.$round.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc $v"; exit $rc;; esac
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value']/1e6, d['rollout_env_steps_per_s']/1e6, d['ppo_update_ms'])" gpurun_out/ab/$v.$round.log $v
  done
done
