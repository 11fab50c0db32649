#!/bin/bash
# GPU box: the update's measurements for profiles/ (ROUND=r03): gradient kernels per minibatch
# size, the tile-parallel kernel's phase stamps (needs libwk_gprof.so: bash scripts/variant.sh
# gprof -DWK_GRAD_PROF wk_ppo_mfma.hip, built on the CPU side) and a kernel trace of one update at
# the 8,192-sample shard with launch gaps.
set -u
R=${ROUND:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/upd; mkdir -p $O
timeout -k 10 300 python3 -u scripts/grad_impls.py ws,tp 4096,8192,16384,24576,32768,65536 2>&1 | grep -v amdgpu.ids > $O/${R}_grad_kernels.txt || exit 1
WK_LIB=$PWD/ppo-bipedalwalker_amd/libwk_gprof.so WK_GRAD_IMPL=tp timeout -k 10 120 python3 -u scripts/grad_prof_tp.py 4096,8192,65536 2>&1 | grep -v amdgpu.ids > $O/${R}_grad_tp_phases.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace8192 -o run --output-format csv -- python3 scripts/ppo_only.py 8192 64 5 > $O/trace_log.txt 2>&1 || exit 1
f=$(find $O/trace8192 -name "*kernel_trace.csv" | head -1)
{ grep ppo_update $O/trace_log.txt | cut -c1-60; python3 scripts/trace_gaps.py $f 100; } > $O/${R}_ppo_trace_8192.txt
cat $O/${R}_grad_kernels.txt $O/${R}_ppo_trace_8192.txt
