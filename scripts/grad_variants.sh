#!/bin/bash
# grad-kernel A/B: kernel-trace mean duration of k_ppo_grad_mfma per minibatch size for each
# variant library (LIBS="libwk.so libwk_x.so ...")
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gradvar
for lib in ${LIBS:-libwk.so}; do
  WK_LIB=ppo-bipedalwalker_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gradvar/$lib -o run --output-format csv -- python3 scripts/grad_scaling.py > gpurun_out/gradvar/$lib.log 2>&1 || exit $?
  echo "== $lib"
  python3 scripts/trace_by_grid.py gpurun_out/gradvar/$lib/run_kernel_trace.csv | grep -E "grad" | cut -d, -f1,2,4,6,7
done
