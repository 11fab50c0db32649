#!/bin/bash
# GPU-box: bench.py's multi-rank path with N ranks on the one GPU (--rehearse), the host (gloo)
# all-reduce vs the one-shot IPC exchange; rank 0's JSON line per run (kernel_ms_one_step holds
# the exchange time per iteration).  Ranks share the GPU, so this is a plumbing / fixed-cost
# check, not an 8-GPU number.
set -u
for n in ${RANKS:-2 4}; do  # (more ranks than that on ONE GPU: the ranks' spinning exchange blocks hold the CUs a peer's gradient kernel needs)
  for x in rccl ipc; do
    port=$((29500 + RANDOM % 1000))
    echo "== ranks=$n exchange=$x"
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 3 --warmup 1 --rehearse --walkers-global $((4096 * n)) --horizon 16 --epochs 2 --regime-iters 1 --exchange $x 2>/dev/null | grep "^{" || exit 1
  done
done
