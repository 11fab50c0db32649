#!/bin/bash
# GPU box: the exchange measured, not assumed.  N ranks of bench.py's multi-rank
# path on the one GPU (--rehearse, IPC exchange), each rank its own process under
# `rocprofv3 --kernel-trace --stats` (the program after -- is python itself), started from this
# shell with the env:// rendezvous variables (no launcher process in between); --xch-profile
# stamps k_reduce_xch_adam per block (entry / published / peers seen / exit) for one untimed
# iteration.  Shard shape: 8,192 walkers and an 8,192-sample minibatch per rank, T_h 64, E 5.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r06_xch
mkdir -p $out
for n in ${RANKS:-2 4}; do
  port=$((29600 + RANDOM % 300))
  pids=()
  for r in $(seq 0 $((n - 1))); do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/n${n}_r$r -o run --output-format csv -- \
      python3 bench.py --gpus $n --steps 3 --warmup 1 --rehearse --walkers 8192 \
      --minibatch-global $((8192 * n)) --regime-iters 2 --xch-profile \
      --detail-file $out/detail_n${n}_r$r.json > $out/line_n${n}_r$r.txt 2> $out/err_n${n}_r$r.txt &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  [ $rc -eq 0 ] || { echo "ranks=$n failed rc=$rc"; tail -5 $out/err_n${n}_r*.txt; exit $rc; }
  echo "== ranks=$n"; cat $out/line_n${n}_r0.txt
done
