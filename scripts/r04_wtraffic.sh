set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wtraffic; mkdir -p $OUT
for O in 0 1; do
  WK_ORDER=$O timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/o$O -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras --regime-iters 8 > $OUT/o$O.json 2> $OUT/o$O.err; echo "order $O rc=$?"
done
