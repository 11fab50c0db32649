# WRITE_SIZE of the 65,536-walker rollout launches: default build (LDS contact faces) vs a build
# with -DWK_FACE_LDS=0 (libwk_nofl.so), same bench command as scripts/r04_wtraffic.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wtraffic_faces; mkdir -p $OUT
for L in libwk.so libwk_nofl.so; do
  WK_LIB=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd/$L timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_env_side" -d $OUT/$L -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/$L.json 2> $OUT/$L.err; rc=$?; echo "$L rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
