#!/bin/bash
# GPU box: the wave-level region profile (probe builds, -DWK_REGION_PROF) of the pair rollout with
# and without the leg-floor helper lanes, in the bench regime; then the shard's speculation
# commit count (scripts/r06_spec_commit.py).
set -u
cd "$(dirname "$0")/.."
for v in fh0 help; do
  echo "== $v"
  WK_LIB=$PWD/ppo-bipedalwalker_amd/libwk_prof_$v.so REGIME_ITERS=8 timeout -k 10 300 python3 scripts/region_prof.py 65536 16 2 || exit 1
done
echo "== speculation commit count"
timeout -k 10 300 python3 scripts/r06_spec_commit.py 8192 16 || exit 1
