set -u
P=ppo-bipedalwalker_amd
for rep in 1 2; do
  for lib in libwk.so libwk_sch.so; do
    echo "== $lib"; WK_LIB=$P/$lib REPS=4 timeout -k 10 200 python -u scripts/regime_ab.py 65536,8192 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
