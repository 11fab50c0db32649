# k_ppo_grad_ws without scratch (the gather's lane group through an opaque copy) vs the previous
# build (libwk_wsold.so: 4 VGPRs / 20 B scratch, one scratch load before every chunk's gather):
# the update's weights bit for bit, the gradient / update tests, then gradient and update times.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/ppo-bipedalwalker_amd
OUT=gpurun_out/wsspill; mkdir -p $OUT; rm -f $OUT/ab.log
for lib in libwk_wsold.so libwk.so; do
  WK_LIB=$L/$lib timeout -k 10 120 python scripts/update_weights.py 65536 $OUT/w_$lib.npy > $OUT/w_$lib.log 2>&1 || exit $?
done
python3 -c "import numpy as np; a=np.load('$OUT/w_libwk_wsold.so.npy'); b=np.load('$OUT/w_libwk.so.npy'); print('weights bit-identical:', a.tobytes()==b.tobytes())"
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad_scale.py tests/test_gpu_baseline_shapes.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for lib in libwk_wsold.so libwk.so; do
  echo "== $lib" >> $OUT/ab.log
  WK_LIB=$L/$lib timeout -k 10 300 python -u scripts/grad_impls.py ws 65536,32768 >> $OUT/ab.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/ab.log
