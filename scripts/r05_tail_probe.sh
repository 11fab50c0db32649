# Where the fused tail's time goes: WK_GRAD_TAIL=3 (every block drains and bumps the arrival
# counter, nothing else) and 4 (also the last arrivers' bounded wait) with the separate reduction
# launch still running, against 0 (no tail) and 2 (the sc1 tail doing the work)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tail; mkdir -p $OUT; rm -f $OUT/probe.log
for rep in 1 2; do for t in 0 3 4 2; do
  echo "== WK_GRAD_TAIL=$t" >> $OUT/probe.log
  WK_GRAD_TAIL=$t timeout -k 10 300 python -u scripts/update_ab.py 10 >> $OUT/probe.log 2>&1 || exit $?
done; done
grep -v amdgpu.ids $OUT/probe.log
