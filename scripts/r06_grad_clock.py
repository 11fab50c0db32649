"""Phase clock of one k_ppo_grad_ws launch (probe build: thread 0 of every block stamps s_memtime at
entry, after the weight staging, after each chunk step's barrier, after the partial sums, after the
slab writes and at exit -- a scratch copy of wk_ppo_mfma.hip, not the product source).
  WK_LIB=ppo-bipedalwalker_amd/libwk_gclk.so python scripts/r06_grad_clock.py"""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_gclk.so"))
import wk  # noqa: E402

n = 65536
eng = wk.Engine(n, seed=20250905, Horizon=64, RandomizeStart=1, Minibatch=n, MinibatchGlobal=n)
lib = eng.lib
lib.wk_grad_clock.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * (1024 * 16))()
for it in range(3):
    eng.rollout(64)
    eng.ppo_update(update_index=it)
    eng.sync()
lib.wk_grad_clock(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.int64)[:256]
names = ["stage", "step0 (producer only)", "step1", "step2", "step3", "step4 (consumer only)",
         "loop end -> partials in R", "row sums -> slabs", "fold + stores"]
pts = [0, 1, 2, 3, 4, 5, 6, 8, 9, 10]
d = np.diff(a[:, pts], axis=1)
tot = a[:, 10] - a[:, 0]
print(f"blocks 256, shader ticks per phase (mean / min / max), total per block mean {tot.mean():.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:28s} {d[:, i].mean():8.0f} {d[:, i].min():8.0f} {d[:, i].max():8.0f}")
print(f"entry skew (max-min over blocks) {a[:, 0].max() - a[:, 0].min()} ticks; "
      f"exit skew {a[:, 10].max() - a[:, 10].min()}; span {a[:, 10].max() - a[:, 0].min()}")
