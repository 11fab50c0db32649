"""Wave-level region profile split by wave class (scratch probe build: csrc/wk_region_prof.h's
records summed per class -- class 1 = every lane of the wave in episode 0 at the launch start,
class 0 = the rest), bench regime (8 PPO iterations at T_h 64), one rollout of T env-steps.
Which regions make the episode-0 waves the slowest (profiles/r06_wave_clock.txt)?
  WK_LIB=ppo-bipedalwalker_amd/libwk_rpcls.so python scripts/r06_region_by_class.py [T]"""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_rpcls.so"))
import wk  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 64
names = ["joint", "integrate", "aabb leg-leg", "aabb leg-floor", "aabb torso-floor", "sat leg-leg",
         "sat leg-floor", "sat torso-floor", "contact leg-leg", "contact leg-floor",
         "contact torso-floor", "move+imp leg-leg", "move+imp leg-floor", "move+imp torso-floor",
         "policy", "other"]
NR = len(names)
n = 65536
eng = wk.Engine(n, seed=20250905, Horizon=64, RandomizeStart=1, Minibatch=n, MinibatchGlobal=n)
for it in range(8):
    eng.rollout(64)
    eng.ppo_update(update_index=it, sync=False)
lib = eng.lib
lib.wk_region_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * (6 * NR))()
eng.sync()
lib.wk_region_prof(buf, 1)
eng.rollout(T)
eng.sync()
lib.wk_region_prof(buf, 1)
a = np.frombuffer(buf, dtype=np.uint64).reshape(2, 3, NR).astype(np.float64)
sub = T * 50
waves = [a[c, 2, NR - 1] / (8 * sub) for c in range(2)]  # 'other' is marked 8 times per wave-substep
print(f"waves: class 0 (mixed / post-reset) {waves[0]:.0f}, class 1 (all episode 0) {waves[1]:.0f}")
tot = [a[c, 0].sum() / max(waves[c], 1) / sub for c in range(2)]
print(f"ticks per wave-substep: class 0 {tot[0]:.0f}, class 1 {tot[1]:.0f} ({100 * (tot[1] / tot[0] - 1):+.1f} %)")
print(f"  {'region':22s} {'c0 ticks':>9s} {'c1 ticks':>9s} {'c1-c0':>7s} {'c0 visits':>9s} {'c1 visits':>9s} {'c0 lanes':>8s} {'c1 lanes':>8s}")
for i in range(NR):
    t0, t1 = (a[c, 0, i] / max(waves[c], 1) / sub for c in range(2))
    v0, v1 = (a[c, 2, i] / max(waves[c], 1) / sub for c in range(2))
    l0, l1 = (a[c, 1, i] / max(a[c, 2, i], 1) for c in range(2))
    print(f"  {names[i]:22s} {t0:9.1f} {t1:9.1f} {t1 - t0:+7.1f} {v0:9.3f} {v1:9.3f} {l0:8.1f} {l1:8.1f}")
