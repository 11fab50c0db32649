"""Per-region wave time of the side-split env-step kernel, WAVE-level (round 5: the wave's first
active lane stamps every region boundary; lanes/visit = mean active lanes when the region ended) (build: make LIB=libwk_prof.so
BUILD=build_prof EXTRA=-DWK_REGION_PROF).  python scripts/region_prof.py [walkers] [T] [lanes]
REGIME_ITERS=k first runs k PPO iterations at T_h = 64 (the bench's regime protocol), so the
profiled launches see the walker mix of the timed iteration rather than the seeded start."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ.setdefault("WK_LIB", os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk_prof.so"))
import torch  # noqa: E402
import wk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
L = int(sys.argv[3]) if len(sys.argv) > 3 else 2
names = ["joint", "integrate", "aabb leg-leg", "aabb leg-floor", "aabb torso-floor", "sat leg-leg",
         "sat leg-floor", "sat torso-floor", "contact leg-leg", "contact leg-floor",
         "contact torso-floor", "move+imp leg-leg", "move+imp leg-floor", "move+imp torso-floor",
         "policy", "other"]  # (csrc/wk_region_prof.h RP_*; round 5's pool regions and round 6's
                             #  helper passes are gone with the code they timed)
NR = len(names)
R = int(os.environ.get("REGIME_ITERS", "0"))
eng = wk.Engine(n, seed=20250905, Horizon=max(T, 64 if R else T), RandomizeStart=1, LanesPerWalker=L)
for it in range(R):
    eng.rollout(64)
    eng.ppo_update(update_index=it, sync=False)
lib = eng.lib
lib.wk_region_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * (3 * NR))()
eng.rollout(T)
eng.sync()
lib.wk_region_prof(buf, 1)
for mode in ("rollout", "physics"):
    if mode == "rollout":
        eng.rollout(T)
    else:
        act = torch.rand((T, n, 4), device="cuda") * 2 - 1
        torch.cuda.synchronize()
        eng.step_device(act.data_ptr(), T, None, None, None, None)
    eng.sync()
    lib.wk_region_prof(buf, 1)
    tot = sum(buf[i] for i in range(NR))
    mp = eng.rollout_mapping()
    waves = mp["waves_launched"]
    print(f"{mode}: total {tot / waves / (T * 50):.0f} ticks per wave-substep "
          f"({waves} waves launched)")
    print(f"  {'region':22s} {'share':>7s} {'ticks/w-sub':>11s} {'visits/w-sub':>12s} {'lanes/visit':>11s}")
    for i in range(NR):
        cnt = buf[2 * NR + i]
        print(f"  {names[i]:22s} {100.0 * buf[i] / tot:6.2f}% {buf[i] / waves / (T * 50):11.1f} "
              f"{cnt / waves / (T * 50):12.3f} {buf[NR + i] / max(1, cnt):11.1f}")
