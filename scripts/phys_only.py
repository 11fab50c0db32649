"""One launch of the fused env-step kernel (for rocprofv3 counter passes).
  python scripts/phys_only.py [walkers] [horizon] [lanes] [rollout|physics]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import torch
import wk
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
L = int(sys.argv[3]) if len(sys.argv) > 3 else 1
mode = sys.argv[4] if len(sys.argv) > 4 else "rollout"
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, LanesPerWalker=L)
if mode == "rollout":
    eng.rollout(T)
else:
    act = torch.rand((T, n, 4), device="cuda") * 2 - 1
    torch.cuda.synchronize()
    eng.step_device(act.data_ptr(), T, None, None, None, None)
eng.sync()
print("ok", n, T, L, mode)
