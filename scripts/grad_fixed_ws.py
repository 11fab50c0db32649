"""k_ppo_grad_ws kernel time (HIP events around each launch, profile level 2) at a few
minibatch sizes, for fixed-cost probe builds: python scripts/grad_fixed_ws.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk  # noqa: E402
n, T = 16384, 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=8192, Epochs=1)
eng.rollout(T)
for M in (2048, 8192, 65536):
    eng.ppo_update(minibatch=M, update_index=0)
    eng.sync()
    eng.profile_reset(); eng.profile_enable(2)
    eng.ppo_update(minibatch=M, update_index=1)
    eng.sync(); eng.profile_enable(0)
    p = eng.profile()
    print(f"M={M:6d} grad {p['grad_ms'] / p['grad_launches'] * 1e3:7.2f} us", flush=True)
