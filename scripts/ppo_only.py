"""One PPO update (E epochs x pool/M minibatches) after a rollout, for profiling.
  python scripts/ppo_only.py [walkers] [horizon] [epochs]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
E = int(sys.argv[3]) if len(sys.argv) > 3 else 1
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=E)
eng.rollout(T)
eng.ppo_update()
eng.sync()
eng.profile_reset(); eng.profile_enable(True)
t0 = time.perf_counter()
eng.ppo_update(update_index=1)
eng.sync()
dt = time.perf_counter() - t0
p = eng.profile()
print(f"ppo_update {dt*1e3:.2f} ms", {k: round(v, 3) for k, v in p.items()})
