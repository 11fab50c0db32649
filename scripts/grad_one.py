"""One PPO update pass (E = 1) at M = walkers (default 65,536: 64 gradient launches) for counter
collection.  python scripts/grad_one.py [walkers]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk
n, T = (int(sys.argv[1]) if len(sys.argv) > 1 else 65536), 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=1)
eng.rollout(T)
eng.ppo_update(minibatch=n, update_index=0)
eng.sync()
print("ok")
