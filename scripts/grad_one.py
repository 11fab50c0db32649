"""One PPO update pass at M = 65,536 (64 gradient launches) for counter collection."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk
n, T = 65536, 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=1)
eng.rollout(T)
eng.ppo_update(minibatch=n, update_index=0)
eng.sync()
print("ok")
