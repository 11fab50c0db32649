"""One rollout launch of the fused physics+policy kernel (for rocprofv3 counter passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1)
eng.rollout(T)
eng.sync()
print("ok", n, T)
