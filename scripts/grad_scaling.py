"""Gradient-kernel time vs minibatch size (per-launch overhead vs per-chunk cost)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk
n, T = 65536, 64
eng = wk.Engine(n, seed=20250905, Horizon=T, RandomizeStart=1, Minibatch=n, Epochs=1)
eng.rollout(T)
sizes = [int(x) for x in os.environ.get("WK_GRAD_SIZES", "16384 32768 65536 131072 262144").split()]
for M in sizes:
    eng.ppo_update(minibatch=M, update_index=0)
    eng.sync()
    eng.profile_reset(); eng.profile_enable(2)
    eng.ppo_update(minibatch=M, update_index=1)
    eng.sync(); eng.profile_enable(0)
    p = eng.profile()
    g = p["grad_ms"] / p["grad_launches"] * 1e3
    r = p["reduce_ms"] / max(1, p["reduce_launches"]) * 1e3
    print(f"M={M:7d} launches={p['grad_launches']:4d} grad {g:8.1f} us  reduce+adam {r:6.1f} us  "
          f"per 1k samples {g / (M / 1000):6.3f} us", flush=True)
