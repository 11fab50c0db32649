"""Rough floor: what a lane order by start offset would buy, measured without one -- the same
multiset of start offsets assigned to the walkers at random (what RandomizeStart does) or sorted
by walker id (each wave's walkers start over the same stretch of terrain), identity lane order
for both (WK_ORDER=0), rollout timed in the bench regime.  usage: rough_dx_sort.py n[,n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
os.environ["WK_ORDER"] = "0"
import wk  # noqa: E402

T, R, reps = 64, 8, int(os.environ.get("REPS", "3"))
for n in [int(x) for x in sys.argv[1].split(",")]:
    base = np.random.default_rng(7).uniform(0.0, 200.0, n).astype(np.float32)
    for how in ("random", "sorted", "random", "sorted"):
        dx = base if how == "random" else np.sort(base)
        eng = wk.Engine(n, seed=20250905, Horizon=T, Minibatch=min(n, 65536), MinibatchGlobal=65536,
                        RoughFloor=1)
        eng.set_offsets(dx)
        eng.reset()
        for it in range(R):
            eng.rollout(T)
            eng.ppo_update(update_index=it, sync=False)
        eng.snapshot()
        eng.restore()
        eng.rollout(T)
        eng.profile_reset()
        eng.profile_enable(1)
        for _ in range(reps):
            eng.restore()
            eng.rollout(T)
        p = eng.profile()
        eng.profile_enable(0)
        ms = p["physics_ms"] / max(1, p["physics_launches"])
        print(f"n={n:6d} dx {how:6s} {eng.rollout_mapping()} rollout {ms:8.3f} ms", flush=True)
        eng.close()
