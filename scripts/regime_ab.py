"""Rollout A/B in the bench's regime: for each walker count, a context runs --regime-iters PPO
iterations (rollout + update) from the seeded start, snapshots, then times `reps` rollouts
(restore + rollout, HIP events around the physics launch) -- once per variant, where a
variant is a set of environment variables read by wk_create (e.g. WK_ORDER=0).  Also prints
the share of walkers still in their first episode at the snapshot (S_POSTRESET == 0) and
checks that every variant produces the same trajectory bit for bit.

  python scripts/regime_ab.py 65536,8192 "WK_ORDER=0" "WK_ORDER=1"
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import numpy as np  # noqa: E402
import wk  # noqa: E402

sizes = [int(x) for x in sys.argv[1].split(",")]
variants = sys.argv[2:] or [""]
T, R, reps = 64, 8, int(os.environ.get("REPS", "5"))
updates = os.environ.get("REGIME_UPDATES", "1") != "0"  # 0: rollouts only (weights stay at init,
# so walker e's trajectory is the same whatever the walker count: chain-floor comparisons)
for n in sizes:
    ref = None
    for var in variants:
        saved = {}
        for kv in var.split():
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        eng = wk.Engine(n, seed=20250905, Horizon=T, Minibatch=min(n, 65536),
                        MinibatchGlobal=65536, RandomizeStart=1,
                        RoughFloor=int(os.environ.get("REGIME_ROUGH", "0")),
                        LanesPerWalker=int(os.environ.get("REGIME_LANES", "0")))
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        for it in range(R):
            eng.rollout(T)
            if updates:
                eng.ppo_update(update_index=it, sync=False)
        eng.snapshot()
        st = eng.get_state()
        ep0 = float((st[:, 109] == 0).mean())
        eng.restore()
        eng.rollout(T)  # warm
        eng.profile_reset()
        eng.profile_enable(1)
        for _ in range(reps):
            eng.restore()
            eng.rollout(T)
        p = eng.profile()
        eng.profile_enable(0)
        tr = eng.get_trajectory(T)
        same = "" if ref is None else (
            " same" if all(np.array_equal(tr[k], ref[k]) for k in tr) else " DIFFERENT")
        if ref is None:
            ref = tr
        ms = p["physics_ms"] / max(1, p["physics_launches"])
        mp = eng.rollout_mapping()
        print(f"n={n:6d} [{var or 'default'}] {mp} episode-0 share {ep0:.3f}  rollout {ms:8.3f} ms "
              f"({n * T / ms / 1e3:7.2f} M env-steps/s, {ms * 1e3 / (T * 50):.3f} us per substep){same}",
              flush=True)
        eng.close()
