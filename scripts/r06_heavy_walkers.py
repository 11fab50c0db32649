"""Why the episode-0 waves are the slowest (profiles/r06_wave_clock.txt): per-walker pair events in
the bench regime, episode-0 walkers against post-reset ones.  8 PPO iterations at T_h 64 from the
seeded start (the bench's regime), then K policy env-steps traced per substep (wk_step_traced):
per walker-substep the leg-leg / leg-floor / torso-floor bounding-box hits, SAT collisions, contact
points and active joints (pair slots: csrc/wk_physics.hip substep), by group.
  python scripts/r06_heavy_walkers.py [walkers] [env-steps]"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
eng = wk.Engine(n, seed=20250905, Horizon=64, Minibatch=min(n, 65536), MinibatchGlobal=65536,
                RandomizeStart=1)
for it in range(8):
    eng.rollout(64)
    eng.ppo_update(update_index=it)
st = eng.get_state()
ep0 = st[:, 109] == 0.0
print(f"walkers {n}, episode-0 {int(ep0.sum())} (mean episode step {st[ep0, 108].mean():.0f}), post-reset "
      f"mean episode step {st[~ep0, 108].mean():.0f}; torso y: ep0 {st[ep0, 105].mean():.1f}, "
      f"post {st[~ep0, 105].mean():.1f}", flush=True)
LL, LF = [0, 2, 5, 7], [1, 3, 6, 8]
acc = {k: [] for k in ("ll_box", "ll_sat", "ll_con", "lf_box", "lf_sat", "lf_con", "tf_box", "joints")}
for k in range(K):
    _, act, _ = eng.policy_sample(eng.get_obs())
    tr = eng.step_traced(act)
    box, sat, nc = tr["aabb_hit"].astype(np.float64), tr["sat_hit"].astype(np.float64), tr["n_contacts"].astype(np.float64)
    acc["ll_box"].append(box[:, :, LL].sum(-1)); acc["ll_sat"].append(sat[:, :, LL].sum(-1))
    acc["ll_con"].append(nc[:, :, LL].sum(-1)); acc["lf_box"].append(box[:, :, LF].sum(-1))
    acc["lf_sat"].append(sat[:, :, LF].sum(-1)); acc["lf_con"].append(nc[:, :, LF].sum(-1))
    acc["tf_box"].append(box[:, :, 4]); acc["joints"].append((tr["joint_depth"] >= 0.1).sum(-1).astype(np.float64))
    ep_now = eng.get_state()[:, 109] == 0.0
print("per walker-substep (mean over the traced env-steps):  episode-0 | post-reset")
for key, v in acc.items():
    m = np.stack(v, 0).mean(axis=(0, 2))  # per walker
    print(f"  {key:8s} {m[ep0].mean():7.3f} | {m[~ep0].mean():7.3f}")
