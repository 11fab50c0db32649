"""Can a launch-start key tell which episode-0 walkers reset during the next 64-env-step launch?
(The episode-0 waves run mixed after their first reset -- profiles/r06_region_by_class.txt -- so a
lane order that groups the soon-to-reset walkers would keep the others' waves uniform longer.)
Bench regime at 65,536 walkers; for the episode-0 walkers at the snapshot: torso height / angle /
angular and vertical velocity and episode step against 'reset within the launch', as ROC AUC."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import wk  # noqa: E402

n = 65536
eng = wk.Engine(n, seed=20250905, Horizon=64, Minibatch=n, MinibatchGlobal=n, RandomizeStart=1)
for it in range(8):
    eng.rollout(64)
    eng.ppo_update(update_index=it)
s0 = eng.get_state()
eng.rollout(64)
s1 = eng.get_state()
ep0 = s0[:, 109] == 0.0
reset = ep0 & (s1[:, 109] != 0.0)
print(f"episode-0 walkers {int(ep0.sum())}, of them reset within the launch {int(reset.sum())}")
# body records: 5 bodies x 20 floats? print the record layout hints
def auc(x, y):
    o = np.argsort(x)
    r = np.empty(len(x)); r[o] = np.arange(len(x))
    pos = y.sum(); neg = len(y) - pos
    return (r[y].sum() - pos * (pos - 1) / 2) / max(pos * neg, 1)
e = np.flatnonzero(ep0)
y = reset[e]
feats = {}
for j in range(100):
    feats[f"f{j}"] = s0[e, j]
res = sorted(((abs(auc(v, y) - 0.5), k, auc(v, y)) for k, v in feats.items()), reverse=True)[:12]
for d, k, a in res:
    print(f"  state float {k}: AUC {a:.3f}")
