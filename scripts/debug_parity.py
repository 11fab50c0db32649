"""Find the first substep / field where the GPU physics departs from the oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ppo-bipedalwalker_amd"), os.path.join(ROOT, "oracle")]
import wk, orc
SEED = 20250905
n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
names = []
for b in ["LLL", "LLU", "BODY", "RLL", "RLU"]:
    names += [f"{b}.v{i//2}{'xy'[i%2]}" for i in range(12)] + [f"{b}.{k}" for k in ["cx","cy","vx","vy","w","th","col","pad"]]
names += ["tq0","tq1","tq2","tq3","posx","posy","prevx","prevy","steps","post","term","eps"]
eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Iterations=1)
envs = [orc.Env(dx=float(orc.env_offset(SEED, e)), material=int(orc.env_material(SEED, e)), Iterations=1) for e in range(n)]
rng = np.random.default_rng(1)
bad = 0
for t in range(steps):
    a = rng.uniform(-1.3, 1.3, (n, 4)).astype(np.float32)
    eng.step(a[None], k=1)
    for i, e in enumerate(envs):
        e.step(a[i])
    g = eng.get_state(); r = np.stack([e.dump() for e in envs])
    diff = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    if len(diff):
        envs_bad = sorted(set(diff[:, 0].tolist()))
        for ei in envs_bad[:4]:
            f = diff[diff[:, 0] == ei][:, 1]
            print(f"step {t} env {ei}: " + ", ".join(f"{names[j]} gpu={g[ei,j]!r} orc={r[ei,j]!r}" for j in f[:8]))
        bad += 1
        if bad >= 2:
            break
print("done; first divergence step" if bad else "no divergence", )
