"""Generate the committed golden fixtures from the CPU oracle (SURVEY.md 8(c) list).

The reference (C#/.NET + MonoGame) cannot be built or run here, so these vectors come
from the oracle restatement after it passes the hand-derived KATs
(tests/test_oracle_kat.py).  They pin the oracle against regressions and give the
GPU parity tests fixed inputs/outputs.  Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import orc  # noqa: E402

SEED = 20250905


def env_step_trace():
    """(i) one env-step from the template with action [0.5, -0.5, 0.25, -0.25]."""
    e = orc.Env()
    s0 = e.dump()
    obs, r, d, tr = e.step([0.5, -0.5, 0.25, -0.25], trace=True)
    return dict(state0=s0, action=np.array([0.5, -0.5, 0.25, -0.25], np.float32),
                obs=obs, reward=np.float32(r), done=np.int32(d), state1=e.dump(),
                aabb_hit=tr["aabb_hit"], sat_hit=tr["sat_hit"], n_contacts=tr["n_contacts"],
                normal=tr["normal"], depth=tr["depth"])


def thousand_steps(n_env=8, steps=1000, every=100):
    """(ii) 1000 env-steps for 8 envs (Philox start offsets + action stream)."""
    snaps = np.zeros((steps // every, n_env, orc.STATE_FLOATS), np.float32)
    rewards = np.zeros((steps, n_env), np.float32)
    dones = np.zeros((steps, n_env), np.uint8)
    dx = np.array([orc.env_offset(SEED, e) for e in range(n_env)], np.float32)
    envs = [orc.Env(dx=float(dx[e])) for e in range(n_env)]
    for t in range(steps):
        for i, env in enumerate(envs):
            _, r, d = env.step(orc.synth_action(SEED, i, t))
            rewards[t, i] = r
            dones[t, i] = d
        if (t + 1) % every == 0:
            for i, env in enumerate(envs):
                snaps[(t + 1) // every - 1, i] = env.dump()
    return dict(dx=dx, snaps=snaps, rewards=rewards, dones=dones)


def train_batch():
    """(iii) one Train(Batch) (B = 64) on fixed weights and inputs."""
    rng = np.random.default_rng(7)
    ag = orc.Agent(seed=SEED)
    w0 = ag.params()
    B = 64
    states = rng.normal(0, 0.5, (B, 12)).astype(np.float32)
    actions = np.zeros((B, 4), np.float32)
    logp = np.zeros((B, 4), np.float32)
    for i in range(B):
        a, lp = ag.sample(states[i], SEED, i, 0)
        actions[i] = a
        # perturb the old log-probs so the ratio leaves the clip range on some samples
        logp[i] = lp + rng.normal(0, 0.3, 4).astype(np.float32)
    returns = rng.normal(0, 2, B).astype(np.float32)
    adv = rng.normal(0, 1, B).astype(np.float32)
    g, cd, ad, sk = ag.train_batch(states, actions, logp, returns, adv)
    return dict(w0=w0, states=states, actions=actions, logp_old=logp, returns=returns, adv=adv,
                grads=g, w1=ag.params(), critic_diag=np.float32(cd), actor_diag=np.float32(ad),
                skipped=np.int32(sk))


def returns_vectors():
    """(iv) MC and GAE returns on a 1001-step reward/value vector."""
    rng = np.random.default_rng(11)
    r = rng.normal(0, 1, 1001).astype(np.float32)
    v = rng.normal(0, 1, 1001).astype(np.float32)
    mc_ret, mc_adv = orc.returns_mc(r, v, None, 0.9)
    gae_ret, gae_adv = orc.returns_gae(r, v, None, 0.9, 0.95)
    return dict(r=r, v=v, mc_ret=mc_ret, mc_adv=mc_adv, gae_ret=gae_ret, gae_adv=gae_adv)


def main():
    orc.build()
    out = {
        "env_step_trace.npz": env_step_trace(),
        "thousand_steps.npz": thousand_steps(),
        "train_batch.npz": train_batch(),
        "returns.npz": returns_vectors(),
    }
    for name, d in out.items():
        np.savez_compressed(os.path.join(HERE, name), **d)
        print("wrote", name, sum(np.asarray(v).nbytes for v in d.values()), "bytes")


if __name__ == "__main__":
    main()
