"""The oracle reproduces the committed golden fixtures (tests/golden/make_golden.py)."""
import numpy as np

SEED = 20250905


def test_env_step_trace(orc, golden):
    g = golden("env_step_trace.npz")
    e = orc.Env()
    np.testing.assert_array_equal(e.dump(), g["state0"])
    obs, r, d, tr = e.step(g["action"], trace=True)
    np.testing.assert_array_equal(obs, g["obs"])
    assert r == g["reward"] and d == g["done"]
    np.testing.assert_array_equal(e.dump(), g["state1"])
    for k in ("aabb_hit", "sat_hit", "n_contacts", "normal", "depth"):
        np.testing.assert_array_equal(tr[k], g[k])


def test_thousand_steps(orc, golden):
    g = golden("thousand_steps.npz")
    n = g["dx"].size
    envs = [orc.Env(dx=float(g["dx"][i])) for i in range(n)]
    for t in range(1000):
        for i, e in enumerate(envs):
            _, r, d = e.step(orc.synth_action(SEED, i, t))
            assert r == g["rewards"][t, i] and d == g["dones"][t, i]
        if (t + 1) % 100 == 0:
            snap = np.stack([e.dump() for e in envs])
            np.testing.assert_array_equal(snap, g["snaps"][(t + 1) // 100 - 1])


def test_train_batch(orc, golden):
    g = golden("train_batch.npz")
    ag = orc.Agent(seed=SEED)
    np.testing.assert_array_equal(ag.params(), g["w0"])
    grads, cd, ad, sk = ag.train_batch(g["states"], g["actions"], g["logp_old"], g["returns"], g["adv"])
    np.testing.assert_array_equal(grads, g["grads"])
    np.testing.assert_array_equal(ag.params(), g["w1"])
    assert cd == g["critic_diag"] and ad == g["actor_diag"] and sk == g["skipped"]


def test_returns(orc, golden):
    g = golden("returns.npz")
    ret, adv = orc.returns_mc(g["r"], g["v"], None, 0.9)
    np.testing.assert_array_equal(ret, g["mc_ret"])
    np.testing.assert_array_equal(adv, g["mc_adv"])
    ret, adv = orc.returns_gae(g["r"], g["v"], None, 0.9, 0.95)
    np.testing.assert_array_equal(ret, g["gae_ret"])
    np.testing.assert_array_equal(adv, g["gae_adv"])


def test_episode_mask_equals_separate_episodes(orc):
    # batched extension: a done mask splits the scan exactly like separate trajectories
    rng = np.random.default_rng(3)
    r = rng.normal(size=10).astype(np.float32)
    v = rng.normal(size=10).astype(np.float32)
    d = np.zeros(10, np.uint8)
    d[3] = 1
    ret, adv = orc.returns_mc(r, v, d, 0.9)
    r1, a1 = orc.returns_mc(r[:4], v[:4], None, 0.9)
    r2, a2 = orc.returns_mc(r[4:], v[4:], None, 0.9)
    np.testing.assert_array_equal(ret, np.concatenate([r1, r2]))
    np.testing.assert_array_equal(adv, np.concatenate([a1, a2]))
