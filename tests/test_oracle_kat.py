"""Known-answer tests pinning the CPU oracle to values derived by hand from the
reference source.  The reference ships no tests or fixtures
and cannot be built here (no .NET), so these KATs are the oracle's only pin."""
import numpy as np
import pytest

f32 = np.float32


def test_k1_template_geometry(orc):
    # Pole.FromSize(centroid, 75) (Pole.cs:18-34): half-width 0.1f*75 = 7.5, half-height 26.25
    s = orc.Env().dump()
    llu = s[20:40]
    exp = np.array([132.5, 856.25, 125, 856.25, 117.5, 856.25, 117.5, 803.75, 125, 803.75,
                    132.5, 803.75], f32)
    assert np.array_equal(llu[:12], exp)
    assert (llu[12], llu[13]) == (125.0, 830.0)
    lll = s[0:20]
    assert np.array_equal(lll[:12], exp + np.array([0, 30] * 6, f32))
    assert (lll[12], lll[13]) == (125.0, 860.0)
    body = s[40:60]  # Walker.cs:158-165, centroid (125, 804) exactly
    assert np.array_equal(body[:10], np.array([145, 820, 125, 820, 105, 820, 105, 780, 145, 780], f32))
    assert (body[12], body[13]) == (125.0, 804.0)
    # InitialState: previous position (125, 800), position = Body centroid
    assert tuple(s[104:108]) == (125.0, 804.0, 125.0, 800.0)
    assert s[109] == 0.0  # episode 0: floor last in the body list


def test_k2_dt():
    dt = f32(166667 / 1e7)  # MonoGame TargetElapsedTime (ticks) -> (float)TotalSeconds
    assert dt == f32(0.0166667)
    assert dt / f32(50) == f32(0.00033333397)


def test_k3_sat_contacts_impulse(orc):
    c = np.array([125.0, 874.75], f32)
    pole = np.array([[c[0] + 7.5, c[1] + 26.25], [c[0], c[1] + 26.25], [c[0] - 7.5, c[1] + 26.25],
                     [c[0] - 7.5, c[1] - 26.25], [c[0], c[1] - 26.25], [c[0] + 7.5, c[1] - 26.25]], f32)
    floor = np.array([[-50, 1050], [-50, 900], [1050, 900], [1050, 1050]], f32)
    hit, n, depth = orc.sat(pole, floor, c, [500, 975])
    assert hit and depth == 1.0
    assert n[0] == 0.0 and np.signbit(n[0]) and n[1] == -1.0  # (-0, -1): first axis wins ties
    cp = orc.contacts(pole, floor, n)
    assert cp.shape == (2, 2)
    np.testing.assert_allclose(cp, [[125, 900], [132.5, 900]], atol=1e-4)
    v = 10.0
    out = orc.kat_pole_floor(v)
    # MoveObjects lifts the pole by the depth; the impulse uses r_A = (3.75, 26.25)
    assert (out[3], out[4]) == (125.0, 873.75)
    assert out[5] == 2
    denom = 5 + 3.75 ** 2 * 0.005  # 5.0703125
    assert out[1] == pytest.approx(v * (1 - 1.3 * 5 / denom), rel=1e-6)   # -0.28197 v
    assert out[2] == pytest.approx(-1.3 * v * 3.75 * 0.005 / denom, rel=1e-5)  # -0.0048074 v
    assert out[0] == 0.0  # friction impulse 0: no tangential velocity


def test_k4_joint(orc):
    e = orc.Env()
    s0 = e.dump()
    e.joint_step(0)  # bodyJointLeft: Body v1 (125, 820) <-> LLU v4 (125, 803.75), d = 16.25
    s1 = e.dump()
    assert s1[40 + 13] - s0[40 + 13] == pytest.approx(-8.125)  # Body moves up by d/2
    assert s1[20 + 13] - s0[20 + 13] == pytest.approx(8.125)   # LLU moves down by d/2
    # restitution-1 joint impulse on bodies at rest is zero
    assert s1[40 + 14] == 0.0 and s1[20 + 15] == 0.0


def test_k5_log_density(orc):
    std = np.exp(f32(-1.0), dtype=f32)
    assert orc.lib().orc_log_density(0.3, float(std), 0.3) == pytest.approx(0.08106148, abs=1e-8)
    assert f32(orc.lib().orc_log_density(0.3, float(std), 0.3)) == f32(0.08106148)


def test_k6_mc_returns(orc):
    ret, adv = orc.returns_mc(np.ones(3, f32), np.zeros(3, f32), None, 0.9)
    g1 = f32(1) + f32(1) * f32(0.9)
    g0 = f32(1) + g1 * f32(0.9)
    assert ret.tolist() == [g0, g1, 1.0]
    assert ret[0] == pytest.approx(2.71, rel=1e-6)
    np.testing.assert_array_equal(adv, ret)


def test_gae_quirk(orc):
    # PPOAgent.cs:414-434: nextGae is never updated -> A_t = delta_t
    r = np.array([1.0, 2.0, 3.0], f32)
    v = np.array([0.5, 0.25, 1.0], f32)
    ret, adv = orc.returns_gae(r, v, None, 0.9, 0.95)
    nv = np.array([v[1], v[2], 0.0], f32)
    np.testing.assert_array_equal(adv, (r + f32(0.9) * nv) - v)
    np.testing.assert_array_equal(ret, adv + v)


def test_k7_adam_first_step(orc):
    ag = orc.Agent(seed=3)
    rng = np.random.default_rng(0)
    B = 16
    s = rng.normal(0, 1, (B, 12)).astype(f32)
    a = rng.normal(0, 0.4, (B, 4)).astype(f32)
    lp = np.stack([[orc.lib().orc_log_density(float(m), float(np.exp(f32(-1))), float(x))
                    for m, x in zip(ag.mean(s[i]), a[i])] for i in range(B)]).astype(f32)
    w0 = ag.params()
    g, *_ = ag.train_batch(s, a, lp, rng.normal(0, 1, B), rng.normal(0, 1, B))
    dw = ag.params() - w0
    big = np.abs(g) > 1e-4
    assert big.sum() > 1000
    # t = 1: m_hat = g, v_hat = g^2 -> dw = -alpha * g / (|g| + 1e-8)
    np.testing.assert_allclose(dw[big], -1e-3 * np.sign(g[big]), atol=2e-7)
    m, v, t = ag.adam()
    assert t == 1


def test_k8_surrogate_gradient(orc):
    # r = 1 and A > 0: dL/dmu = -A (a - mu) / sigma^2 / B, then through tanh
    ag = orc.Agent(seed=5)
    s = np.linspace(-1, 1, 12).astype(f32)
    mu = ag.mean(s)
    std = np.exp(f32(-1.0), dtype=f32)
    a = (mu + np.array([0.1, -0.2, 0.05, 0.3], f32)).astype(f32)
    lp = np.array([orc.lib().orc_log_density(float(m), float(std), float(x)) for m, x in zip(mu, a)], f32)
    A = 1.5
    g, cd, ad, sk = ag.train_batch(s[None], a[None], lp[None], np.zeros(1), np.array([A]),
                                   apply_adam=False)
    dmu = -A * (a - mu) / (std * std)
    db3 = dmu * (1 - mu.astype(np.float64) ** 2)
    np.testing.assert_allclose(g[6145:6149], db3, rtol=1e-5)
    assert ad == pytest.approx(dmu.mean(), rel=1e-5)
    assert sk == 0


def test_k9_body_order(orc):
    a = orc.Env()
    b = orc.Env()
    b.reset()  # same template, floor first in the body list
    da, db = a.dump(), b.dump()
    assert da[109] == 0 and db[109] == 1
    da[109] = db[109] = 0
    np.testing.assert_array_equal(da, db)
    diverged = False
    for t in range(50):
        act = orc.synth_action(1, 0, t)
        a.step(act)
        b.step(act)
        x, y = a.dump(), b.dump()
        x[109] = y[109] = 0
        if not np.array_equal(x, y):
            diverged = True
            break
    assert diverged  # only the pair order differs, and it matters once a leg meets the floor


def test_philox_known_answers(orc):
    # Random123 kat_vectors, philox4x32-10
    assert orc.philox(0, [0, 0, 0, 0]).tolist() == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert orc.philox(0xffffffffffffffff, [0xffffffff] * 4).tolist() == [
        0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert orc.philox(0x299f31d0a4093822, [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344]).tolist() == [
        0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


@pytest.mark.parametrize("n", [1, 2, 3, 64, 100, 1001, 4096])
def test_minibatch_permutation_is_bijection(orc, n):
    key = orc.perm_key(7, 3, 1)
    p = [orc.perm(i, n, key) for i in range(n)]
    assert sorted(p) == list(range(n))


def test_synthetic_streams(orc):
    a = np.stack([orc.synth_action(20250905, e, t) for e in range(16) for t in range(16)])
    assert a.min() >= -1 and a.max() < 1
    mats = {orc.env_material(20250905, e) for e in range(200)}
    assert mats == {0, 1, 2}
    dx = [orc.env_offset(20250905, e) for e in range(200)]
    assert min(dx) >= 0 and max(dx) <= 200


def test_episode_terminal_rules(orc):
    # steps > MaxTimesteps ends an episode at step MaxTimesteps + 1 (Environment.cs:106-110)
    e = orc.Env(MaxTimesteps=3)
    dones = [e.step([0, 0, 0, 0])[2] for _ in range(4)]
    assert dones == [0, 0, 0, 1]
    assert e.dump()[109] == 1 and e.dump()[108] == 0
