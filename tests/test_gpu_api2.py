"""GPU: the round-2 boundary additions, through the C ABI.

* wk_step_sampled -- Environment.Update with the agent's own sampling returns exactly what
  Environment.cs:70-89 records in the Trajectory (state before the step, UNCLIPPED action,
  per-dimension log-probability, reward, terminal) plus the value and the next state, so a
  single-instance C# host can train through PPOAgent.Train(Trajectory);
* wk_count_events -- the counting replay's physics events equal the oracle's per-substep
  bookkeeping (RigidBody.cs:66-96, Joint.cs:31-41) summed over the same env-steps, and the
  replay leaves the walkers in the rollout's final state bit for bit;
* wk_snapshot -- save / restore reproduces an iteration bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905
F = np.float32
LL, LF, BF = [0, 2, 5, 7], [1, 3, 6, 8], [4]  # wk_pair_trace pair slots by class


@pytest.mark.parametrize("lanes", [1, 2, 16])
def test_step_sampled_matches_oracle(wk, orc, lanes):
    n, k = 48, 6
    ag = orc.Agent(seed=SEED)
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, LanesPerWalker=lanes)
    eng.set_weights(ag.params())
    out = eng.step_sampled(k)
    for i in range(n):
        e = orc.Env(dx=float(orc.env_offset(SEED, i)), material=int(orc.env_material(SEED, i)))
        for t in range(k):
            s = out["states"][t, i]
            np.testing.assert_array_equal(s, e.obs())
            a, lp = ag.sample(s, SEED, i, t)
            np.testing.assert_allclose(out["actions"][t, i], a, rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(out["logp"][t, i], lp, rtol=1e-5, atol=1e-5)
            assert out["values"][t, i] == pytest.approx(ag.value(s), rel=1e-5, abs=1e-5)
            # the recorded unclipped action drives the physics (Environment.cs:78, 86)
            _, r, d = e.step(out["actions"][t, i])
            assert r == out["rewards"][t, i] and d == out["dones"][t, i], (i, t)
            np.testing.assert_array_equal(out["next_obs"][t, i], e.obs())
    np.testing.assert_array_equal(out["states"][1:], out["next_obs"][:-1])
    assert not out["fault"].any()


def test_step_sampled_equals_rollout(wk):
    """the host-facing call and the device rollout are the same kernel path: identical
    trajectories and final states from the same start"""
    n, k = 512, 8
    a = wk.Engine(n, seed=SEED, Horizon=k, RandomizeStart=1)
    b = wk.Engine(n, seed=SEED, Horizon=k, RandomizeStart=1)
    out = a.step_sampled(k)
    b.rollout(k)
    tr = b.get_trajectory(k)
    for key, ref in (("states", "states"), ("actions", "actions"), ("logp", "logp"),
                     ("values", "values"), ("rewards", "rewards"), ("dones", "dones")):
        np.testing.assert_array_equal(out[key], tr[ref], err_msg=key)
    np.testing.assert_array_equal(a.get_state(), b.get_state())


def test_count_events_match_oracle_bookkeeping(wk, orc):
    n, T = 64, 40
    eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, MaxTimesteps=20)
    eng.snapshot()
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    after = eng.get_state()
    eng.restore()
    eng.rollout(T)  # the restore brought back the starting state: same trajectory
    np.testing.assert_array_equal(eng.get_trajectory(T)["actions"], tr["actions"])
    eng.restore()
    eng.rollout(T)
    eng.restore()
    cnt = eng.count_events(T)
    np.testing.assert_array_equal(eng.get_state(), after)  # replay == rollout physics
    ev = dict(zip(wk.EVENTS, cnt.tolist()))
    ref = dict.fromkeys(wk.EVENTS, 0)
    for i in range(n):
        e = orc.Env(dx=float(orc.env_offset(SEED, i)), MaxTimesteps=20)
        for t in range(T):
            _, _, d, trc = e.step(tr["actions"][t, i], trace=True)
            ref["joint"] += int((trc["joint_depth"] != 0).sum())
            ref["steps_lf"] += int(trc["aabb_hit"][:, LF].any())
            ref["steps_satll"] += int(trc["sat_hit"][:, LL].any())
            for cls, slots in (("ll", LL), ("lf", LF), ("bf", BF)):
                ref["aabb_" + cls] += int(trc["aabb_hit"][:, slots].sum())
                ref["sat_" + cls] += int(trc["sat_hit"][:, slots].sum())
                ref["imp_" + cls] += int((trc["n_contacts"][:, slots] > 0).sum())
            ref["contacts"] += int(trc["n_contacts"].sum())
            ref["substeps"] += len(trc)
            ref["env_steps"] += 1
            ref["resets"] += int(d)
    assert ref["resets"] > 0 and ref["aabb_lf"] > 0
    for k in ref:
        assert ev[k] == ref[k], (k, ev[k], ref[k])


def test_count_events_rough_floor(wk, orc):
    """the counting replay on CreateRoughFloor's terrain (bench.py's rough-floor rooflines): the
    replay's physics is the rollout's bit for bit, and the classes the oracle's trace keeps on
    the rough floor (joints, leg-leg pairs, substeps, env-steps, resets) equal its bookkeeping;
    the segment pairs (untraced) count as leg-floor / torso-floor events"""
    n, T = 64, 24
    eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RoughFloor=1, MaxTimesteps=20)
    eng.snapshot()
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    after = eng.get_state()
    eng.restore()
    ev = dict(zip(wk.EVENTS, eng.count_events(T).tolist()))
    np.testing.assert_array_equal(eng.get_state(), after)
    ref = dict.fromkeys(wk.EVENTS, 0)
    for i in range(n):
        e = orc.Env(dx=float(orc.env_offset(SEED, i)), rough=(SEED, i), MaxTimesteps=20)
        for t in range(T):
            _, _, d, trc = e.step(tr["actions"][t, i], trace=True)
            ref["joint"] += int((trc["joint_depth"] != 0).sum())
            ref["aabb_ll"] += int(trc["aabb_hit"][:, LL].sum())
            ref["sat_ll"] += int(trc["sat_hit"][:, LL].sum())
            ref["imp_ll"] += int((trc["n_contacts"][:, LL] > 0).sum())
            ref["substeps"] += len(trc)
            ref["env_steps"] += 1
            ref["resets"] += int(d)
    for k in ("joint", "aabb_ll", "sat_ll", "imp_ll", "substeps", "env_steps", "resets"):
        assert ev[k] == ref[k], (k, ev[k], ref[k])
    assert ev["aabb_lf"] > 0 and ev["sat_lf"] > 0 and ev["resets"] > 0


def test_snapshot_restore_repeats_an_iteration(wk):
    n, T = 1024, 8
    eng = wk.Engine(n, seed=SEED, Horizon=T, Minibatch=1024, RandomizeStart=1)
    eng.rollout(T)
    eng.ppo_update(update_index=0)
    eng.snapshot()
    res = []
    for _ in range(2):
        eng.rollout(T)
        d = eng.ppo_update(update_index=1)
        res.append((eng.get_state(), eng.get_weights(), eng.get_adam(), d,
                    eng.get_trajectory(T)["rewards"]))
        eng.restore()
    a, b = res
    for x, y in zip(a[:2] + a[4:], b[:2] + b[4:]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a[2], b[2]):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    assert a[3] == b[3]
    with pytest.raises(wk.WkError):
        wk.Engine(8, seed=SEED).restore()  # nothing saved
