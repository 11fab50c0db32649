"""GPU: walkers with a non-finite vertex follow the reference's NaN semantics.

SATCollision.IsColliding (SATCollision.cs:15-104) returns false as soon as an axis's
projections do not overlap; with a NaN vertex the edge axes next to it are NaN, every
projection on them is NaN, `Projection.IsOverlapping`'s compares are false (`:100-104`), and
the pair does not collide.  The kernels decide SAT as `depth > 0` over a NaN-propagating
minimum (v_minimum3, .NET Math.Min's IEEE 754:2019 semantics), so a NaN axis keeps depth NaN
and the verdict false -- in every mapping, including the split ones that combine two lanes'
depths.  The oracle (oracle/orc_physics.c) restates the reference's compares directly.

Walkers 0-15 get a NaN lower-left-leg vertex 0 (not a joint point: the leg keeps moving,
Skeleton.Rotate / Move carry the NaN, the centroid is never recomputed), walkers 16-31 a NaN
x on the right lower leg's vertex 5, walkers 32-39 a NaN torso vertex 3; the legs reach the
floor within the first env-steps, so the bounding boxes overlap (Collided, RigidBody.cs:73-76)
while SAT must say no.  Per-substep bookkeeping, states, rewards and dones must equal the
oracle's bit for bit (NaN where the oracle has NaN), and the fault bit flags those walkers.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905
LLL, RLL, BODY = 0, 3, 2


def _inject(st):
    st = st.copy()
    st[0:16, LLL * 20 + 0] = np.nan
    st[0:16, LLL * 20 + 1] = np.nan
    st[16:32, RLL * 20 + 10] = np.nan
    st[32:40, BODY * 20 + 6] = np.nan
    return st


@pytest.mark.parametrize("lanes", [1, 2, 4, 16])
def test_nan_vertex_walkers_match_oracle(wk, orc, lanes):
    n, k_traced, k_more = 64, 24, 40
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, LanesPerWalker=lanes)
    st = _inject(eng.get_state())
    eng.set_state(st)
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e)), material=int(orc.env_material(SEED, e)))
            for e in range(n)]
    for i, e in enumerate(envs):
        e.load(st[i])
    rng = np.random.default_rng(7)
    acts = rng.uniform(-1.2, 1.2, (k_traced + k_more, n, 4)).astype(np.float32)
    nan_leg_box_hits = 0
    for t in range(k_traced):
        tr = eng.step_traced(acts[t])
        for i, e in enumerate(envs):
            _, _, _, ot = e.step(acts[t, i], trace=True)
            for key in ("aabb_hit", "sat_hit", "n_contacts"):
                np.testing.assert_array_equal(tr[i][key], ot[key], err_msg=f"t {t} env {i} {key}")
            for key in ("normal", "depth", "contact", "impulse", "joint_depth", "joint_impulse"):
                np.testing.assert_array_equal(tr[i][key], ot[key], err_msg=f"t {t} env {i} {key}")
        # pair 1 = (LLL, FLOOR), 6 = (RLL, FLOOR): box overlap but never a SAT collision
        nan_leg_box_hits += int(tr[:16]["aabb_hit"][:, :, 1].sum() + tr[16:32]["aabb_hit"][:, :, 6].sum())
        assert not tr[:16]["sat_hit"][:, :, [0, 1, 2]].any()
        assert not tr[16:32]["sat_hit"][:, :, [5, 6, 7]].any()
        np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]),
                                      err_msg=f"t {t}")
    assert nan_leg_box_hits > 0  # the NaN legs did reach the floor's bounding box
    obs, rew, done, fault = eng.step(acts[k_traced:], k=k_more)
    for i, e in enumerate(envs):
        for t in range(k_more):
            o, r, d = e.step(acts[k_traced + t, i])
            np.testing.assert_array_equal(o, obs[t, i], err_msg=f"t {t} env {i}")
            assert (r == rew[t, i] or (np.isnan(r) and np.isnan(rew[t, i]))) and d == done[t, i]
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    # WK_FAULT_NONFINITE for the walkers still carrying a NaN at the end of an env-step of
    # this call (an auto-reset rebuilds the template, clearing it)
    still_nan = np.isnan(eng.get_state()[:40]).any(axis=1)
    assert (fault[:40][still_nan] & 1).all()
    assert not (fault[40:] & 1).any()
