"""GPU: the rough floor against the oracle, bit-exact.

CreateRoughFloor (Environment.cs:230-261) builds 10 static 4-vertex Metal segments after
the walker (15 bodies; the walker is re-appended after them on every reset).  The
reference's unseeded Random is replaced by a per-walker Philox terrain (documented
deviation); the oracle uses the same draws.  Bars as for the flat floor: bodies, flags,
rewards and dones bit-exact for every mapping (1, 2, 4 and 16 lanes per walker; the pair and
quad mappings resolve the segment pairs unsplit and keep their leg-leg split)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905
F = np.float32
lanes_param = pytest.mark.parametrize("lanes", [1, 2, 4, 16])


def rough_envs(orc, n, offset=0):
    return [orc.Env(dx=float(orc.env_offset(SEED, offset + e)),
                    material=int(orc.env_material(SEED, offset + e)),
                    rough=(SEED, offset + e)) for e in range(n)]


@lanes_param
def test_rough_multi_step_bitexact(wk, orc, lanes):
    n, k = 256, 60
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, RoughFloor=1,
                    LanesPerWalker=lanes)
    envs = rough_envs(orc, n)
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    rng = np.random.default_rng(9)
    acts = rng.uniform(-1.2, 1.2, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    ndone = 0
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
            np.testing.assert_array_equal(o, obs[t, i])
            ndone += d
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    assert ndone > 0 and not fault.any()


@lanes_param
def test_rough_trace_bitexact(wk, orc, lanes):
    """per-substep pair trace: joints and the leg-segment pairs (floor-segment pairs are
    not traced in either implementation)"""
    n = 64
    eng = wk.Engine(n, seed=SEED, RoughFloor=1, LanesPerWalker=lanes)
    envs = [orc.Env(rough=(SEED, e)) for e in range(n)]
    acts = np.random.default_rng(2).uniform(-1, 1, (n, 4)).astype(F)
    tr = eng.step_traced(acts)
    for i, e in enumerate(envs):
        _, _, _, t = e.step(acts[i], trace=True)
        for key in ("aabb_hit", "sat_hit", "n_contacts", "normal", "depth", "contact", "impulse",
                    "joint_depth", "joint_impulse"):
            np.testing.assert_array_equal(tr[i][key], t[key], err_msg=f"env {i} {key}")
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))


@lanes_param
def test_rough_rollout_replays_exactly(wk, orc, lanes):
    n, T = 128, 48
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RoughFloor=1, Horizon=T, LanesPerWalker=lanes)
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e)), rough=(SEED, e)) for e in range(n)]
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    for i, e in enumerate(envs):
        for t in range(T):
            np.testing.assert_array_equal(tr["states"][t, i], e.obs(), err_msg=f"env {i} t {t}")
            _, r, d = e.step(tr["actions"][t, i])
            assert r == tr["rewards"][t, i] and d == tr["dones"][t, i], (i, t)
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))


def test_rough_body_views(wk, orc):
    n = 8
    eng = wk.Engine(n, seed=SEED, RoughFloor=1, EnvOffset=1000)
    envs = [orc.Env(rough=(SEED, 1000 + e)) for e in range(n)]
    for i, e in enumerate(envs):
        segs = e.floor_bodies()
        assert len(segs) == 10
        for k, verts in enumerate(segs):
            v = eng.body_view(i, 5 + k)
            assert v.n_vertices == 4 and v.is_static == 1
            np.testing.assert_array_equal(np.array(v.vertices[:4]), verts)
            np.testing.assert_array_equal(np.array(v.centroid[:]), verts.sum(0, dtype=F) * F(0.25))
    with pytest.raises(wk.WkError):
        eng.body_view(0, 15)


@pytest.mark.parametrize("lanes", [2, 4, 16])
def test_rough_first_segment_degenerate_edges(wk, orc, lanes):
    """walkers placed over segment 0 (three collinear vertices; a zero edge when draws 0
    and 1 coincide -- about 1 walker in 100): SAT skips the zero axis and the contact
    faces take Normalize's NaN exactly as the reference does"""
    n, k = 4096, 25
    eng = wk.Engine(n, seed=SEED, RoughFloor=1, LanesPerWalker=lanes)
    eng.set_offsets(np.full(n, -150.0, F))  # start x = -25
    eng.reset()
    envs = [orc.Env(dx=-150.0, rough=(SEED, e)) for e in range(n)]
    for e in envs:
        e.reset()
    degenerate = sum(orc.terrain_draws(SEED, e)[0] == orc.terrain_draws(SEED, e)[1] for e in range(n))
    assert degenerate > 10
    acts = np.random.default_rng(4).uniform(-1, 1, (k, n, 4)).astype(F)
    obs, rew, done, _ = eng.step(acts, k=k)
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))


@pytest.mark.parametrize("n,lanes", [(65536, 2), (8192, 4)], ids=["65536-pair", "8192-quad"])
def test_rough_bench_size_rollout_sampled_replay(wk, orc, n, lanes):
    """the rough floor's bench lines at their sizes (`rough_floor_65536`: the pair mapping,
    `rough_floor_shard_8192`: the sparse quad mapping; the fused policy, the lane order and the
    terrain in LDS over the whole grid): a sample of the walkers -- the first and last of every
    eighth block and 256 at random -- replayed through the oracle with the GPU's own recorded
    actions, states / rewards / dones and final records bit for bit"""
    T = 64
    eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RoughFloor=1, Minibatch=n, Epochs=1)
    m = eng.rollout_mapping()
    assert m["lanes_per_walker"] == lanes
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    state = eng.get_state()
    wpb = 256 // lanes if lanes == 2 else 4 * m["walkers_per_wave"]  # walkers per 4-wave block
    blocks = np.arange(0, n // wpb, 8)
    rng = np.random.default_rng(n)
    sample = np.unique(np.concatenate([blocks * wpb, blocks * wpb + wpb - 1, rng.choice(n, 256, replace=False)]))
    ndone = 0
    for i in sample:
        e = orc.Env(dx=float(orc.env_offset(SEED, int(i))), rough=(SEED, int(i)))
        for t in range(T):
            np.testing.assert_array_equal(tr["states"][t, i], e.obs(), err_msg=f"env {i} t {t}")
            _, r, d = e.step(tr["actions"][t, i])
            assert r == tr["rewards"][t, i] and d == tr["dones"][t, i], (i, t)
            ndone += d
        np.testing.assert_array_equal(state[i], e.dump(), err_msg=f"env {i}")
    assert ndone > 0
    eng.close()
