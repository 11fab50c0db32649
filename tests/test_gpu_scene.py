"""GPU: scene props (Square / Triangle / Hexagon + SmoothCorners) against
the oracle, bit-exact.

Every walker carries its own copy of the props, listed after the floor (the line a
maintainer adds after CreateFloor() in the Environment constructor, Environment.cs:39-51),
and walker resets keep them (Walker.Reset only re-appends the walker's five bodies,
Walker.cs:212-234).  The props meet the walker's parts, the floor and each other through the
reference's ResolveCollisions (RigidBody.cs:66-113).  Bars as for the walker itself: every
walker body, every prop vertex / velocity, rewards and dones bit-exact -- on the flat floor and
on the rough floor's segments."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905
F = np.float32


def scene_a(m):
    # a static Titanium hexagon among the walkers' feet, a Wood box dropped on the torsos,
    # a spinning smoothed Rubber triangle and a Paper square resting near the start
    return [m(shape="Hexagon", material="Titanium", is_static=True, cx=200, cy=890, size=30),
            m(shape="Square", smooth=1, material="Wood", cx=150, cy=700, size=30, ay=980),
            m(shape="Triangle", smooth=1, material="Rubber", cx=260, cy=820, size=40, w=2.0,
              vx=-30.0, ay=980),
            m(shape="Square", material="Paper", cx=320, cy=870, size=24, ay=980)]


def scene_b(m):  # 24 + 4 + 3 = 31 vertices: the hexagon smoothed twice
    return [m(shape="Hexagon", smooth=2, material="SuperRubber", cx=180, cy=760, size=50,
              ay=980, vx=20.0),
            m(shape="Square", material="Metal", is_static=True, cx=260, cy=880, size=20,
              vx=-5.0),  # a static body still moves by its velocity (kinematic)
            m(shape="Triangle", material="Ice", cx=230, cy=700, size=20, ay=980)]


def oracle_envs(orc, n, props, offset=0, rough=False):
    return [orc.Env(dx=float(orc.env_offset(SEED, offset + e)),
                    material=int(orc.env_material(SEED, offset + e)), props=props,
                    rough=(SEED, offset + e) if rough else None)
            for e in range(n)]


def check_props(eng, envs, n_props):
    for i, e in enumerate(envs):
        for k in range(n_props):
            verts, st = e.prop(k)
            v = eng.prop_view(i, k)
            np.testing.assert_array_equal(v.vertex_array(), verts, err_msg=f"env {i} prop {k}")
            got = np.array([v.centroid[0], v.centroid[1], v.linear_velocity[0],
                            v.linear_velocity[1], v.angular_velocity, v.angle], F)
            np.testing.assert_array_equal(got, st, err_msg=f"env {i} prop {k} state")


@pytest.mark.parametrize("scene", [scene_a, scene_b])
def test_scene_multi_step_bitexact(wk, orc, scene):
    n, k = 192, 160
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    eng.set_scene(scene(wk.make_prop))
    envs = oracle_envs(orc, n, scene(orc.make_prop))
    check_props(eng, envs, len(scene(orc.make_prop)))
    acts = np.random.default_rng(11).uniform(-1.2, 1.2, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    ndone = 0
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
            np.testing.assert_array_equal(o, obs[t, i])
            ndone += d
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    check_props(eng, envs, len(scene(orc.make_prop)))
    assert ndone > 0 and not fault.any()  # resets happened: post-reset list order exercised


def test_scene_changes_walkers(wk, orc):
    """the props really interact: the same actions give other walker states without them"""
    n, k = 64, 80
    acts = np.random.default_rng(5).uniform(-1, 1, (k, n, 4)).astype(F)
    a = wk.Engine(n, seed=SEED, RandomizeStart=1)
    a.set_scene(scene_a(wk.make_prop))
    b = wk.Engine(n, seed=SEED, RandomizeStart=1, LanesPerWalker=1)
    a.step(acts, k=k)
    b.step(acts, k=k)
    differ = (a.get_state() != b.get_state()).any(1).sum()
    assert differ > 4


def test_scene_trace_bitexact(wk, orc):
    """per-substep pair trace of the walker's own 9 pairs with props present"""
    n = 64
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    eng.set_scene(scene_a(wk.make_prop))
    envs = oracle_envs(orc, n, scene_a(orc.make_prop))
    acts = np.random.default_rng(2).uniform(-1, 1, (n, 4)).astype(F)
    tr = eng.step_traced(acts)
    for i, e in enumerate(envs):
        _, _, _, t = e.step(acts[i], trace=True)
        for key in ("aabb_hit", "sat_hit", "n_contacts", "normal", "depth", "contact", "impulse",
                    "joint_depth", "joint_impulse"):
            np.testing.assert_array_equal(tr[i][key], t[key], err_msg=f"env {i} {key}")
    check_props(eng, envs, 4)


def test_scene_rollout_replays_exactly(wk, orc):
    n, T = 128, 64
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, Horizon=T)
    eng.set_scene(scene_a(wk.make_prop))
    envs = oracle_envs(orc, n, scene_a(orc.make_prop))
    for _ in range(2):  # two rollouts: props persist across launches
        eng.rollout(T)
        tr = eng.get_trajectory(T)
        for i, e in enumerate(envs):
            for t in range(T):
                np.testing.assert_array_equal(tr["states"][t, i], e.obs(), err_msg=f"env {i} t {t}")
                _, r, d = e.step(tr["actions"][t, i])
                assert r == tr["rewards"][t, i] and d == tr["dones"][t, i], (i, t)
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    check_props(eng, envs, 4)
    eng.ppo_update()
    assert np.isfinite(eng.get_weights()).all()


def test_scene_checkpoint_resume(wk, tmp_path):
    n, T = 96, 32
    mk = lambda: wk.Engine(n, seed=SEED, RandomizeStart=1, Horizon=T, Minibatch=n)
    a = mk()
    a.set_scene(scene_b(wk.make_prop))
    a.rollout(T)
    a.ppo_update(update_index=0)
    path = str(tmp_path / "scene.ckpt")
    a.checkpoint_save(path)
    b = mk()  # no scene yet: loading brings the checkpoint's
    b.checkpoint_load(path)
    for eng in (a, b):
        eng.rollout(T)
        eng.ppo_update(update_index=1)
    np.testing.assert_array_equal(a.get_state(), b.get_state())
    np.testing.assert_array_equal(a.get_weights(), b.get_weights())
    for k in range(3):
        np.testing.assert_array_equal(a.prop_view(7, k).vertex_array(), b.prop_view(7, k).vertex_array())
    # removing the scene returns to the fast mappings
    b.set_scene([])
    with pytest.raises(wk.WkError):
        b.prop_view(0, 0)


def test_scene_validation(wk):
    eng = wk.Engine(8, seed=SEED)
    m = wk.make_prop
    with pytest.raises(wk.WkError):
        eng.set_scene([m(shape="Hexagon", smooth=3)])           # 48 vertices
    with pytest.raises(wk.WkError):
        eng.set_scene([m(shape="Hexagon", smooth=2), m(shape="Square", smooth=2)])  # 24 + 16 > 32
    with pytest.raises(wk.WkError):
        eng.set_scene([m()] * 5)                                 # > 4 props
    with pytest.raises(wk.WkError):
        eng.set_scene([m(size=0.0)])
    with pytest.raises(wk.WkError):
        eng.set_scene([m(material=9)])
    side = wk.Engine(8, seed=SEED, LanesPerWalker=2)
    with pytest.raises(wk.WkError):
        side.set_scene([m()])


def test_scene_at_bench_scale(wk, orc):
    """65,536 walkers with the four props (the scene kernel at the bench's per-GPU size):
    a strided sample of walkers replays bit-exactly through the oracle"""
    n, k = 65536, 6
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    eng.set_scene(scene_a(wk.make_prop))
    acts = np.random.default_rng(21).uniform(-1.2, 1.2, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    sample = list(range(0, n, 1021))
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e)), material=int(orc.env_material(SEED, e)),
                    props=scene_a(orc.make_prop)) for e in sample]
    st = eng.get_state()
    for i, e in zip(sample, envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
        np.testing.assert_array_equal(st[i], e.dump(), err_msg=f"walker {i}")
        for p in range(4):
            np.testing.assert_array_equal(eng.prop_view(i, p).vertex_array(), e.prop(p)[0])
    assert not fault.any()


@pytest.mark.parametrize("scene", [scene_a, scene_b])
def test_scene_on_rough_floor_bitexact(wk, orc, scene):
    """scene props on CreateRoughFloor's terrain (the combination the reference's
    list-based environment admits, Environment.cs:39-51,230-261): list [walker, 10 segments,
    props], after a reset [segments, props, walker]; every prop resolves against every
    segment.  Bodies, props, rewards and dones bit-exact over env-steps with resets, then a
    policy rollout replayed through the oracle"""
    n, k, T = 128, 120, 32
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1, RoughFloor=1, Horizon=T)
    eng.set_scene(scene(wk.make_prop))
    envs = oracle_envs(orc, n, scene(orc.make_prop), rough=True)
    n_props = len(scene(orc.make_prop))
    check_props(eng, envs, n_props)
    acts = np.random.default_rng(13).uniform(-1.2, 1.2, (k, n, 4)).astype(F)
    obs, rew, done, fault = eng.step(acts, k=k)
    ndone = 0
    for i, e in enumerate(envs):
        for t in range(k):
            o, r, d = e.step(acts[t, i])
            assert r == rew[t, i] and d == done[t, i], (i, t)
            np.testing.assert_array_equal(o, obs[t, i])
            ndone += d
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    check_props(eng, envs, n_props)
    assert ndone > 0 and not fault.any()
    eng.rollout(T)
    tr = eng.get_trajectory(T)
    for i, e in enumerate(envs):
        for t in range(T):
            np.testing.assert_array_equal(tr["states"][t, i], e.obs(), err_msg=f"env {i} t {t}")
            _, r, d = e.step(tr["actions"][t, i])
            assert r == tr["rewards"][t, i] and d == tr["dones"][t, i], (i, t)
    np.testing.assert_array_equal(eng.get_state(), np.stack([e.dump() for e in envs]))
    check_props(eng, envs, n_props)


def test_scene_on_rough_floor_trace(wk, orc):
    """the walker's traced pairs (joints, leg-leg; segment pairs are not traced) with props on
    the rough floor"""
    n = 64
    eng = wk.Engine(n, seed=SEED, RandomizeStart=1, RoughFloor=1)
    eng.set_scene(scene_b(wk.make_prop))
    envs = [orc.Env(dx=float(orc.env_offset(SEED, e)), props=scene_b(orc.make_prop),
                    rough=(SEED, e)) for e in range(n)]
    acts = np.random.default_rng(3).uniform(-1, 1, (n, 4)).astype(F)
    tr = eng.step_traced(acts)
    for i, e in enumerate(envs):
        _, _, _, t = e.step(acts[i], trace=True)
        for key in ("aabb_hit", "sat_hit", "n_contacts", "normal", "depth", "contact", "impulse",
                    "joint_depth", "joint_impulse"):
            np.testing.assert_array_equal(tr[i][key], t[key], err_msg=f"env {i} {key}")
    check_props(eng, envs, 3)
