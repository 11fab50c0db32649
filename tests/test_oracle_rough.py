"""Oracle restatement of CreateRoughFloor (Environment.cs:230-261), CPU only: geometry of
the 10 segments, the Random.Next(0, 100) draw range, list order, and the degenerate first
segment (three vertices on x = -50, a zero edge when draws 0 and 1 coincide)."""
import numpy as np

SEED = 20250905


def test_terrain_draws_range_and_determinism(orc):
    d = np.array([orc.terrain_draws(SEED, e) for e in range(2000)])
    assert d.shape == (2000, 11) and d.min() == 0 and d.max() == 99
    assert np.array_equal(d[17], orc.terrain_draws(SEED, 17))
    assert abs(d.mean() - 49.5) < 1.0  # uniform over 0..99


def test_segment_geometry(orc):
    draws = orc.terrain_draws(SEED, 3)
    e = orc.Env(rough=(SEED, 3))
    segs = e.floor_bodies()
    assert len(segs) == 10
    prev = (-50.0, 800.0 + draws[0])
    for i, s in enumerate(segs):
        x, y = -50 + 120 * i, 800 + draws[i + 1]
        np.testing.assert_array_equal(s, [[x, 1050], prev, [x, y], [x + 120, 1050]])
        prev = (x, y)


def test_degenerate_first_segment_steps(orc):
    env = next(e for e in range(5000) if orc.terrain_draws(SEED, e)[0] == orc.terrain_draws(SEED, e)[1])
    e = orc.Env(dx=-150.0, rough=(SEED, env))  # start over segment 0
    rng = np.random.default_rng(0)
    for _ in range(100):
        o, r, d = e.step(rng.uniform(-1, 1, 4).astype(np.float32))
        assert np.isfinite(o).all() and np.isfinite(r)
    assert np.isfinite(e.dump()).all()


def test_rough_floor_changes_the_dynamics(orc):
    a, b = orc.Env(dx=20.0), orc.Env(dx=20.0, rough=(SEED, 0))
    act = np.float32([0.3, -0.2, 0.1, 0.4])
    ra = [a.step(act)[1] for _ in range(5)]
    rb = [b.step(act)[1] for _ in range(5)]
    assert ra != rb
