"""CPU: the oracle's scene props (generic polygons).

Square / Triangle / Hexagon.FromSize (Objects/RigidBodies/*.cs) and Skeleton.SmoothCorners
(Skeleton.cs:33-53) hand-derived, the centroid kept from the FromSize vertices, and the
physics of props in the body list (RigidBody.cs:54-113): a box falling under gravity comes
to rest on the floor, a static prop never moves, walkers resets keep the props."""
import numpy as np
import pytest

F = np.float32


def test_prop_vertices_kat(orc):
    # Square.FromSize(m, (300, 700), 40): adjustment 20
    sq = orc.prop_vertices(orc.make_prop("Square", cx=300, cy=700, size=40))
    np.testing.assert_array_equal(sq, [[320, 720], [280, 720], [280, 680], [320, 680]])
    tri = orc.prop_vertices(orc.make_prop("Triangle", cx=300, cy=700, size=40))
    np.testing.assert_array_equal(tri, [[300, 720], [280, 680], [320, 680]])
    hexa = orc.prop_vertices(orc.make_prop("Hexagon", cx=300, cy=700, size=40))
    np.testing.assert_array_equal(hexa, [[310, 720], [290, 720], [280, 700], [290, 680],
                                         [310, 680], [320, 700]])
    # SmoothCorners once: per vertex j, v_j + 0.2 (v_{j-1} - v_j) then v_j + 0.2 (v_{j+1} - v_j)
    s1 = orc.prop_vertices(orc.make_prop("Square", smooth=1, cx=300, cy=700, size=40))
    np.testing.assert_array_equal(s1[:4], [[320, 712], [312, 720], [288, 720], [280, 712]])
    assert len(s1) == 8
    # twice: 16 vertices, each the fp32 expression of the rule
    s2 = orc.prop_vertices(orc.make_prop("Square", smooth=2, cx=300, cy=700, size=40))
    assert len(s2) == 16
    v0, vp, vn = s1[0], s1[7], s1[1]
    np.testing.assert_array_equal(s2[0], v0 + (vp - v0) * F(0.2))
    np.testing.assert_array_equal(s2[1], v0 + (vn - v0) * F(0.2))
    assert len(orc.prop_vertices(orc.make_prop("Hexagon", smooth=2))) == 24
    with pytest.raises(ValueError):
        orc.prop_vertices(orc.make_prop("Hexagon", smooth=3))  # 48 > 24


def test_smoothed_prop_keeps_fromsize_centroid(orc):
    # the centroid is FindCentroid of the 3 FromSize vertices (sum * (1/3)); SmoothCorners
    # never recomputes it
    p = orc.make_prop("Triangle", smooth=1, cx=400, cy=700, size=30, is_static=True)
    e = orc.Env(props=[p])
    verts, st = e.prop(0)
    base = orc.prop_vertices(orc.make_prop("Triangle", cx=400, cy=700, size=30))
    c = base.sum(0, dtype=F) * (F(1) / F(3))
    np.testing.assert_array_equal(st[:2], c)
    assert len(verts) == 6


def test_box_rests_on_floor_and_static_prop_stays(orc):
    box = orc.make_prop("Square", smooth=1, material="Wood", cx=600, cy=820, size=40, ay=980)
    post = orc.make_prop("Hexagon", material="Titanium", is_static=True, cx=700, cy=880, size=30)
    e = orc.Env(props=[box, post])
    v_post0, s_post0 = e.prop(1)
    for _ in range(150):
        e.step(np.zeros(4, F))
    verts, st = e.prop(0)
    assert 898.0 < verts[:, 1].max() < 901.0            # bottom face on the floor (y = 900)
    assert abs(st[3]) < 1.0 and abs(st[2]) < 1.0         # at rest
    v_post, s_post = e.prop(1)
    np.testing.assert_array_equal(v_post, v_post0)       # static: never moves
    np.testing.assert_array_equal(s_post, s_post0)


def test_walker_pushes_prop_and_resets_keep_props(orc):
    # a light Paper box dropped on the walker's torso: walker and box interact
    box = orc.make_prop("Square", material="Paper", cx=125, cy=740, size=30, ay=980)
    e, e0 = orc.Env(props=[box]), orc.Env()
    rng = np.random.default_rng(3)
    moved, resets = False, 0
    for t in range(300):
        a = rng.uniform(-1, 1, 4).astype(F)
        _, _, d = e.step(a)
        e0.step(a)
        resets += d
        if not np.array_equal(e.dump(), e0.dump()):
            moved = True
    assert moved            # the box changed the walker's trajectory
    assert resets > 0
    verts, st = e.prop(0)   # the box survives walker resets
    assert len(verts) == 4 and np.isfinite(st).all()


def test_rough_floor_and_props_compose_in_oracle(orc):
    e = orc.Env(rough=(20250905, 0), props=[orc.make_prop("Triangle", cx=500, cy=600, ay=980)])
    for _ in range(50):
        e.step(np.zeros(4, F))
    assert len(e.floor_bodies()) == 10 and np.isfinite(e.prop(0)[1]).all()
