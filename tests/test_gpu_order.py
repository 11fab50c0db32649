"""GPU: the lane order of the split physics kernels (wk_order.hip) changes no result.

Before every launch the lane-pair / quad mappings order their lanes so that walkers still in
their first episode come first (their floor pairs run in the other list order,
RigidBody.cs:66-96 / Walker.cs:212-234); on the rough floor the order is static, the walkers
sorted by start offset (wk_api.cpp rough_order_upload, recomputed when the offsets change).  The order only decides which walkers share a wave;
every walker's arithmetic, Philox stream and trajectory rows are its own, so a context with the
ordering and one with the identity order (WK_ORDER=0, read at wk_create) must produce the same
trajectories, walker records and PPO updates bit for bit -- here with short episodes
(MaxTimesteps 30) and 40 % of the walkers reset up front, so that launches start with a mix
of episode-0 and post-reset walkers."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905


def _engine(wk, n, ordered, **cfg):
    old = os.environ.get("WK_ORDER")
    os.environ["WK_ORDER"] = "1" if ordered else "0"
    try:
        return wk.Engine(n, seed=SEED, **cfg)
    finally:
        if old is None:
            os.environ.pop("WK_ORDER")
        else:
            os.environ["WK_ORDER"] = old


@pytest.mark.parametrize("n,lanes,rough", [(3000, 4, 0), (4096, 4, 0), (20011, 2, 0), (40000, 2, 0),
                                           (20011, 2, 1), (3000, 4, 1)])
def test_lane_order_is_invisible(wk, n, lanes, rough):
    """rough = 1: the rough-floor pair kernel fills its per-walker terrain column in
    LDS from the reordered walker id"""
    T = 16
    cfg = dict(Horizon=T, Minibatch=n * T // 4, Epochs=1, RandomizeStart=1, RandomizeMaterial=1,
               MaxTimesteps=30, LanesPerWalker=lanes, RoughFloor=rough)
    a, b = _engine(wk, n, True, **cfg), _engine(wk, n, False, **cfg)
    # Environment.Reset of a random 40 % (wk_reset: those walkers continue post-reset, the
    # floor first in their body list), so every launch starts with both kinds of walker
    mask = (np.random.default_rng(n).random(n) < 0.4).astype(np.uint8)
    for e in (a, b):
        e.reset(mask)
    mixed = False
    for it in range(4):
        post = a.get_state()[:, 109]
        mixed |= bool(0 < post.sum() < n)
        for e in (a, b):
            e.rollout(T)
        ta, tb = a.get_trajectory(T), b.get_trajectory(T)
        for k in ta:
            np.testing.assert_array_equal(ta[k], tb[k], err_msg=f"iteration {it}: {k}")
        np.testing.assert_array_equal(a.get_state(), b.get_state())
        for e in (a, b):
            e.ppo_update(update_index=it)
        np.testing.assert_array_equal(a.get_weights(), b.get_weights())
    assert mixed  # launches started with both kinds of walker
    a.close()
    b.close()


@pytest.mark.parametrize("lanes", [2, 4])
def test_rough_offset_order_follows_the_offsets(wk, tmp_path, lanes):
    """the rough floor's offset order is rebuilt when the offsets change: new offsets through
    wk_set_offsets (reversed: the old order would now be the worst one) and a checkpoint written
    by another context, loaded into both -- ordered and identity contexts stay bit-identical"""
    n, T = 5000, 16
    cfg = dict(Horizon=T, Minibatch=n * T // 4, Epochs=1, RandomizeStart=1, MaxTimesteps=30,
               LanesPerWalker=lanes, RoughFloor=1)
    a, b = _engine(wk, n, True, **cfg), _engine(wk, n, False, **cfg)
    dx = np.linspace(199.0, 0.0, n).astype(np.float32)
    for e in (a, b):
        e.set_offsets(dx)
        e.reset()
        e.rollout(T)
    ta, tb = a.get_trajectory(T), b.get_trajectory(T)
    for k in ta:
        np.testing.assert_array_equal(ta[k], tb[k], err_msg=k)
    other = wk.Engine(n, seed=SEED, **cfg)  # (a checkpoint must come from the same seed)
    other.set_offsets(np.random.default_rng(3).permutation(dx))
    other.reset()
    for _ in range(2):
        other.rollout(T)
    path = str(tmp_path / "other.ckpt")
    other.checkpoint_save(path)
    other.close()
    for e in (a, b):
        e.checkpoint_load(path)
        e.rollout(T)
    ta, tb = a.get_trajectory(T), b.get_trajectory(T)
    for k in ta:
        np.testing.assert_array_equal(ta[k], tb[k], err_msg=f"after load: {k}")
    np.testing.assert_array_equal(a.get_state(), b.get_state())
    a.close()
    b.close()



@pytest.mark.parametrize("n,lanes,rough", [(40000, 2, 0), (40000, 2, 1), (20011, 1, 0), (3000, 16, 0)])
def test_wave_pacing_is_invisible(wk, n, lanes, rough):
    """the pacing of co-resident waves (wk_physics.hip pace_partner: per-SIMD progress slots,
    s_setprio; the pair kernel and k_env_step) only decides which wave of a SIMD issues first: a
    context without it (WK_PACE=0, read at wk_create) gives the same trajectories, records and
    update"""
    T = 16
    cfg = dict(Horizon=T, Minibatch=n * T // 4, Epochs=1, RandomizeStart=1, RandomizeMaterial=1,
               MaxTimesteps=30, LanesPerWalker=lanes, RoughFloor=rough)
    old = os.environ.get("WK_PACE")
    try:
        os.environ["WK_PACE"] = "0"
        b = wk.Engine(n, seed=SEED, **cfg)
    finally:
        if old is None:
            os.environ.pop("WK_PACE")
        else:
            os.environ["WK_PACE"] = old
    a = wk.Engine(n, seed=SEED, **cfg)
    for it in range(3):
        for e in (a, b):
            e.rollout(T)
        ta, tb = a.get_trajectory(T), b.get_trajectory(T)
        for k in ta:
            np.testing.assert_array_equal(ta[k], tb[k], err_msg=f"iteration {it}: {k}")
        np.testing.assert_array_equal(a.get_state(), b.get_state())
        for e in (a, b):
            e.ppo_update(update_index=it)
        np.testing.assert_array_equal(a.get_weights(), b.get_weights())
    a.close()
    b.close()
