"""GPU: weights files and checkpoint / resume through a live context.

* save_weights writes exactly format_weights(get_weights()) (PPOAgent.Save PPOAgent.cs:192-213);
  load_weights reproduces the weights bit-for-bit, including the matrix-core operand image
  the rollout reads (trajectories and the following PPO update agree bit-exactly with a
  context given the same weights through wk_set_weights);
* checkpoint_save -> checkpoint_load into a fresh context of the same seed resumes
  bit-exactly: the next rollout and PPO update equal the uninterrupted run's.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905


def _assert_bits(x, y):
    np.testing.assert_array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))


def test_weights_files_round_trip(wk, tmp_path):
    n, T = 256, 8
    kw = dict(Horizon=T, Minibatch=256, Epochs=1, RandomizeStart=1)
    a = wk.Engine(n, seed=SEED, **kw)
    b = wk.Engine(n, seed=SEED, **kw)
    rng = np.random.default_rng(7)
    w = (a.get_weights() * (1 + 0.1 * rng.standard_normal(wk.NPARAM))).astype(np.float32)
    a.set_weights(w)
    cp, ap = tmp_path / "critic.weights", tmp_path / "actor.weights"
    a.save_weights(cp, ap)
    ct, at = wk.format_weights(w)
    assert cp.read_text(encoding="utf-8") == ct and ap.read_text(encoding="utf-8") == at
    b.load_weights(cp, ap)
    _assert_bits(b.get_weights(), w)
    obs = rng.standard_normal((64, 12)).astype(np.float32)
    ids = np.arange(64, dtype=np.int32)
    steps = np.zeros(64, np.uint32)
    for x, y in zip(a.policy_sample(obs, ids, steps), b.policy_sample(obs, ids, steps)):
        _assert_bits(x, y)
    a.rollout(T)
    b.rollout(T)
    ta, tb = a.get_trajectory(T), b.get_trajectory(T)
    for k in ta:
        np.testing.assert_array_equal(ta[k], tb[k], err_msg=k)
    a.ppo_update(update_index=0)
    b.ppo_update(update_index=0)
    _assert_bits(a.get_weights(), b.get_weights())
    a.close()
    b.close()


def test_weights_load_errors_leave_weights(wk, tmp_path):
    a = wk.Engine(64, seed=SEED)
    w0 = a.get_weights()
    cp, ap = tmp_path / "c.weights", tmp_path / "a.weights"
    a.save_weights(cp, ap)
    cp.write_text(cp.read_text(encoding="utf-8").replace("|64|", "|32|", 1), encoding="utf-8")
    with pytest.raises(wk.WkError, match="does not match"):
        a.load_weights(cp, ap)
    with pytest.raises(wk.WkError, match="cannot read"):
        a.load_weights(tmp_path / "missing.weights", ap)
    _assert_bits(a.get_weights(), w0)
    a.close()


@pytest.mark.parametrize("lanes", [1, 2, 16])
def test_checkpoint_resume_bitexact(wk, tmp_path, lanes):
    n, T = 512, 16
    kw = dict(Horizon=T, Minibatch=512, Epochs=2, RandomizeStart=1, RandomizeMaterial=1,
              LanesPerWalker=lanes)
    a = wk.Engine(n, seed=SEED, **kw)
    a.rollout(T)
    a.ppo_update(update_index=0)
    ck = tmp_path / "run.ckpt"
    a.checkpoint_save(ck)  # walkers mid-episode, Philox counters and Adam state advanced
    a.rollout(T)
    ref_tr = a.get_trajectory(T)
    a.ppo_update(update_index=1)

    b = wk.Engine(n, seed=SEED, **kw)
    b.rollout(T)  # diverge first: load must overwrite everything that matters
    b.checkpoint_load(ck)
    with pytest.raises(wk.WkError):
        b.ppo_update(update_index=1)  # the trajectory buffer is not part of the checkpoint
    b.rollout(T)
    tr = b.get_trajectory(T)
    for k in ref_tr:
        np.testing.assert_array_equal(tr[k], ref_tr[k], err_msg=k)
    b.ppo_update(update_index=1)
    _assert_bits(b.get_state(), a.get_state())
    _assert_bits(b.get_weights(), a.get_weights())
    (ma, va, ta), (mb, vb, tb) = a.get_adam(), b.get_adam()
    _assert_bits(ma, mb)
    _assert_bits(va, vb)
    assert ta == tb
    a.close()
    b.close()


def test_checkpoint_mismatch_rejected(wk, tmp_path):
    a = wk.Engine(128, seed=SEED)
    ck = tmp_path / "x.ckpt"
    a.checkpoint_save(ck)
    with wk.Engine(256, seed=SEED) as e, pytest.raises(wk.WkError, match="walkers"):
        e.checkpoint_load(ck)
    with wk.Engine(128, seed=SEED + 1) as e, pytest.raises(wk.WkError, match="seed"):
        e.checkpoint_load(ck)
    (tmp_path / "junk.ckpt").write_bytes(b"not a checkpoint at all, really" * 4)
    with pytest.raises(wk.WkError, match="not a wk checkpoint"):
        a.checkpoint_load(tmp_path / "junk.ckpt")
    a.close()


def test_checkpoint_version2_still_loads(wk, tmp_path):
    """a version-2 file (no scene section: the layout before scene props) loads into a
    context and clears its scene"""
    import struct
    a = wk.Engine(64, seed=SEED, RandomizeStart=1)
    a.step(np.random.default_rng(1).uniform(-1, 1, (3, 64, 4)).astype(np.float32), k=3)
    ck = tmp_path / "v3.ckpt"
    a.checkpoint_save(ck)
    raw = bytearray(ck.read_bytes())
    assert struct.unpack_from("<I", raw, 4)[0] == 3 and raw[-4:] == b"\0\0\0\0"
    struct.pack_into("<I", raw, 4, 2)
    (tmp_path / "v2.ckpt").write_bytes(bytes(raw[:-4]))
    b = wk.Engine(64, seed=SEED)
    b.set_scene([wk.make_prop()])
    b.checkpoint_load(tmp_path / "v2.ckpt")
    np.testing.assert_array_equal(a.get_state(), b.get_state())
    with pytest.raises(wk.WkError):
        b.prop_view(0, 0)
    a.close()
    b.close()
