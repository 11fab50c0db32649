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


def _downgrade(raw, version):
    """a version-4 file rewritten in an older layout: v3 drops the 16-byte CkptExt after the
    48-byte header; v2 also drops the (empty) scene section's count"""
    import struct
    assert struct.unpack_from("<I", raw, 4)[0] == 4 and raw[-4:] == b"\0\0\0\0"
    out = bytearray(raw[:48] + raw[64:])
    struct.pack_into("<I", out, 4, version)
    return bytes(out if version == 3 else out[:-4])


@pytest.mark.parametrize("version", [2, 3])
def test_checkpoint_older_versions_refused(wk, tmp_path, version):
    """version-2 (no scene section) and version-3 files (no CkptExt) do not record RoughFloor,
    which existed when they were written, and the walker records cannot tell the floors apart:
    they are refused and the context -- walkers, weights and scene -- is unchanged"""
    a = wk.Engine(64, seed=SEED, RandomizeStart=1)
    a.step(np.random.default_rng(1).uniform(-1, 1, (3, 64, 4)).astype(np.float32), k=3)
    ck = tmp_path / "v4.ckpt"
    a.checkpoint_save(ck)
    old = tmp_path / f"v{version}.ckpt"
    old.write_bytes(_downgrade(ck.read_bytes(), version))
    b = wk.Engine(64, seed=SEED)
    b.set_scene([wk.make_prop()])
    s0, w0 = b.get_state(), b.get_weights()
    with pytest.raises(wk.WkError, match="floor type"):
        b.checkpoint_load(old)
    np.testing.assert_array_equal(b.get_state(), s0)
    np.testing.assert_array_equal(b.get_weights(), w0)
    b.prop_view(0, 0)  # the scene is still there
    a.close()
    b.close()


def test_rejected_checkpoint_leaves_context_unchanged(wk, tmp_path):
    """every precondition is checked before the first device write: a file from
    a different Iterations / MaxTimesteps / RoughFloor, or with scene props for a context that
    cannot run them, is refused and the context's weights, Adam state, walkers and scene stay
    as they were"""
    rng = np.random.default_rng(3)
    acts = rng.uniform(-1, 1, (2, 32, 4)).astype(np.float32)
    cases = [(dict(Iterations=40), {}, "Iterations"),
             (dict(MaxTimesteps=500), {}, "MaxTimesteps"),
             (dict(RoughFloor=1), {}, "RoughFloor"),
             ({}, dict(LanesPerWalker=2), "scene props")]
    for i, (src_cfg, dst_cfg, what) in enumerate(cases):
        src = wk.Engine(32, seed=SEED, **src_cfg)
        if what == "scene props":
            src.set_scene([wk.make_prop(cx=300.0, cy=700.0)])
        src.step(acts, k=2)
        ck = tmp_path / f"c{i}.ckpt"
        src.checkpoint_save(ck)
        dst = wk.Engine(32, seed=SEED + 0, RandomizeStart=1, **dst_cfg)
        dst.step(acts[::-1].copy(), k=2)
        dst.set_weights(dst.get_weights() * np.float32(0.5))
        before = (dst.get_state(), dst.get_weights(), dst.get_adam())
        with pytest.raises(wk.WkError, match=what):
            dst.checkpoint_load(ck)
        after = (dst.get_state(), dst.get_weights(), dst.get_adam())
        np.testing.assert_array_equal(before[0], after[0])
        np.testing.assert_array_equal(before[1], after[1])
        for x, y in zip(before[2], after[2]):
            np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
        src.close()
        dst.close()


def test_contexts_on_two_devices(wk):
    """every entry point binds the context's device, so two contexts on devices
    0 and 1 used alternately from one thread keep their buffers and kernels apart, and the
    caller's current device is left unchanged"""
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    rng = np.random.default_rng(5)
    acts = rng.uniform(-1, 1, (4, 256, 4)).astype(np.float32)
    torch.cuda.set_device(0)
    a = wk.Engine(256, seed=SEED, device=0, RandomizeStart=1)
    b = wk.Engine(256, seed=SEED, device=1, RandomizeStart=1)
    ref = wk.Engine(256, seed=SEED, device=0, RandomizeStart=1)
    for t in range(4):
        a.step(acts[t:t + 1], k=1)
        b.step(acts[t:t + 1], k=1)
        ref.step(acts[t:t + 1], k=1)
        assert torch.cuda.current_device() == 0
    np.testing.assert_array_equal(a.get_state(), ref.get_state())
    np.testing.assert_array_equal(b.get_state(), ref.get_state())
    for e in (a, b, ref):
        e.close()
