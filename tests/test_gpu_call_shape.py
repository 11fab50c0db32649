"""GPU: the reference's per-body call shape through the C ABI.

A C# host that keeps Environment.StepObjects (Environment.cs:126-143) calls, per frame, for each of
Iterations substeps Joint.Step on the 4 joints (Joint.cs:31-41) and IObject.Update
(Objects/IObject.cs:9) on every body of its list, after Walker.TakeActions (Walker.cs:66-75).  This
test drives wk_take_actions / wk_joint_step / wk_object_update exactly so (the emulation of
cs/Api.cs's RigidBody.Update / Joint.Step / Walker.TakeActions, which are one-line P/Invoke calls)
and requires:
* one frame (4 + 6 calls x 50 substeps) advances exactly one env-step, bit-identical to wk_step
  with the same torques; the frame's first Update call is the one that steps;
* a frame without TakeActions keeps the walkers' torques (no kick), bit-identical to wk_step with
  the current torques; a walker given none while another is given some keeps its own;
* wk_body_order: [LLL, LLU, Body, RLL, RLU, Floor] in episode 0, the floor first after a reset;
* the rigid-pole guard: wk_set_state and wk_checkpoint_load refuse a deformed pole and leave the
  context unchanged."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905


def _frame(eng, bodies, iterations=50, dt=0.0166667):
    """Environment.StepObjects' call sequence (Environment.cs:128-141); returns which calls stepped"""
    stepped = []
    for _ in range(iterations):
        for _ in range(4):
            eng.joint_step()
        for _ in range(len(bodies)):
            stepped.append(eng.object_update(len(bodies), dt / iterations))
    return stepped


def test_reference_frame_is_one_step_bit_identical(wk):
    n = 24
    a = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    b = wk.Engine(n, seed=SEED, RandomizeStart=1, RandomizeMaterial=1)
    rng = np.random.default_rng(3)
    for frame in range(6):
        acts = (rng.uniform(-1.3, 1.3, (n, 4))).astype(np.float32)
        for e in range(n):
            a.take_actions(e, acts[e])
        bodies = a.body_order(0)
        st = _frame(a, bodies)
        assert st[0] and not any(st[1:]), frame  # the first Update call of the frame steps
        b.step(acts, k=1)
        np.testing.assert_array_equal(a.get_state(), b.get_state(), err_msg=f"frame {frame}")
    # a frame with no TakeActions: every walker keeps its torques (Joint.SetTorque with the same
    # value, Joint.cs:56-61: no kick) -- wk_step with the clipped current torques
    torques = b.get_state()[:, 100:104].copy()
    _frame(a, a.body_order(0))
    b.step(torques, k=1)
    np.testing.assert_array_equal(a.get_state(), b.get_state())
    # only walker 5 given new torques: the others keep theirs
    new = np.array([0.3, -0.7, 0.9, -0.1], np.float32)
    a.take_actions(5, new)
    torques = b.get_state()[:, 100:104].copy()
    torques[5] = new
    _frame(a, a.body_order(0))
    b.step(torques, k=1)
    np.testing.assert_array_equal(a.get_state(), b.get_state())
    a.close()
    b.close()


def test_body_order_episode0_then_post_reset(wk):
    eng = wk.Engine(4, seed=SEED)
    assert eng.body_order(2) == [0, 1, 2, 3, 4, 5]
    mask = np.zeros(4, np.uint8)
    mask[2] = 1
    eng.reset(mask)
    assert eng.body_order(2) == [5, 0, 1, 2, 3, 4]
    assert eng.body_order(1) == [0, 1, 2, 3, 4, 5]
    rough = wk.Engine(2, seed=SEED, RoughFloor=1)
    assert rough.body_order(0) == [0, 1, 2, 3, 4] + list(range(5, 15))
    rough.reset()
    assert rough.body_order(1) == list(range(5, 15)) + [0, 1, 2, 3, 4]
    eng.close()
    rough.close()


def test_deformed_pole_is_refused_by_set_state_and_checkpoint(wk, tmp_path):
    eng = wk.Engine(8, seed=SEED, RandomizeStart=1)
    eng.step(np.full((3, 8, 4), 0.4, np.float32), k=3)
    good = eng.get_state()
    path = str(tmp_path / "ck.bin")
    eng.checkpoint_save(path)
    bad = good.copy()
    bad[6, 3 * 20 + 2] -= 10.0  # RLL vertex 1 x, past the side edge: not a rigid pole
    with pytest.raises(wk.WkError, match="walker 6 body 3 is not a rigid walker pole"):
        eng.set_state(bad)
    np.testing.assert_array_equal(eng.get_state(), good)
    # the same records inside a checkpoint file
    data = bytearray(open(path, "rb").read())
    rec0 = data.find(good[0].tobytes())
    assert rec0 > 0
    off = rec0 + (6 * 112 + 3 * 20 + 2) * 4
    data[off:off + 4] = np.float32(good[6, 62] - 10.0).tobytes()
    bad_path = str(tmp_path / "bad.bin")
    open(bad_path, "wb").write(bytes(data))
    eng.step(np.zeros((8, 4), np.float32), k=1)
    before = eng.get_state()
    with pytest.raises(wk.WkError, match="not a rigid walker pole"):
        eng.checkpoint_load(bad_path)
    np.testing.assert_array_equal(eng.get_state(), before)
    eng.checkpoint_load(path)  # the intact file still loads
    np.testing.assert_array_equal(eng.get_state(), good)
    eng.close()
