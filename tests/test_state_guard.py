"""CPU: the rigid-pole guard of wk_set_state / wk_checkpoint_load, through the
host-only export wk_check_state (no device).  The kernels project a walker pole onto its own edge
axes with min / max over fixed vertex groups (pole_own_minmax, csrc/wk_device.h) -- exact for
Pole.FromSize's shape (Objects/RigidBodies/Pole.cs:18-34) moved and rotated rigidly, where every
left-out vertex lies >= 7.5 px beyond the group; SATCollision.ProjectPoints (:63-76) takes the
min / max over all six.  States from the oracle's template and after many steps pass; a deformed
or reordered pole is refused with its walker and body; a non-finite pole is not checked (the NaN
path is exact, tests/test_gpu_nonfinite.py)."""
import numpy as np
import pytest

SEED = 20250905
LLL, LLU, BODY, RLL, RLU, BSTRIDE = 0, 1, 2, 3, 4, 20


def _states(orc, n=4, steps=0):
    out = []
    for i in range(n):
        e = orc.Env(dx=float(orc.env_offset(SEED, i)))
        for t in range(steps):
            e.step(orc.synth_action(SEED, i, t))
        out.append(e.dump())
    return np.stack(out).astype(np.float32)


def test_template_and_stepped_states_pass(wk, orc):
    wk.load_library()
    ok, e, b = wk.check_state(_states(orc))
    assert ok and e == -1 and b == -1
    ok, _, _ = wk.check_state(_states(orc, n=3, steps=300))  # after falls and resets
    assert ok


@pytest.mark.parametrize("body", [LLL, LLU, RLL, RLU])
def test_deformed_pole_is_refused(wk, orc, body):
    st = _states(orc)
    # move vertex 1 (the middle of an end edge) 10 px along x, past the side edge 2-3: on edge
    # 2's own axis the group {2, 3} no longer holds the minimum, vertex 1 does
    st[2, body * BSTRIDE + 2] -= 10.0  # x of vertex 1
    ok, e, b = wk.check_state(st)
    assert not ok and e == 2 and b == body


def test_reordered_pole_is_refused(wk, orc):
    st = _states(orc)
    v = st[1, RLU * BSTRIDE: RLU * BSTRIDE + 12].reshape(6, 2).copy()
    st[1, RLU * BSTRIDE: RLU * BSTRIDE + 12] = v[[1, 2, 3, 4, 5, 0]].ravel()  # rotated order
    ok, e, b = wk.check_state(st)
    assert not ok and (e, b) == (1, RLU)


def test_small_rigid_drift_passes_and_nonfinite_is_not_checked(wk, orc):
    st = _states(orc)
    st[0, LLU * BSTRIDE + 4] += 2.0  # vertex 2 x, 2 px: 5.5 px margin left (>= 3.5)
    ok, _, _ = wk.check_state(st)
    assert ok
    st[3, LLL * BSTRIDE + 0] = np.nan
    ok, _, _ = wk.check_state(st)
    assert ok
    st[3, RLL * BSTRIDE + 1] = np.inf
    assert wk.check_state(st)[0]
