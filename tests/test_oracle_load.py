"""CPU: orc_env_load, the inverse of orc_env_dump (test infrastructure for the GPU tests that
start the oracle from a state given to the context, e.g. tests/test_gpu_nonfinite.py).  A
loaded copy must continue exactly like the original, before and after an auto-reset (the
body order after Walker.Reset, Walker.cs:212-234, is rebuilt from the post-reset flag)."""
import numpy as np


def test_load_continues_like_the_original(orc):
    rng = np.random.default_rng(11)
    a = orc.Env(dx=37.0, material=2)
    acts = rng.uniform(-1.2, 1.2, (600, 4)).astype(np.float32)
    for t in range(40):
        a.step(acts[t])
    b = orc.Env(dx=37.0, material=2)
    b.load(a.dump())
    np.testing.assert_array_equal(b.dump(), a.dump())
    np.testing.assert_array_equal(b.obs(), a.obs())
    resets = 0
    for t in range(40, 600):
        oa, ra, da = a.step(acts[t])
        ob, rb, db = b.step(acts[t])
        np.testing.assert_array_equal(oa, ob)
        assert ra == rb and da == db
        resets += da
    assert resets > 0
    np.testing.assert_array_equal(b.dump(), a.dump())
