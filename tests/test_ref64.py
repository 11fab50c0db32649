"""CPU: the float64 gradient restatement used by the GPU gradient tests (tests/ref64.py)
agrees with the oracle's fp32 Train(Batch) where the oracle's own rounding is small (B <= 2,048),
including the skipped-sample rule; and at B = 65,536 the oracle's sequential fp32 sum carries
visible rounding of its own (the reason tests/test_gpu_grad_scale.py bounds against float64)."""
import numpy as np
import pytest

import ref64

F = np.float32


def _batch(B, seed, skip_at=None):
    rng = np.random.default_rng(seed)
    S = rng.normal(0, 1, (B, 12)).astype(F)
    A = rng.normal(0, 1, (B, 4)).astype(F)
    L = rng.normal(-3, 1, (B, 4)).astype(F)
    G = rng.normal(0, 5, B).astype(F)
    Ad = rng.normal(0, 1, B).astype(F)
    if skip_at is not None:
        L[skip_at, 1] = -200.0
    return S, A, L, G, Ad


@pytest.mark.parametrize("B,skip_at", [(64, None), (257, 3), (2048, 2047)])
def test_ref64_matches_oracle_small(orc, B, skip_at):
    ag = orc.Agent(seed=20250905)
    S, A, L, G, Ad = _batch(B, B, skip_at)
    og, ocd, oad, osk = ag.train_batch(S, A, L, G, Ad, b_div=B, apply_adam=False)
    g, asum, cd, ad, sk = ref64.train_batch_grad64(ag.params(), S, A, L, G, Ad, B)
    assert sk == osk == (0 if skip_at is None else 1)
    assert (np.abs(og - g) <= 2e-6 * asum + 1e-9).all()
    assert ocd == pytest.approx(cd, rel=1e-5, abs=1e-7) and oad == pytest.approx(ad, rel=1e-5, abs=1e-7)


def test_oracle_sequential_sum_at_65536(orc):
    B = 65536
    ag = orc.Agent(seed=20250905)
    S, A, L, G, Ad = _batch(B, B)
    og, _, _, _ = ag.train_batch(S, A, L, G, Ad, b_div=B, apply_adam=False)
    g, asum, _, _, _ = ref64.train_batch_grad64(ag.params(), S, A, L, G, Ad, B)
    err = np.abs(og - g)
    assert err.max() > 2e-5 * np.abs(g).max()  # the sequential sum's own rounding is visible
    assert (err <= 1e-3 * asum + 1e-9).all()  # up to 1.5e-4 of sum|t| for same-sign terms
