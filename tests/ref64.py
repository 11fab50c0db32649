"""Float64 restatement of PPOAgent.Train(Batch)'s gradient (PPOAgent.cs:218-346,
NeuralNetwork.FeedForward / FeedBack, DenseLayer.cs:82-120, ActivationLayer.cs:18-21),
vectorised over samples with numpy -- test infrastructure only.

The oracle (oracle/orc_ppo.c) sums samples sequentially in fp32, as the reference does; the
GPU sums them in 16-sample matrix-core blocks and a fixed tree.  Neither is "the" answer at
B = 65,536: both carry fp32 rounding of their own.  This float64 version gives the exact
value up to ~1e-16 and, per parameter, the sum of |per-sample contributions| -- the
condition of that sum -- so a test can bound each fp32 result by c * eps32 * sum|t| and ask
that the GPU be no less accurate than the reference's own sequential order.

Parameter layout: critic W1 (64x12) b1 W2 (1x64) b2, then actor W1 b1 W2 (64x64) b2 W3
(4x64) b3 (wk_common.h OFF_*).
"""
import numpy as np

OFF_C_W1, OFF_C_B1, OFF_C_W2, OFF_C_B2 = 0, 768, 832, 896
OFF_A_W1 = 897
OFF_A_B1 = OFF_A_W1 + 768
OFF_A_W2 = OFF_A_W1 + 832
OFF_A_B2 = OFF_A_W2 + 4096
OFF_A_W3 = OFF_A_B2 + 64
OFF_A_B3 = OFF_A_W3 + 256
NPARAM = OFF_A_B3 + 4


def _lrelu(z):
    return np.where(z < 0, 0.2 * z, z)


def _dlrelu(z):
    return np.where(z < 0, 0.2, 1.0)


def train_batch_grad64(w, S, A, L, G, Ad, b_div, log_std=-1.0, eps_clip=0.3):
    """Returns (grad, abs_sum, critic_diag, actor_diag, skipped) in float64; abs_sum[p] is
    sum over samples of |contribution to grad[p]|."""
    w = np.asarray(w, np.float64)
    S, A, L = (np.asarray(x, np.float64) for x in (S, A, L))
    G, Ad = np.asarray(G, np.float64), np.asarray(Ad, np.float64)
    std = float(np.float32(np.exp(np.float32(log_std))))  # MathF.Exp(-1) in fp32
    lp_const = float(-np.log(np.float32(std)) - np.log(np.sqrt(2 * np.pi)))
    cW1 = w[OFF_C_W1:OFF_C_B1].reshape(64, 12)
    cb1 = w[OFF_C_B1:OFF_C_W2]
    cW2 = w[OFF_C_W2:OFF_C_B2]
    cb2 = w[OFF_C_B2]
    aW1 = w[OFF_A_W1:OFF_A_B1].reshape(64, 12)
    ab1 = w[OFF_A_B1:OFF_A_W2]
    aW2 = w[OFF_A_W2:OFF_A_B2].reshape(64, 64)
    ab2 = w[OFF_A_B2:OFF_A_W3]
    aW3 = w[OFF_A_W3:OFF_A_B3].reshape(4, 64)
    ab3 = w[OFF_A_B3:NPARAM]
    # forward (cache=true)
    zc1 = S @ cW1.T + cb1
    hc1 = _lrelu(zc1)
    V = hc1 @ cW2 + cb2
    z1 = S @ aW1.T + ab1
    h1 = _lrelu(z1)
    z2 = h1 @ aW2.T + ab2
    h2 = _lrelu(z2)
    z3 = h2 @ aW3.T + ab3
    mean = np.tanh(z3)
    # PPO derivative per action dimension (PPOAgent.cs:234-326)
    up, lo = 1.0 + eps_clip, 1.0 - eps_clip
    lp = lp_const - ((A - mean) / std) ** 2 / 2.0
    r = np.exp(lp - L)
    cr = np.clip(r, lo, up)
    Acol = Ad[:, None]
    partA = (r * Acol <= cr * Acol) * Acol
    partB = (cr * Acol < r * Acol) * Acol
    partC = (r >= lo) & (r <= up)
    l = -(partA + partB * partC)
    eo = np.exp(L)
    use = ~(np.float32(0) == np.exp(np.asarray(L, np.float32))).any(axis=1)  # fp32 underflow
    actor = np.exp(lp) * ((A - mean) / std ** 2) * (l / np.where(eo == 0, 1.0, eo)) / b_div
    critic = 2.0 * (V - G) / b_div
    actor[~use] = 0.0
    critic[~use] = 0.0
    # backward (FeedBack)
    gz3 = actor * (1.0 - mean * mean)
    gz2 = (gz3 @ aW3) * _dlrelu(z2)
    gz1 = (gz2 @ aW2) * _dlrelu(z1)
    gzc1 = critic[:, None] * cW2[None, :] * _dlrelu(zc1)
    g = np.zeros(NPARAM)
    a = np.zeros(NPARAM)

    def put(off, val, aval):
        val = np.ravel(val)
        g[off:off + val.size] = val
        a[off:off + val.size] = np.ravel(aval)

    put(OFF_C_W1, gzc1.T @ S, np.abs(gzc1).T @ np.abs(S))
    put(OFF_C_B1, gzc1.sum(0), np.abs(gzc1).sum(0))
    put(OFF_C_W2, critic @ hc1, np.abs(critic) @ np.abs(hc1))
    put(OFF_C_B2, critic.sum(), np.abs(critic).sum())
    put(OFF_A_W1, gz1.T @ S, np.abs(gz1).T @ np.abs(S))
    put(OFF_A_B1, gz1.sum(0), np.abs(gz1).sum(0))
    put(OFF_A_W2, gz2.T @ h1, np.abs(gz2).T @ np.abs(h1))
    put(OFF_A_B2, gz2.sum(0), np.abs(gz2).sum(0))
    put(OFF_A_W3, gz3.T @ h2, np.abs(gz3).T @ np.abs(h2))
    put(OFF_A_B3, gz3.sum(0), np.abs(gz3).sum(0))
    return g, a, critic.sum(), actor.mean(axis=1).sum(), int((~use).sum())
