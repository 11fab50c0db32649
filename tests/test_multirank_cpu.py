"""Multi-rank (world_size 2, gloo, CPU) checks of the sharded PPO math that
wk_ppo_update performs with RCCL on GPUs: each rank accumulates its shard of the global
minibatch with the per-sample divisor = global minibatch size; the all-reduced (summed)
gradient equals the single-rank gradient of the whole minibatch (fp32 reassociation
tolerance), and the replicated Adam then lands on the same weights on every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20250905


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def batch(orc, B):
    rng = np.random.default_rng(21)
    ag = orc.Agent(seed=SEED)
    s = rng.normal(0, 0.7, (B, 12)).astype(np.float32)
    a = np.zeros((B, 4), np.float32)
    lp = np.zeros((B, 4), np.float32)
    for i in range(B):
        a[i], lp[i] = ag.sample(s[i], SEED, i, 0)
        lp[i] += rng.normal(0, 0.2, 4).astype(np.float32)
    return s, a, lp, rng.normal(0, 1, B).astype(np.float32), rng.normal(0, 1, B).astype(np.float32)


def _worker(rank, world, port, B, q):
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ppo-bipedalwalker_amd")]
    import torch
    import torch.distributed as dist
    import orc
    from wk.dist import make_shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = make_shard(rank, world, rank, walkers_per_rank=B // world)
    s, a, lp, G, A = batch(orc, B)
    lo, hi = sh.env_offset, sh.env_offset + sh.n_local
    ag = orc.Agent(seed=SEED)
    g, cd, ad, _ = ag.train_batch(s[lo:hi], a[lo:hi], lp[lo:hi], G[lo:hi], A[lo:hi],
                                  b_div=sh.minibatch_global, apply_adam=False)
    t = torch.from_numpy(np.concatenate([g, [cd, ad]]).astype(np.float32))
    dist.all_reduce(t)
    gsum = t.numpy()[:-2]
    # replicated Adam from identical weights: feed the reduced gradient through one Adam step
    # (a one-sample batch with zero loss would not do; use the oracle's Adam directly)
    w0 = ag.params()
    m = np.zeros_like(w0)
    v = np.zeros_like(w0)
    f = np.float32
    m = gsum * (f(1) - f(0.9))
    v = (gsum * gsum) * (f(1) - f(0.999))
    bc1 = np.float32(1 - np.float64(np.float32(0.9)))
    bc2 = np.float32(1 - np.float64(np.float32(0.999)))
    w1 = w0 - ((m / bc1) / (np.sqrt(v / bc2) + f(1e-8))) * f(1e-3)
    q.put((rank, gsum, t.numpy()[-2:], w1))
    dist.destroy_process_group()


def test_shard_sum_equals_full_minibatch(orc):
    B, world = 64, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, a, lp, G, A = batch(orc, B)
    ag = orc.Agent(seed=SEED)
    g_full, cd, ad, _ = ag.train_batch(s, a, lp, G, A, b_div=B, apply_adam=False)
    for rank, gsum, diags, w1 in res:
        np.testing.assert_allclose(gsum, g_full, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(diags, [cd, ad], rtol=1e-5, atol=1e-8)
    np.testing.assert_array_equal(res[0][3], res[1][3])  # replicated Adam: identical weights


def test_shard_geometry():
    sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
    from wk.dist import make_shard
    shards = [make_shard(r, 8, r, 8192) for r in range(8)]
    assert [s.env_offset for s in shards] == [r * 8192 for r in range(8)]
    assert all(s.minibatch_global == 65536 for s in shards)
    with pytest.raises(ValueError):
        make_shard(8, 8, 0, 8192)
