"""GPU: the device episode / loss logs against a numpy restatement of
the reference's bookkeeping.

The reference adds trajectory.Rewards.Sum() once per finished episode (PPOAgent.cs:151;
Enumerable.Sum over float accumulates in double, then rounds to float) and the last
minibatch's (valueLoss, actorLoss) once per Train (PPOAgent.cs:165-166).  Bar: bit-exact
(totals, lengths, walker ids, completion order)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250905


class Book:
    """per-walker double accumulators carried across rollouts, like the device's"""

    def __init__(self, n):
        self.acc = np.zeros(n, np.float64)
        self.len = np.zeros(n, np.int64)
        self.clock = 0

    def rollout(self, rewards, dones, env_offset=0):
        T, n = rewards.shape
        out = []
        for t in range(T):
            self.acc += rewards[t].astype(np.float64)
            self.len += 1
            for e in np.nonzero(dones[t])[0]:
                out.append((np.float32(self.acc[e]), env_offset + e, self.len[e], self.clock + t))
                self.acc[e] = 0.0
                self.len[e] = 0
        self.clock += T
        return out

    def reset(self, mask):
        self.acc[mask] = 0.0
        self.len[mask] = 0


def _as_tuples(recs):
    return [(np.float32(r["total_reward"]), int(r["env"]), int(r["length"]), int(r["step"]))
            for r in recs]


@pytest.mark.parametrize("lanes", [1, 2])
def test_episode_log_matches_bookkeeping(wk, lanes):
    n, T = 2048, 64
    eng = wk.Engine(n, seed=SEED, Horizon=T, RandomizeStart=1, RandomizeMaterial=1,
                    MaxTimesteps=100, LanesPerWalker=lanes)
    book = Book(n)
    expect = []
    for k in range(4):
        eng.rollout(T)
        tr = eng.get_trajectory(T)
        expect += book.rollout(tr["rewards"], tr["dones"])
        if k == 1:  # Environment.Reset for a subset: their running sums restart
            mask = (np.arange(n) % 3 == 0).astype(np.uint8)
            eng.reset(mask)
            book.reset(mask.astype(bool))
    recs, dropped = eng.drain_episodes()
    assert dropped == 0 and len(expect) > 1000
    got = _as_tuples(recs)
    assert len(got) == len(expect)
    for g, x in zip(got, expect):
        assert g[1:] == tuple(int(v) for v in x[1:]) and \
            np.float32(g[0]).view(np.uint32) == np.float32(x[0]).view(np.uint32), (g, x)
    assert eng.drain_episodes()[0].size == 0  # drained
    eng.close()


def test_loss_log_and_collect_switch(wk, tmp_path):
    n, T = 512, 16
    eng = wk.Engine(n, seed=SEED, Horizon=T, Minibatch=512, Epochs=2, MaxTimesteps=20)
    diags = []
    for u in range(3):
        eng.rollout(T)
        diags.append(eng.ppo_update(update_index=u))
    c, a = eng.drain_losses()
    np.testing.assert_array_equal(c, np.float32([d[0] for d in diags]))
    np.testing.assert_array_equal(a, np.float32([d[1] for d in diags]))
    recs, _ = eng.drain_episodes()
    assert recs.size > 0
    p = tmp_path / "data.txt"
    wk.write_data_file(p, recs["total_reward"], c, a)
    lines = p.read_text(encoding="utf-8").split("\n")
    assert lines[1] == f"length {recs.size}, total rewards" and lines[4] == "length 3, critic losses"
    eng.collect_data(False)  # Hyperparameters.CollectData = false
    eng.rollout(T)
    eng.ppo_update(update_index=3)
    assert eng.episode_log_count() == (0, 0)
    eng.close()


def test_episode_log_survives_checkpoint(wk, tmp_path):
    n, T = 1024, 32
    kw = dict(Horizon=T, RandomizeStart=1, MaxTimesteps=50)
    a = wk.Engine(n, seed=SEED, **kw)
    a.rollout(T)
    a.drain_episodes()
    a.checkpoint_save(tmp_path / "c.ckpt")  # walkers mid-episode: running sums saved
    a.rollout(T)
    ref, _ = a.drain_episodes()
    b = wk.Engine(n, seed=SEED, **kw)
    b.checkpoint_load(tmp_path / "c.ckpt")
    b.rollout(T)
    got, _ = b.drain_episodes()
    assert ref.size > 0 and got.tobytes() == ref.tobytes()
    a.close()
    b.close()
