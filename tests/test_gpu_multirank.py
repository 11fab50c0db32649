"""GPU, two (and three) processes sharing GPU 0: libwk's multi-rank minibatch sequence.

RCCL refuses two ranks on one device, so the ranks' all-reduce goes through
wk_comm_init_host (the same sequence: ordered block reduction -> all-reduce of the 6,153-float
slab -> replicated Adam) with torch.distributed over gloo -- and, as the second exchange, through
the one-shot IPC exchange (wk_comm_init_ipc: each rank's slab published in its own
peer-mapped region, read by the others, summed in rank order, Adam fused), which must give the
host all-reduce's results bit for bit (two processes on one GPU still run on different XCDs'
L2 caches: the system-scope release / acquire of the exchange is exercised).  Each rank holds its contiguous
shard of the walkers (EnvOffset = rank x 256) and the global minibatch divisor; checked:

  * each rank's rollout equals a communicator-free context on the same shard (sharding by
    EnvOffset: Philox streams keyed by the global walker id);
  * after one minibatch the all-reduced update is exactly Adam(t = 1) of the SUM of the two
    ranks' local gradients (each recomputed by the same kernel on the same permuted samples,
    divisor = global minibatch), bit for bit in float32 -- the sum the RCCL all-reduce forms;
  * the diagnostics are the sums of the ranks' local diagnostics;
  * the two replicas' weights and Adam state stay bit-identical through a second iteration.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _adam_t1(w, g, alpha=np.float32(0.001), beta1=0.9, beta2=0.999, eps=np.float32(1e-8)):
    """DenseLayer.Adam at t = 1 from zero moments, op for op as adam_param (wk_ppo.hip)"""
    f = np.float32
    c1, c2 = f(1.0) - f(beta1), f(1.0) - f(beta2)
    bc1 = f(1.0 - np.float64(f(beta1)) ** 1)
    bc2 = f(1.0 - np.float64(f(beta2)) ** 1)
    m = (g * c1) + (np.zeros_like(g) * f(beta1))
    v = (np.zeros_like(g) * f(beta2)) + ((g * g) * c2)
    mh = m / bc1
    vh = v / bc2
    den = np.sqrt(vh) + eps
    return w - ((mh / den) * alpha), m, v


def _run_two_ranks(out, mode, n=2, **extra_env):
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **extra_env)
        procs.append(subprocess.Popen(
            ["timeout", "-k", "10", "240", sys.executable,
             os.path.join(ROOT, "tests", "workers", "multirank_worker.py"), str(out), mode],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate()[0] for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return [np.load(out / f"rank{r}.npz") for r in range(n)]


@pytest.fixture(scope="module")
def two_rank_runs(tmp_path_factory):
    """both exchanges, each with two processes on GPU 0"""
    return {mode: _run_two_ranks(tmp_path_factory.mktemp(mode), mode) for mode in ("host", "ipc")}


@pytest.mark.parametrize("mode", ["host", "ipc"])
def test_two_ranks_allreduce(two_rank_runs, mode):
    r0, r1 = two_rank_runs[mode]
    for r in (r0, r1):
        assert r["same_traj"] and r["same_state"]
    np.testing.assert_array_equal(r0["w0"], r1["w0"])
    g_sum = r0["g_local"] + r1["g_local"]
    w_ref, m_ref, v_ref = _adam_t1(r0["w0"], g_sum)
    for r in (r0, r1):
        np.testing.assert_array_equal(r["w1"], w_ref)
        np.testing.assert_array_equal(r["m1"], m_ref)
        np.testing.assert_array_equal(r["v1"], v_ref)
        assert int(r["t1"]) == 1
        assert float(r["cd"]) == np.float32(r0["cd_l"]) + np.float32(r1["cd_l"])
        assert float(r["ad"]) == np.float32(r0["ad_l"]) + np.float32(r1["ad_l"])
    for r in (r0, r1):  # gradient-only calls are collective: the sum over the ranks
        np.testing.assert_array_equal(r["g_x"], g_sum)
    np.testing.assert_array_equal(r0["w2"], r1["w2"])
    np.testing.assert_array_equal(r0["w3"], r1["w3"])
    assert int(r0["t3"]) == int(r1["t3"]) == 2 + 2 * 3 * 4
    assert not np.array_equal(r0["state"], r1["state"])  # different shards


def test_ipc_exchange_equals_host_allreduce(two_rank_runs):
    """the one-shot IPC exchange (peer-mapped slabs, rank-order sum, fused Adam) gives the host
    all-reduce's weights and Adam moments bit for bit -- through 26 Adam steps with several
    minibatches and epochs per update (sequence numbers, double-buffered slabs)"""
    for h, i in zip(two_rank_runs["host"], two_rank_runs["ipc"]):
        for k in ("w1", "m1", "v1", "w2", "w3", "m3", "v3", "state"):
            np.testing.assert_array_equal(h[k], i[k], err_msg=k)
        assert float(h["cd"]) == float(i["cd"]) and float(h["ad"]) == float(i["ad"])


def test_ipc_exchange_clock_stamps(two_rank_runs):
    """wk_comm_xch_profile stamps every exchange launch per block -- entry, slab
    published, every peer's flag seen, exit -- in that order, and the launches follow each other
    on the stream (the next launch's first entry after this one's last exit: a gradient kernel
    runs between them); the summary bench.py --xch-profile prints from them is consistent"""
    import bench
    for r in two_rank_runs["ipc"]:
        st = r["stamps"]
        assert st.shape == (24, 97, 4), st.shape  # 2 updates x 3 epochs x 4 minibatches
        assert (st > 0).all()
        d = np.diff(st.astype(np.int64), axis=2)
        assert (d >= 0).all()  # entry <= published <= peers seen <= exit
        assert (st[1:, :, 0].min(axis=1) >= st[:-1, :, 3].max(axis=1)).all()
        s = bench.xch_stamp_summary(st)
        assert s["launches"] == 24 and 0 < s["own_us_median"] < s["span_us_median"] + 1e-9


def test_three_ranks_ipc_rank_order_sum(tmp_path):
    """three processes (an odd rank count): the IPC exchange sums the ranks' local slabs in rank
    order, ((g0 + g1) + g2) in float32, and every replica applies the same Adam step"""
    rs = _run_two_ranks(tmp_path, "ipc", n=3)
    for r in rs:
        assert r["same_traj"] and r["same_state"]
    g_sum = (rs[0]["g_local"] + rs[1]["g_local"]) + rs[2]["g_local"]
    w_ref, m_ref, v_ref = _adam_t1(rs[0]["w0"], g_sum)
    cd_ref = (np.float32(rs[0]["cd_l"]) + np.float32(rs[1]["cd_l"])) + np.float32(rs[2]["cd_l"])
    for r in rs:
        np.testing.assert_array_equal(r["w1"], w_ref)
        np.testing.assert_array_equal(r["m1"], m_ref)
        np.testing.assert_array_equal(r["v1"], v_ref)
        assert float(r["cd"]) == cd_ref
    for k in ("w2", "w3", "m3", "v3"):
        np.testing.assert_array_equal(rs[0][k], rs[1][k], err_msg=k)
        np.testing.assert_array_equal(rs[0][k], rs[2][k], err_msg=k)
    assert int(rs[2]["t3"]) == 2 + 2 * 3 * 4


def test_ipc_peer_never_publishes(tmp_path):
    """rank 1 maps the exchange and then never publishes.  Rank 0's update
    fails with WK_ERR_COMM after the bound (WK_XCH_TIMEOUT_S = 2 s of the 100 MHz constant clock
    here; 30 s by default; the later minibatches return at once) and applies no Adam step: W, m
    and v are bit-identical before and after"""
    r0, _ = _run_two_ranks(tmp_path, "ipc_silent", WK_XCH_TIMEOUT_S="2")
    print(f"failing update took {float(r0['elapsed']):.2f} s: {r0['raised']}")
    assert "did not publish" in str(r0["raised"])
    assert 1.5 <= float(r0["elapsed"]) <= 8.0
    for k in ("w", "m", "v"):
        np.testing.assert_array_equal(r0[k + "_before"], r0[k + "_after"], err_msg=k)


def test_ipc_late_peer_fails_the_same_minibatch(tmp_path):
    """rank 1 is alive but late (busy past the 2-s bound while rank 0 has its update
    queued).  Rank 0 times out and marks its flags aborted; rank 1 then fails the same minibatch
    at once instead of applying it.  Both replicas keep the first update's W / m / v bit for bit,
    and both report Adam step 1 (the steps applied), not 2 (the steps attempted)"""
    r0, r1 = _run_two_ranks(tmp_path, "ipc_late", WK_XCH_TIMEOUT_S="2")
    print(f"rank 0 failed after {float(r0['elapsed']):.2f} s, rank 1 after {float(r1['elapsed']):.2f} s")
    for r in (r0, r1):
        assert "did not publish" in str(r["raised"]) and "step 1" in str(r["raised"])
        assert int(r["t1"]) == 1 and int(r["t2"]) == 1
        for k in ("w", "m", "v"):
            np.testing.assert_array_equal(r[k + "1"], r[k + "2"], err_msg=k)
    np.testing.assert_array_equal(r0["w2"], r1["w2"])
    assert 1.5 <= float(r0["elapsed"]) <= 8.0
    assert float(r1["elapsed"]) < 1.0  # the abort value, not a second timeout


def test_ipc_refuses_more_than_four_ranks_per_gpu(wk):
    """wk_comm_init_ipc counts the ranks whose record names this rank's GPU and refuses more than
    four (their waiting exchange blocks would hold the CUs a peer's gradient kernel needs)"""
    eng = wk.Engine(64, seed=20250905, Horizon=4, Minibatch=64)
    rec = eng.comm_ipc_handle()
    assert len(rec) == wk.IPC_HANDLE_BYTES and rec[64:].rstrip(b"\0")  # the PCI bus id
    with pytest.raises(wk.WkError, match="at most 4 ranks per GPU"):
        eng.comm_init_ipc_records(0, 5, [rec] * 5)
    eng.close()


def test_failing_host_allreduce_is_reported(wk):
    """a host all-reduce callback that raises fails wk_ppo_update with WK_ERR_COMM,
    and the error names the callback's exception (the caller must abort the job)"""
    eng = wk.Engine(64, seed=20250905, Horizon=4, Minibatch=64, Epochs=1)

    def broken(buf):
        raise ConnectionError("peer 1 went away")

    eng.comm_init_host(0, 1, broken)
    eng.rollout(4)
    with pytest.raises(wk.WkError, match="ConnectionError: peer 1 went away"):
        eng.ppo_update(update_index=0)
    eng.close()
