"""GPU: bench.py's multi-rank path end to end on one GPU (`--rehearse`): two ranks launched as
the driver launches the 8-GPU run (torch.distributed.run, 127.0.0.1), both on device 0, the
per-minibatch all-reduce on the host over gloo (RCCL refuses two ranks on one device).  Checks
the launcher plumbing, the strong-scaling shard (walkers and minibatch split over the ranks),
the barrier / max-over-ranks timing and the one JSON line from rank 0 -- not a performance
number.  Small shapes: 4,096 global walkers (2,048 per rank: the quad mapping), T = 8."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("exchange", ["rccl", "ipc"])
def test_bench_two_rank_rehearsal(exchange):
    """exchange rccl: with --rehearse the all-reduce goes over the host (gloo); ipc: the one-shot
    exchange over IPC-mapped memory runs on the device, as it would on 8 GPUs"""
    cmd = ["timeout", "-k", "10", "240", sys.executable, "-m", "torch.distributed.run",
           "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--rehearse", "--walkers-global", "4096",
           "--horizon", "8", "--epochs", "1", "--regime-iters", "1", "--exchange", exchange]
    if exchange == "ipc":
        cmd.append("--xch-profile")  # (the exchange kernel's per-block clock split, untimed)
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0, p.stdout[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and "rehearsal" in out
    if exchange == "ipc":  # one split per rank: span / wait / own / gap in microseconds
        prof = out["xch_profile_us"]
        assert len(prof) == 2 and all(r is not None for r in prof), prof
        for r in prof:
            assert r["span"] > 0 and r["own"] > 0 and r["wait"] >= 0 and r["own"] <= r["span"], r
    assert out["config"]["walkers_per_gpu"] == 2048 and out["config"]["global_walkers"] == 4096
    assert out["config"]["minibatch_global"] == 4096
    assert out["config"]["exchange"] == ("ipc" if exchange == "ipc" else "host (gloo)")
    assert "quad" in out["roofline"]["kernel"]
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert abs(out["value"] - 4096 * 8 * 2 / (out["ms_per_step"] * 2e-3)) < 1e-6 * out["value"]


def test_bench_ipc_fallback_when_one_rank_fails():
    """rank 1's IPC test round reports a wrong sum (WK_BENCH_FAULT_RANK, honoured
    only under --rehearse); every rank must vote the IPC exchange down, rebuild its engine, take
    the fallback (the host all-reduce over gloo in a rehearsal, RCCL on a real node) and the job
    must still end with rc 0 and exactly one JSON line"""
    cmd = ["timeout", "-k", "10", "240", sys.executable, "-m", "torch.distributed.run",
           "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--rehearse", "--walkers-global", "4096",
           "--horizon", "8", "--epochs", "1", "--regime-iters", "1", "--exchange", "ipc",
           "--detail-file", ""]
    env = dict(os.environ, WK_BENCH_FAULT_RANK="1")
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       env=env)
    assert p.returncode == 0, p.stdout[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["config"]["exchange"] == "host (gloo)"
    assert out["config"]["exchange_checked"] is False
    assert "rank 1: IPC exchange test gave wrong sums" in p.stdout
    assert out["value"] > 0 and len(lines[0]) < 4096


def test_bench_four_rank_ipc_rehearsal():
    """four ranks on device 0 with the one-shot IPC exchange (three peers' gradients read per
    minibatch, the flag protocol over four ranks): the shard split 4,096 / 4 = 1,024 walkers, the
    exchange checked against the host all-reduce before timing, one JSON line"""
    cmd = ["timeout", "-k", "10", "300", sys.executable, "-m", "torch.distributed.run",
           "--nnodes=1", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "4",
           "--steps", "2", "--warmup", "1", "--rehearse", "--walkers-global", "4096",
           "--horizon", "8", "--epochs", "1", "--regime-iters", "1", "--exchange", "ipc",
           "--detail-file", ""]
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0, p.stdout[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["walkers_per_gpu"] == 1024
    assert out["config"]["exchange"] == "ipc" and out["config"]["exchange_checked"] is True
    assert abs(out["value"] - 4096 * 8 * 2 / (out["ms_per_step"] * 2e-3)) < 1e-6 * out["value"]

