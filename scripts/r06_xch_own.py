"""the IPC exchange's own work per minibatch, measured without contention.

In bench.py's one-GPU rehearsal every rank runs the same shard, so the ranks' gradient kernels
share the GPU and the exchange kernel's stamps carry the other rank's load.  Here rank 0 runs
the 8-GPU shard's update (8,192 walkers, 8,192-sample minibatches: k_ppo_grad_tp<2> +
k_reduce_xch_adam with Adam, per minibatch of wk_ppo_update) while the other ranks run 16 walkers
with 16-sample minibatches (the same number of minibatches): their tiny gradient kernels finish
first and their exchange blocks sit in the bounded wait (s_sleep), so rank 0's exchange kernel
runs on an otherwise idle GPU.  Its per-block stamps (wk_comm_xch_profile) split each launch into
reduction + publish (entry -> published), wait (published -> peers seen: ~0 here) and peer reads
+ Adam (peers seen -> exit).  A solo context (no exchange) runs the same minibatches through the
single-GPU path (k_grad_reduce_fused<true>) for the difference.

usage (GPU box): python3 scripts/r06_xch_own.py [ranks] [updates] -- the parent never touches the
GPU; it starts one child process per rank under `rocprofv3 --kernel-trace --stats` (the program
after -- is python3 itself) and prints rank 0's JSON summary."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "r06_xch_own")


def child(rank, world, reps, port):
    sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import wk
    import torch.distributed as dist
    from bench import xch_stamp_summary
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # the update path (wk_ppo_update: the tile-parallel gradient kernel at 8,192 samples, then the
    # exchange); rank 0 the shard (8,192 walkers, M 8,192), the others 16 walkers (M 16): the same
    # 8 minibatches per epoch, 40 per update
    T, E = 8, 5
    n, M = (8192, 8192) if rank == 0 else (16, 16)
    mk = lambda: wk.Engine(n, seed=20250905, Horizon=T, Minibatch=M, MinibatchGlobal=8192 * world,
                           Epochs=E, RandomizeStart=1, EnvOffset=rank * 8192)
    eng = mk()

    def allgather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    eng.comm_init_ipc(rank, world, allgather)
    mb = E * (n * T // M)
    eng.rollout(T)
    eng.ppo_update(update_index=0)  # warm
    eng.xch_profile(mb * reps)
    for u in range(reps):
        eng.rollout(T)
        eng.ppo_update(update_index=1 + u)
    st = eng.xch_stamps(mb * reps)
    summ = xch_stamp_summary(st)
    f = st.astype(np.float64) * 0.01
    summ["reduce_publish_us_median"] = float(np.median(np.median(f[:, :, 1] - f[:, :, 0], axis=1)))
    summ["read_adam_us_median"] = float(np.median(np.median(f[:, :, 3] - f[:, :, 2], axis=1)))
    summ["grad_kernel"] = eng.grad_kernel(M)
    if rank == 0:  # the single-GPU path on the same shard (k_grad_reduce_fused<true> in the trace)
        one = wk.Engine(n, seed=20250905, Horizon=T, Minibatch=M, MinibatchGlobal=8192 * world,
                        Epochs=E, RandomizeStart=1)
        for u in range(reps + 1):
            one.rollout(T)
            one.ppo_update(update_index=u)
        one.close()
    res = allgather({"rank": rank, "walkers": n, "minibatch": M, "summary": summ})
    eng.close()
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"ranks": world, "updates": reps, "per_rank": res}, indent=1))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    os.makedirs(OUT, exist_ok=True)
    port = 29700 + int(time.time()) % 200
    procs = []
    for r in range(world):
        cmd = ["timeout", "-k", "10", "240", "rocprofv3", "--kernel-trace", "--stats", "-d",
               os.path.join(OUT, f"n{world}_r{r}"), "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--child", str(r), str(world), str(reps),
               str(port)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      text=True, cwd=ROOT))
    out0 = procs[0].communicate()[0]
    rcs = [p.wait() for p in procs]
    print(out0)
    if any(rcs):
        raise SystemExit(f"rank exit codes {rcs}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    else:
        main()
