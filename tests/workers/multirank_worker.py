"""One rank of tests/test_gpu_multirank.py: RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from
the environment, gloo control plane, a libwk context on GPU 0 whose minibatch all-reduce goes
through wk_comm_init_host -> torch.distributed.all_reduce (RCCL refuses two ranks on one
device) or, with argv[2] = ipc, through the one-shot exchange over IPC-mapped memory
(wk_comm_init_ipc).  Writes its results to <out>/rank<r>.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ppo-bipedalwalker_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import wk  # noqa: E402
from wk.dist import env_from_launcher, make_shard  # noqa: E402

SEED = 20250905
out_dir = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else "host"  # host all-reduce (gloo) or the IPC exchange
n_local, T = 256, 8
rank, world, _ = env_from_launcher()
dist.init_process_group("gloo")
shard = make_shard(rank, world, 0, n_local, n_local * T)  # one minibatch = the local pool
cfg = dict(Horizon=T, Minibatch=shard.minibatch_local, MinibatchGlobal=shard.minibatch_global,
           EnvOffset=shard.env_offset, RandomizeStart=1, RandomizeMaterial=1, Epochs=1)


def allreduce(a):
    t = torch.from_numpy(a)  # shares the slab's memory
    dist.all_reduce(t)       # gloo sum over the ranks, in place


eng = wk.Engine(n_local, seed=SEED, **cfg)
if mode == "ipc_silent":
    # rank 1 maps the exchange and then never publishes; rank 0's update must
    # fail with WK_ERR_COMM within the 2-s bound and leave W / m / v exactly as they were
    import time

    def allgather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    eng.comm_init_ipc(rank, world, allgather)
    res = {}
    if rank == 0:
        eng.rollout(T)
        eng.sync()
        w_before = eng.get_weights()
        m_before, v_before, _ = eng.get_adam()
        t0 = time.perf_counter()
        try:
            eng.ppo_update(update_index=0)
            raised = ""
        except wk.WkError as ex:
            raised = str(ex)
        res = dict(elapsed=time.perf_counter() - t0, raised=raised, w_before=w_before,
                   w_after=eng.get_weights(), m_before=m_before, v_before=v_before,
                   m_after=eng.get_adam()[0], v_after=eng.get_adam()[1])
    dist.barrier()  # rank 1 waits here (gloo), publishing nothing, until rank 0 is done
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    eng.close()
    dist.destroy_process_group()
    sys.exit(0)
if mode == "ipc_late":
    # a slow but live peer.  One good update on both ranks, then rank 0 updates while
    # rank 1 is busy past the bound; rank 0 fails and aborts its flags, and rank 1, arriving
    # late, must fail the SAME minibatch at once (it reads the abort, not a sequence number)
    # instead of applying it -- both replicas keep the first update's W / m / v, and both report
    # the Adam steps actually applied (1), not the steps attempted
    import time

    def allgather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    eng.comm_init_ipc(rank, world, allgather)
    eng.rollout(T)
    eng.ppo_update(update_index=0)
    eng.sync()
    w1, (m1, v1, t1) = eng.get_weights(), eng.get_adam()
    eng.rollout(T)
    eng.sync()
    dist.barrier()
    if rank == 1:
        dist.barrier()  # busy elsewhere until rank 0 has given up
    t0 = time.perf_counter()
    try:
        eng.ppo_update(update_index=1)
        raised = ""
    except wk.WkError as ex:
        raised = str(ex)
    elapsed = time.perf_counter() - t0
    if rank == 0:
        dist.barrier()
    w2, (m2, v2, t2) = eng.get_weights(), eng.get_adam()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), elapsed=elapsed, raised=raised, w1=w1, m1=m1,
             v1=v1, t1=t1, w2=w2, m2=m2, v2=v2, t2=t2)
    dist.barrier()
    eng.close()
    dist.destroy_process_group()
    sys.exit(0)
solo = wk.Engine(n_local, seed=SEED, **cfg)  # same shard, no communicator
if mode == "ipc":
    def allgather(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    eng.comm_init_ipc(rank, world, allgather)
    # one round of the exchange on exact small integers (bench.py's check of a fresh mapping)
    base = (np.arange(wk.NPARAM) % 97).astype(np.float32)
    ar_test = eng.allreduce_test(base + np.float32(rank + 1))
    ar_want = base * np.float32(world) + np.float32(world * (world + 1) // 2)
    assert np.array_equal(ar_test, ar_want), "IPC exchange test round"
else:
    eng.comm_init_host(rank, world, allreduce)
w0 = eng.get_weights()
eng.rollout(T)
solo.rollout(T)
tr = eng.get_trajectory(T)
tr_solo = solo.get_trajectory(T)
same_traj = all(np.array_equal(tr[k], tr_solo[k]) for k in tr)
same_state = np.array_equal(eng.get_state(), solo.get_state())
# this rank's local gradient of the same (only) minibatch, recomputed by the same kernel
pool = n_local * T
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import orc  # noqa: E402  (checker: the permutation the engine draws its minibatch with)
key = orc.perm_key(SEED, 0, 0)
idx = np.array([orc.perm(i, pool, key) for i in range(pool)])
flat = lambda x, d: x.reshape(pool, d) if d > 1 else x.reshape(pool)
mb = (flat(tr["states"], 12)[idx], flat(tr["actions"], 4)[idx], flat(tr["logp"], 4)[idx],
      flat(tr["returns"], 1)[idx], flat(tr["advantages"], 1)[idx])
g_local, cd_l, ad_l, sk = solo.minibatch_gradient(*mb, b_div=shard.minibatch_global)
# a gradient-only call is collective on every kind of context: the sum over the ranks
# (IPC contexts used to return the rank-local sum here); same weights w0
g_x, _, _, _ = eng.minibatch_gradient(*mb, b_div=shard.minibatch_global)
cd, ad = eng.ppo_update(update_index=0)
w1 = eng.get_weights()
m1, v1, t1 = eng.get_adam()
eng.rollout(T)  # a second iteration: the replicas stay identical
eng.ppo_update(update_index=1)
w2 = eng.get_weights()
# several minibatches and epochs per update (the exchange's sequence numbers and double
# buffering): 3 epochs x 4 minibatches, twice -- on the IPC exchange with the clock stamps on
if mode == "ipc":
    eng.xch_profile(32)
for u in (2, 3):
    eng.rollout(T)
    eng.ppo_update(epochs=3, minibatch=shard.minibatch_local // 4,
                   minibatch_global=shard.minibatch_global // 4, update_index=u)
w3 = eng.get_weights()
m3, v3, t3 = eng.get_adam()
stamps = eng.xch_stamps(32) if mode == "ipc" else np.zeros((0, 0, 4), np.uint64)
np.savez(os.path.join(out_dir, f"rank{rank}.npz"), w0=w0, w1=w1, m1=m1, v1=v1, t1=t1, w2=w2, stamps=stamps,
         w3=w3, m3=m3, v3=v3, t3=t3,
         g_local=g_local, g_x=g_x, cd=cd, ad=ad, cd_l=cd_l, ad_l=ad_l, same_traj=same_traj,
         same_state=same_state, state=eng.get_state())
eng.close()
solo.close()
dist.destroy_process_group()
