"""Multi-GPU sharding for the walker engine (one process per GPU).

Walkers are independent (each owns its floor copy, Environment.cs:27,43-48), so env
ranges shard with no data-path collective; the only exchange is the RCCL all-reduce
of the flat 6,149-float policy gradient per minibatch inside wk_ppo_update (each rank
scales its per-sample gradients by 1/global minibatch, so the sum is the reference's
sum / BatchSize over the global minibatch).  Adam then runs replicated on every rank
from identically seeded weights (no broadcast).
"""
import os
from dataclasses import dataclass


@dataclass
class Shard:
    rank: int
    world: int
    local_rank: int
    n_local: int
    env_offset: int
    minibatch_local: int
    minibatch_global: int


def env_from_launcher():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def make_shard(rank, world, local_rank, walkers_per_rank, minibatch_per_rank=None):
    """Contiguous env range per rank; global env id = rank * walkers_per_rank + e, so
    every Philox stream (start offsets, materials, action noise) is independent of the
    number of GPUs."""
    if walkers_per_rank <= 0 or world <= 0 or not (0 <= rank < world):
        raise ValueError("bad shard geometry")
    m = walkers_per_rank if minibatch_per_rank is None else minibatch_per_rank
    return Shard(rank=rank, world=world, local_rank=local_rank, n_local=walkers_per_rank,
                 env_offset=rank * walkers_per_rank, minibatch_local=m,
                 minibatch_global=m * world)


def broadcast_unique_id(uid_or_none, group=None):
    """Rank 0's RCCL unique id to every rank over torch.distributed (control plane)."""
    import torch
    import torch.distributed as dist
    buf = torch.zeros(128, dtype=torch.uint8)
    if dist.get_rank() == 0:
        buf[:] = torch.tensor(list(uid_or_none), dtype=torch.uint8)
    dist.broadcast(buf, src=0, group=group)
    return bytes(buf.tolist())


def gather_episode_log(recs, group=None):
    """Cross-rank aggregation for the data file: every rank's drained episode records are
    gathered to all ranks (torch.distributed, any backend) and merged in completion order
    (env-step, global walker id) -- the order one context holding all walkers would log."""
    import numpy as np
    import torch.distributed as dist
    from . import EPISODE_DTYPE
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, np.asarray(recs, EPISODE_DTYPE).tobytes(), group=group)
    allr = np.concatenate([np.frombuffer(b, EPISODE_DTYPE) for b in parts])
    return allr[np.lexsort((allr["env"], allr["step"]))]
