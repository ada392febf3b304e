"""Data-parallel plumbing: one process per GPU, torch.distributed (backend "nccl" = RCCL over xGMI).

Rollout shards envs across ranks with no collective (envs are independent). The learner
is replicated; each rank samples its own PER shard and the flat gradient buffer
``P = [agent | mixer]`` is summed with ONE all-reduce per update, then averaged by
1/world inside the clip/Adam kernel (post-reduce global-norm clipping).
Equal per-rank batches make the averaged gradient the gradient of the mean loss over
the union batch.
"""
import os

import torch
import torch.distributed as tdist


def init_from_env(device=None, backend=None):
    """Read RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (torch.distributed.run) and init the group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not tdist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        tdist.init_process_group(backend, **kw)
    return rank, world


def make_allreduce(group=None):
    """Returns f(flat_grad) -> world: in-place SUM all-reduce of the flat gradient buffer."""
    world = tdist.get_world_size(group)

    def allreduce(g):
        tdist.all_reduce(g, op=tdist.ReduceOp.SUM, group=group)
        return world

    return allreduce


def broadcast_params(flat, src=0, group=None):
    """Make every replica start from rank ``src``'s parameters."""
    tdist.broadcast(flat, src, group=group)


def max_over_ranks(x, device):
    t = torch.tensor([float(x)], device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())
