"""Multi-GPU plumbing: one process per GPU, envs sharded by global id.

Envs are independent (no cross-env reads anywhere in worlds/craft.py), so the
data path has no collective: rank r simulates global env ids
[r * N, (r + 1) * N) and every per-env random draw is keyed by global id, which
makes results identical for any number of GPUs.  The only exchange is the
episode summary {successes, episodes, env-steps} (int64[3]) all-reduced once
over RCCL (torch.distributed backend "nccl" on ROCm), and the max over ranks
of the timed region.
"""
import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(device=None, backend=None, force=False):
    """Initialise the process group when WORLD_SIZE > 1 (RCCL for GPUs, gloo on
    CPU; backend="gloo" with a GPU device keeps the data on the GPU and runs the
    two scalar collectives through host copies — a rehearsal of several ranks on
    one card).  force=True initialises a one-rank group too (the RCCL path on a
    one-GPU box)."""
    rank, ws, _ = world()
    if (ws > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if device is not None and device.type == "cuda" else "gloo"
        kw = {"device_id": device} if backend == "nccl" and device is not None else {}
        dist.init_process_group(backend, **kw)
    return rank, ws


def _reduce(t, op):
    """all_reduce in place; through a host copy when the backend is gloo and t is on a GPU."""
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def env_shard(rank, envs_per_rank):
    """Global id of this rank's first env and its env count (weak scaling)."""
    return rank * envs_per_rank, envs_per_rank


def active(any_size=False):
    """A process group with more than one rank (any_size: with at least one)."""
    return dist.is_available() and dist.is_initialized() and (any_size or dist.get_world_size() > 1)


def reduce_episode_stats(stats):
    """Sum the int64[3] episode summaries of all ranks (in place)."""
    if active():
        _reduce(stats, dist.ReduceOp.SUM)
    return stats


def max_over_ranks(value, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if active():
        _reduce(t, dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if active():
        dist.barrier()


def shutdown():
    if active():
        dist.barrier()
        dist.destroy_process_group()
