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


def _all_gather(t):
    """all_gather of a small tensor; through host copies when the backend is gloo and t is on a
    GPU.  Returns a list with one tensor per rank (on t's device)."""
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        out = [torch.empty_like(h) for _ in range(dist.get_world_size())]
        dist.all_gather(out, h)
        return [o.to(t.device) for o in out]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return out


def group_size():
    """World size as the process group reports it (1 without a process group)."""
    return dist.get_world_size() if active(any_size=True) else 1


def run_report(per_rank_s, env_id_base, n_envs, episodes, device,
               names=("successes", "episodes", "env_steps")):
    """What the process group itself says about the run, for the bench line: its backend and
    world size (dist.get_backend / get_world_size, not the launcher's environment) and every
    rank's timed seconds, shard (first global env id, env count) and local episode summary
    {successes, episodes, env-steps}, all-gathered, so a line can be checked for shard
    invariance against N = 1 on its own.  `episodes` holds one integer per name in `names`.
    Without a process group: this process only."""
    row = torch.tensor([dist.get_rank() if active(any_size=True) else 0, int(env_id_base), int(n_envs),
                        *[int(x) for x in episodes], int(round(float(per_rank_s) * 1e9))],
                       dtype=torch.int64, device=device)
    if active(any_size=True):
        rows, backend, ws = _all_gather(row), dist.get_backend(), dist.get_world_size()
    else:
        rows, backend, ws = [row], None, 1
    ranks = []
    for r in rows:
        v = r.cpu().tolist()
        k = len(names)
        ranks.append({"rank": v[0], "env_id_base": v[1], "envs": v[2],
                      "episodes": dict(zip(names, v[3:3 + k])), "per_rank_s": v[3 + k] * 1e-9})
    return {"backend": backend, "world_size": ws, "process_group": backend is not None,
            "per_rank_s": [r["per_rank_s"] for r in ranks], "ranks": ranks}


def barrier():
    if active():
        dist.barrier()


def shutdown():
    if active():
        dist.barrier()
        dist.destroy_process_group()
