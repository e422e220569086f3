"""World-size-2 gloo tests of the sharding plumbing on CPU: each rank runs its
shard of a synthetic rollout (on the CPU oracle, standing in for the GPU kernel
here) and the all-reduced episode summary equals the single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.helpers import make_tables


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_shard(rank, envs_per_rank, T, pool, cfg):
    import oracle
    from psketch_amd import distributed as D
    from psketch_amd.sim import synthetic_specs
    base, n = D.env_shard(rank, envs_per_rank)
    specs = synthetic_specs(pool, 12, 12, n, base, seed=3, task_ids=list(range(12, 26)))
    o = oracle.Oracle(cfg, pool)
    envs = o.init_envs(*specs)
    stats = np.zeros(3, dtype=np.int64)
    obs_sum = 0.0
    for t in range(T):
        rc, obs, _, _, _ = o.batch_tick(envs, base, None, 5, t, True, True, stats)
        assert rc == 0
        obs_sum += float(obs.sum())
    return stats, obs_sum, specs


def _worker(rank, world_size, port, envs_per_rank, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank))
    from psketch_amd import distributed as D
    params, cb, tm, cfg = make_tables("craft_medium_12x12")
    from psketch_amd.sim import sample_scenarios
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    r, ws = D.init(device=torch.device("cpu"))
    assert (r, ws) == (rank, world_size) and D.active()
    stats, obs_sum, specs = _run_shard(rank, envs_per_rank, T, pool, cfg)
    t = torch.tensor(stats, dtype=torch.int64)
    D.reduce_episode_stats(t)
    mx = D.max_over_ranks(float(rank + 1), torch.device("cpu"))
    o = torch.tensor([obs_sum], dtype=torch.float64)
    torch.distributed.all_reduce(o)
    q.put((rank, t.tolist(), mx, float(o.item()), [a.tolist() for a in specs]))
    D.shutdown()


def test_two_rank_shards_equal_single_process():
    world_size, per, T = 2, 300, 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, per, T, q)) for r in range(world_size)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params, cb, tm, cfg = make_tables("craft_medium_12x12")
    from psketch_amd.sim import sample_scenarios, synthetic_specs
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    stats, obs_sum, specs = _run_shard(0, world_size * per, T, pool, cfg)
    for rank, red, mx, osum, sp in res:
        assert red == stats.tolist()
        assert mx == float(world_size)
        assert osum == pytest.approx(obs_sum, rel=0, abs=0)
    cat = [np.concatenate([np.asarray(res[0][4][k]), np.asarray(res[1][4][k])]) for k in range(5)]
    for a, b in zip(cat, specs):
        np.testing.assert_array_equal(a, b)
    assert stats[2] == world_size * per * T
