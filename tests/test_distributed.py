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
    report = D.run_report(0.5 * (rank + 1), D.env_shard(rank, envs_per_rank)[0], envs_per_rank,
                          t.tolist(), torch.device("cpu"))
    D.reduce_episode_stats(t)
    mx = D.max_over_ranks(float(rank + 1), torch.device("cpu"))
    o = torch.tensor([obs_sum], dtype=torch.float64)
    torch.distributed.all_reduce(o)
    q.put((rank, t.tolist(), mx, float(o.item()), [a.tolist() for a in specs], report,
           stats.tolist()))
    D.shutdown()


def test_run_report_without_a_process_group():
    """N = 1 without a process group: the line says so (backend None) and reports this process."""
    from psketch_amd import distributed as D
    rep = D.run_report(1.25, 0, 64, [1, 2, 3], torch.device("cpu"))
    assert rep["backend"] is None and rep["world_size"] == 1 and rep["process_group"] is False
    assert rep["ranks"] == [{"rank": 0, "env_id_base": 0, "envs": 64, "per_rank_s": 1.25,
                             "episodes": {"successes": 1, "episodes": 2, "env_steps": 3}}]
    rep = D.run_report(0.0, 8, 4, [5, 6, 7], torch.device("cpu"), names=("a", "b", "c"))
    assert rep["ranks"][0]["episodes"] == {"a": 5, "b": 6, "c": 7}


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
    local = [r[6] for r in res]
    for rank, red, mx, osum, sp, report, _ in res:
        assert red == stats.tolist()
        assert mx == float(world_size)
        assert osum == pytest.approx(obs_sum, rel=0, abs=0)
        # the bench line's "dist" block: the process group's own backend and size, and every
        # rank's shard, clock and local summary, identical on every rank
        assert report["backend"] == "gloo" and report["world_size"] == world_size
        assert report["process_group"] is True
        assert [r["rank"] for r in report["ranks"]] == list(range(world_size))
        assert [r["env_id_base"] for r in report["ranks"]] == [r * per for r in range(world_size)]
        assert [r["envs"] for r in report["ranks"]] == [per] * world_size
        assert report["per_rank_s"] == pytest.approx([0.5, 1.0])
        assert [list(r["episodes"].values()) for r in report["ranks"]] == local
        # shard invariance from the line alone: the per-rank summaries add up to N = 1's
        assert np.sum(local, axis=0).tolist() == stats.tolist()
    cat = [np.concatenate([np.asarray(res[0][4][k]), np.asarray(res[1][4][k])]) for k in range(5)]
    for a, b in zip(cat, specs):
        np.testing.assert_array_equal(a, b)
    assert stats[2] == world_size * per * T
