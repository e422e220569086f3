"""BASELINE.json configs[0] and configs[3] on the HIP path.

configs[0]: one CraftWorld env on the first craft_medium_train.json instance,
a 100-step random rollout, replayed bit-exactly against the reference's own
run (tests/golden/config1_train0.npz) through the drop-in
psketch_amd.worlds.CraftWorld and through CraftSim.

configs[3]: 524288 envs, the 8-GPU sharding of the bench workload, on one
GPU: one CraftSim of 524288 envs against 8 CraftSims of 65536 envs with
env_id_base = r * 65536 (what each rank of an 8-GPU run simulates), through
craft_rollout (K = 32, the default shape) and craft_step; plus an oracle
spot-check of 256 random global ids.  Envs are independent (craft.py:332-424
reads no other env), so every output must be identical."""
from types import SimpleNamespace as NS

import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs, worlds
from psketch_amd import distributed as D
from psketch_amd.cookbook import Task
from tests.helpers import make_tables

pytestmark = pytest.mark.gpu


def host(t):
    return t.cpu().numpy()


def _onehot(ids, W, H, K=21):
    g = np.zeros((W, H, K))
    ids = np.asarray(ids).reshape(W, H)
    for k in range(1, K):
        g[..., k] = ids == k
    return g


def test_config1_dropin_world_replays_reference(golden):
    g = golden("config1_train0.npz")
    cfg = NS(recipes="resources/craft/recipes.yaml", world=NS(name="CraftWorld", config="craft_medium"),
             student=NS(model=NS()), teacher=NS(name="DemonstrationTeacher"),
             trainer=NS(hints="resources/craft/hints.hierarchy.yaml", max_timesteps=40),
             random=np.random.RandomState(0))
    w = worlds.load(cfg)
    t_ref = w.task_manager.tasks[int(g["task"][0])]
    task = Task(f"{t_ref.goal_name}[{t_ref.goal_arg}]")
    x, y = (int(v) for v in g["init_pos"])
    s = w.init_state(_onehot(g["grid"][0], 8, 8), (x, y))
    states = [s]
    for t in range(len(g["actions"]) + 1):
        if t:
            r, s = s.step(int(g["actions"][t - 1]))
            assert r == 0
            states.append(s)
        assert s.pos == tuple(int(v) for v in g["pos"][t]) and s.dir == int(g["dir"][t]), t
        np.testing.assert_array_equal(s.inventory, g["inv"][t].astype(np.float64))
        ids = s.grid.argmax(axis=2).reshape(-1) * (s.grid.max(axis=2).reshape(-1) > 0)
        np.testing.assert_array_equal(ids, g["grid"][t])
        np.testing.assert_array_equal(s.features(), g["features"][t].astype(np.float64))
        assert s.satisfies(task) == bool(g["satisfies"][t])
    # the reference's states are immutable: earlier ones still read as recorded
    for t in (0, 1, 50):
        assert states[t].pos == tuple(int(v) for v in g["pos"][t])
        np.testing.assert_array_equal(states[t].features(), g["features"][t].astype(np.float64))


def test_config1_craftsim_replays_reference(golden):
    g = golden("config1_train0.npz")
    sim = CraftSim("craft_medium", n_envs=1, device=0, pool_capacity=1)
    sim.load_pool(g["grid"][:1])
    x, y = (int(v) for v in g["init_pos"])
    task = int(g["task"][0])

    def one(v):
        return torch.tensor([v], dtype=torch.int32, device="cuda")

    sim.reset(one(0), one(x), one(y), one(0), one(task))
    obs = sim.empty_obs()
    sat = torch.empty(1, dtype=torch.int8, device="cuda")
    for t in range(len(g["actions"]) + 1):
        if t:
            sim.transition(one(int(g["actions"][t - 1])))
        sim.observe(obs=obs, sat=sat)
        st = sim.get_state()
        a = host(st["agent"])[0]
        assert (a[0], a[1], a[2]) == (g["pos"][t][0], g["pos"][t][1], g["dir"][t]), t
        np.testing.assert_array_equal(host(st["inventory"])[0], g["inv"][t])
        np.testing.assert_array_equal(host(st["grid"])[0], g["grid"][t])
        np.testing.assert_array_equal(host(obs)[0], g["features"][t].astype(np.float32))
        assert int(sat[0]) == g["satisfies"][t]
    sim.check()
    # the reference's first demonstration action from the initial state
    sim.reset(one(0), one(x), one(y), one(0), one(task))
    act, _ = sim.teacher()
    assert int(act[0]) == int(g["demo"][0])
    sim.check()


def test_config4_524288_envs_sharded_eight_ways(oracle_mod):
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 1024)
    G, per, K, L = 8, 65536, 32, 2
    n = G * per
    tasks = [t.id for t in tm.dataset_tasks()]
    seed = 11

    def make(base, count):
        sim = CraftSim(world, n_envs=count, device=0, env_id_base=base, pool_capacity=1024)
        sim.load_pool(pool)
        sim.reset(*synthetic_specs(pool, 12, 12, count, base, seed=0, task_ids=tasks))
        return sim

    big, stepper = make(0, n), make(0, n)
    shards = [make(r * per, per) for r in range(G)]
    F = big.n_features
    dev = torch.device("cuda", 0)

    def rings(count):
        return (torch.empty((K, count, F), dtype=torch.float32, device=dev),
                {k: torch.empty((K, count), dtype=dt, device=dev) for k, dt in
                 (("reward", torch.float32), ("done", torch.uint8), ("success", torch.int8))})

    big_obs, big_out = rings(n)
    sh_obs, sh_out = rings(per)
    st_obs = torch.empty((n, F), dtype=torch.float32, device=dev)
    st_out = {k: torch.empty(n, dtype=v.dtype, device=dev) for k, v in big_out.items()}
    ids = np.sort(np.random.RandomState(2).choice(n, 256, replace=False))
    ids_t = torch.as_tensor(ids, device=dev)
    picked = []                                    # per launch: obs rows of the spot-check ids
    for launch in range(L):
        tick0 = launch * K
        big.rollout(K, seed=seed, tick0=tick0, obs=big_obs, **big_out)
        for r, sh in enumerate(shards):
            sh.rollout(K, seed=seed, tick0=tick0, obs=sh_obs, **sh_out)
            sl = slice(r * per, (r + 1) * per)
            assert torch.equal(sh_obs, big_obs[:, sl]), (launch, r)
            for k in sh_out:
                assert torch.equal(sh_out[k], big_out[k][:, sl]), (launch, r, k)
        for t in range(K):
            stepper.step(seed=seed, tick=tick0 + t, obs=st_obs, **st_out)
            assert torch.equal(st_obs, big_obs[t]), tick0 + t
            for k in st_out:
                assert torch.equal(st_out[k], big_out[k][t]), (tick0 + t, k)
        picked.append(host(big_obs[:, ids_t]))
    state = big.get_state()
    cat = [sh.get_state() for sh in shards]
    st2 = stepper.get_state()
    for k in state:
        assert torch.equal(torch.cat([c[k] for c in cat]), state[k]), k
        assert torch.equal(st2[k], state[k]), k
    total = sum(host(sh.stats()) for sh in shards)
    np.testing.assert_array_equal(total, host(big.stats()))
    np.testing.assert_array_equal(host(D.reduce_episode_stats(big.stats())), host(stepper.stats()))
    assert total[2] == n * K * L
    for s in [big, stepper] + shards:
        s.check()
    # oracle spot-check on 256 random global ids, every tick
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=0, task_ids=tasks)
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*[a[ids] for a in specs])
    picked = np.concatenate(picked, 0)             # [K * L, 256, F]
    for t in range(K * L):
        for j, gid in enumerate(ids):
            rc, oobs, _, _, _ = o.batch_tick(envs[j:j + 1], int(gid), None, seed, t, True)
            assert rc == 0
            np.testing.assert_array_equal(picked[t, j], oobs[0], err_msg=f"gid {gid} tick {t}")
