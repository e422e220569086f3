"""On-device scenario generation (craft_pool_generate) against the oracle's
restatement of make_data.sample_scenario with the same per-scenario stream."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim
from psketch_amd.cookbook import generator_primitives
from tests.helpers import make_tables
from tests.test_oracle_golden import check_scenario_invariants

pytestmark = pytest.mark.gpu


def gen_args(world):
    params, cb, _, _ = make_tables(world)
    ws = [cb.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])]
    return params, cb, generator_primitives(cb), ws


@pytest.mark.parametrize("world", ["craft_medium", "craft_medium_12x12", "craft_large", "craft_16x16_w7"])
def test_pool_generate_matches_oracle(gpu, oracle_mod, world):
    params, cb, prims, ws = gen_args(world)
    W, H = params["WIDTH"], params["HEIGHT"]
    n = 2048
    sim = CraftSim(world, n_envs=64, device=0, pool_capacity=n + 16)
    init = sim.generate_pool(n, seed=77, first=16, scenario_id0=5000, init_pos=True)
    sim.check()
    want_g, want_i, _ = oracle_mod.generate_scenarios(W, H, cb.index["boundary"], prims,
                                                      params["N_PRIMITIVES"], ws, n, 77,
                                                      scenario_id0=5000)
    assert np.array_equal(init.cpu().numpy(), want_i)
    # read the generated rows back: reset envs onto them and fetch their grids
    m = 64
    for lo in range(0, n, m):
        scen = np.arange(16 + lo, 16 + lo + m, dtype=np.int32)
        sim.reset(scen, want_i[lo:lo + m, 0], want_i[lo:lo + m, 1], np.zeros(m, np.int32),
                  np.zeros(m, np.int32))
        grid = sim.get_state(fields=("grid",))["grid"].cpu().numpy()
        assert np.array_equal(grid, want_g[lo:lo + m]), lo
    sim.check()


def test_pool_generate_full_size_invariants_and_sharding(gpu):
    """524288 worlds (config 4's env count, every env its own world) in one call:
    invariants on a sample, and the same worlds when generated in two shards."""
    params, cb, prims, ws = gen_args("craft_medium_12x12")
    n = 524288
    sim = CraftSim("craft_medium_12x12", n_envs=64, device=0, pool_capacity=n)
    init = sim.generate_pool(n, seed=3, init_pos=True)
    sim.check()
    torch.cuda.synchronize()
    half = CraftSim("craft_medium_12x12", n_envs=64, device=0, pool_capacity=n // 2)
    init_hi = half.generate_pool(n // 2, seed=3, scenario_id0=n // 2, init_pos=True)
    assert torch.equal(init[n // 2:], init_hi)
    # grids of a sample, via reset + get_state, against the invariants
    rng = np.random.RandomState(0)
    pick = rng.choice(n, 64, replace=False).astype(np.int32)
    ini = init.cpu().numpy()
    sim.reset(pick, ini[pick, 0], ini[pick, 1], np.zeros(64, np.int32), np.zeros(64, np.int32))
    grids = sim.get_state(fields=("grid",))["grid"].cpu().numpy()
    check_scenario_invariants(grids, ini[pick], 12, 12, cb.index["boundary"], prims,
                              params["N_PRIMITIVES"], ws)
    # worlds of the top half, generated as a shard of their own, are the same worlds
    def grids_of(sim_, rows, ini_):
        sim_.reset(rows, ini_[rows, 0], ini_[rows, 1], np.zeros(64, np.int32), np.zeros(64, np.int32))
        return sim_.get_state(fields=("grid",))["grid"].cpu().numpy()
    hi = rng.choice(n // 2, 64, replace=False).astype(np.int32)
    assert np.array_equal(grids_of(half, hi, init_hi.cpu().numpy()),
                          grids_of(sim, (hi + n // 2).astype(np.int32), ini))
    sim.check()
    half.check()


def test_generated_pool_rollout_matches_oracle(gpu, oracle_mod):
    """Envs on device-generated worlds step bit-exactly like the oracle."""
    from psketch_amd.sim import synthetic_specs
    params, cb, prims, ws = gen_args("craft_medium_12x12")
    P, n = 512, 2048
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=P)
    sim.generate_pool(P, seed=11)
    grids, _, _ = oracle_mod.generate_scenarios(12, 12, cb.index["boundary"], prims,
                                                params["N_PRIMITIVES"], ws, P, 11)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, 12, 12, n, 0, seed=1, task_ids=tasks)
    sim.reset(*specs)
    o = oracle_mod.Oracle(sim.config, grids)
    envs = o.init_envs(*specs)
    obs = sim.empty_obs()
    for t in range(30):
        sim.step(seed=2, tick=t, obs=obs)
        rc, oobs, _, _, _ = o.batch_tick(envs, 0, None, 2, t, True)
        assert rc == 0
        assert np.array_equal(obs.cpu().numpy(), oobs), t
    sim.check()


@pytest.mark.parametrize("n,kernel", [(65536, 0), (4096, 0), (40000, 1)])
def test_generated_pool_teacher_labels_match_oracle(gpu, oracle_mod, n, kernel):
    """Teacher labels on device-generated worlds (craft_pool_generate marks their free cells
    connected, which the teacher's reachability test uses): the fused labels of craft_step_teach
    (two-tile at 65,536 / one-tile at 4096 and when forced) and craft_teacher against the literal
    BFS oracle on every tick of a sample."""
    from psketch_amd.sim import synthetic_specs
    params, cb, prims, ws = gen_args("craft_medium_12x12")
    P = 1024
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=P)
    sim.tune_teach(kernel)
    sim.generate_pool(P, seed=21)
    grids, _, _ = oracle_mod.generate_scenarios(12, 12, cb.index["boundary"], prims,
                                                params["N_PRIMITIVES"], ws, P, 21)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, 12, 12, n, 0, seed=4, task_ids=tasks)
    sim.reset(*specs)
    o = oracle_mod.Oracle(sim.config, grids)
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    sep = torch.empty(n, dtype=torch.int32, device="cuda")
    ids = np.random.RandomState(n).choice(n, 256, replace=False)
    for t in range(12):
        sim.step(seed=9, tick=t, labels=lab)
        sim.teacher(action_out=sep)
        assert torch.equal(lab, sep), t
        st = {k: v.cpu().numpy() for k, v in sim.get_state(fields=("agent", "inventory", "grid")).items()}
        got = lab.cpu().numpy()
        for i in ids:
            x, y, d, _ = st["agent"][i]
            env = o.env(st["grid"][i], x, y, d, st["inventory"][i])
            rc, act = o.teacher(env, int(specs[4][i]))
            assert rc == 0 and act == got[i], (t, i)
    sim.check()
