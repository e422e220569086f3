"""The CPU variant of the C ABI (libpsketch_craft_cpu.so, SURVEY.md §8(b): the same entry points
and signatures over host pointers), through psketch_amd.CraftSim(device="cpu"), checked here on
the CPU against the reference's fixtures and the oracle exactly as tests/test_gpu_parity.py checks
the HIP library; tests/test_gpu_cpu_variant.py compares the two libraries on the GPU box."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from psketch_amd import _native as N
from tests.helpers import make_tables, world_for
from tests.test_gpu_parity import set_states


def cpu_sim(world, n, pool, **kw):
    sim = CraftSim(world, n_envs=n, device="cpu", pool_capacity=max(1, len(pool)), **kw)
    sim.load_pool(pool)
    return sim


def test_cpu_library_is_separate_and_explicit():
    """device="cpu" loads the CPU variant; a GPU index never does (no fallback)."""
    assert N.CPU_LIB_PATH != N.LIB_PATH
    params, cb, tm, cfg = make_tables("craft_medium")
    sim = CraftSim("craft_medium", n_envs=4, device="cpu", pool_capacity=1)
    assert sim._L is N.lib(cpu=True) and sim._L is not N.lib()
    with pytest.raises(ValueError):
        CraftSim("craft_medium", n_envs=4, device="meta")


def test_edge_kats_cpu(golden):
    cases = golden("kat_edges.json")
    pool = np.asarray([c["grid"] for c in cases], dtype=np.uint8)
    sim = cpu_sim("craft_medium", len(cases), pool)
    set_states(sim, np.arange(len(cases)), [c["pos"] + [c["dir"]] for c in cases], [c["inv"] for c in cases])
    sim.transition(torch.tensor([c["action"] for c in cases], dtype=torch.int32))
    st = sim.get_state()
    sim.check()
    for i, c in enumerate(cases):
        assert st["agent"][i, :3].tolist() == c["post_pos"] + [c["post_dir"]], c["name"]
        assert st["inventory"][i].tolist() == c["post_inv"], c["name"]
        assert st["grid"][i].tolist() == c["post_grid"], c["name"]


@pytest.mark.parametrize("W", [8, 12])
def test_random_step_kats_cpu(golden, W):
    g = golden("kat_step.npz")
    p = f"w{W}_"
    n = len(g[p + "action"])
    sim = cpu_sim(world_for(W, 3), n, g[p + "pre_grid"])
    set_states(sim, np.arange(n), g[p + "pre_agent"], g[p + "pre_inv"])
    obs = sim.empty_obs(n)
    sim.observe(obs=obs, n=n)
    np.testing.assert_array_equal(obs.numpy(), g[p + "features"].astype(np.float32))
    sat = torch.empty(n, dtype=torch.int8)
    for t in range(g[p + "satisfies"].shape[1]):
        sim.observe(tasks=torch.full((n,), t, dtype=torch.int32), sat=sat, n=n)
        np.testing.assert_array_equal(sat.numpy(), g[p + "satisfies"][:, t], err_msg=f"task {t}")
    sim.transition(torch.as_tensor(g[p + "action"].astype(np.int32)))
    st = sim.get_state()
    sim.check()
    np.testing.assert_array_equal(st["agent"][:, :3].numpy(), g[p + "post_agent"])
    np.testing.assert_array_equal(st["inventory"].numpy(), g[p + "post_inv"])
    np.testing.assert_array_equal(st["grid"].numpy(), g[p + "post_grid"])


def test_teacher_12x12_cpu(golden):
    g = golden("teacher_12x12.npz")
    n = len(g["grid"])
    sim = cpu_sim("craft_medium_12x12", n, g["grid"])
    set_states(sim, np.arange(n), g["agent"], g["inv"])
    plen = torch.empty(n, dtype=torch.int32)
    for t in range(g["action"].shape[1]):
        a, _ = sim.teacher(tasks=torch.full((n,), t, dtype=torch.int32), path_len_out=plen, n=n)
        np.testing.assert_array_equal(a.numpy(), g["action"][:, t], err_msg=f"task {t}")
        ref = g["path_len"][:, t]
        if (ref != -3).all():
            np.testing.assert_array_equal(plen.numpy(), ref, err_msg=f"task {t}")
        try:
            sim.check()
        except N.CraftError as e:
            assert e.status == N.ETEACHER and (g["action"][:, t] == -2).any()


@pytest.mark.parametrize("split", ["dev"])
def test_replay_reference_demonstrations_cpu(golden, split):
    g = golden("devtest.npz")
    n = len(g[f"{split}_task"])
    sim = cpu_sim("craft_medium", n, g[f"{split}_grids"])
    pos = g[f"{split}_pos"].astype(np.int32)
    agent = np.concatenate([pos, np.zeros((n, 1), np.int32)], 1)
    set_states(sim, g[f"{split}_world"], agent, np.zeros((n, 1)), task=g[f"{split}_task"])
    acts = g[f"{split}_actions"].astype(np.int32)
    for t in range(acts.shape[1]):
        ta, _ = sim.teacher(n=n)
        live = acts[:, t] >= 0
        np.testing.assert_array_equal(ta.numpy()[live], acts[live, t], err_msg=f"t={t}")
        step = np.where(live & (acts[:, t] != N.STOP), acts[:, t], -1).astype(np.int32)
        sim.transition(torch.as_tensor(step))
    sat = torch.empty(n, dtype=torch.int8)
    sim.observe(sat=sat, n=n)
    sim.check()
    assert (sat.numpy() == 1).all()


@pytest.mark.parametrize("window", [3, 5])
def test_rollout_fixture_cpu(golden, window):
    g = golden(f"rollout_12x12_w{window}.npz")
    E = g["spec"].shape[0]
    sim = cpu_sim(world_for(12, window), E, g["pool"])
    sp = g["spec"]
    sim.reset(sp[:, 0], sp[:, 1], sp[:, 2], sp[:, 3], sp[:, 4])
    obs = sim.empty_obs()
    rew = torch.empty(E, dtype=torch.float32)
    done = torch.empty(E, dtype=torch.uint8)
    succ = torch.empty(E, dtype=torch.int8)
    ticks = list(g["obs_ticks"])
    seed = int(g["seed"][0])
    for t in range(g["done"].shape[0]):
        sim.step(seed=seed, tick=t, obs=obs, reward=rew, done=done, success=succ)
        st = sim.get_state()
        np.testing.assert_array_equal(done.numpy(), g["done"][t])
        np.testing.assert_array_equal(succ.numpy(), g["success"][t])
        np.testing.assert_array_equal(rew.numpy(), g["reward"][t].astype(np.float32))
        np.testing.assert_array_equal(st["agent"].numpy(), g["agent"][t])
        np.testing.assert_array_equal(st["inventory"].numpy(), g["inv"][t])
        np.testing.assert_array_equal(st["grid"].numpy(), g["grid"][t])
        if t in ticks:
            np.testing.assert_array_equal(obs.numpy(), g["obs"][ticks.index(t)].astype(np.float32))
    sim.check()


@pytest.mark.parametrize("window,autoreset,policy,fmt", [(3, True, False, "f32"), (5, True, True, "bf16"),
                                                         (3, False, True, "u8"), (7, True, False, "f32")])
def test_lockstep_vs_oracle_cpu(oracle_mod, window, autoreset, policy, fmt):
    """Config 2 on the CPU variant: 12x12 (16x16 for 7x7 windows) envs bit-exact against the
    oracle every tick (observation in every format, done, success, reward, counters, states)."""
    W = 16 if window == 7 else 12
    world = "craft_16x16_w7" if window == 7 else world_for(12, window)
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    n = 600
    specs = synthetic_specs(pool, W, W, n, 0, seed=11, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = cpu_sim(world, n, pool)
    sim.set_obs_format(fmt)
    sim.reset(*specs)
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*specs)
    obs = sim.empty_obs()
    rew = torch.empty(n, dtype=torch.float32)
    done = torch.empty(n, dtype=torch.uint8)
    succ = torch.empty(n, dtype=torch.int8)
    rng = np.random.RandomState(window)
    stats = np.zeros(3, dtype=np.int64)
    for t in range(60 if autoreset else 45):
        acts = rng.randint(0, 6, size=n).astype(np.int32) if policy else None
        sim.step(None if acts is None else torch.as_tensor(acts), seed=5, tick=t, autoreset=autoreset, obs=obs,
                 reward=rew, done=done, success=succ)
        rc, oobs, orew, odone, osucc = o.batch_tick(envs, 0, acts, 5, t, autoreset, True, stats)
        assert rc == 0
        np.testing.assert_array_equal(done.numpy(), odone, err_msg=f"t={t}")
        np.testing.assert_array_equal(succ.numpy(), osucc, err_msg=f"t={t}")
        np.testing.assert_array_equal(rew.numpy(), orew, err_msg=f"t={t}")
        np.testing.assert_array_equal(obs.float().numpy(), oobs, err_msg=f"t={t}")
    st = sim.get_state()
    np.testing.assert_array_equal(st["agent"].numpy(), np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1))
    np.testing.assert_array_equal(st["inventory"].numpy(), envs["inv"][:, :cfg.n_kinds])
    np.testing.assert_array_equal(st["grid"].numpy(), envs["grid"][:, :W * W])
    np.testing.assert_array_equal(sim.stats().numpy(), stats)
    sim.check()


def test_multi_tick_rollout_equals_steps_cpu():
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    n, R = 300, 3
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=3, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = cpu_sim(world, n, pool), cpu_sim(world, n, pool)
    for s in (a, b):
        s.reset(*specs)
    ring = torch.zeros((R, n, a.n_features))
    done = torch.zeros((R, n), dtype=torch.uint8)
    obs = torch.zeros((n, a.n_features))
    d1 = torch.zeros(n, dtype=torch.uint8)
    acts = torch.as_tensor(np.random.RandomState(1).randint(0, 6, size=(7, n)).astype(np.int32))
    a.rollout(7, seed=2, tick0=5, actions=acts, obs=ring, done=done)
    for k in range(7):
        b.step(acts[k], seed=2, tick=5 + k, obs=obs, done=d1)
        if k >= 7 - R:
            assert torch.equal(ring[(5 + k) % R], obs) and torch.equal(done[(5 + k) % R], d1), k
    for k, v in a.get_state().items():
        assert torch.equal(v, b.get_state()[k]), k
    assert torch.equal(a.stats(), b.stats())


def test_pool_generate_cpu_matches_oracle_splitmix(oracle_mod):
    """craft_pool_generate on the CPU variant: the HIP kernel's per-scenario splitmix64 stream and
    acceptance test, checked against the oracle's restatement with the same source."""
    world = "craft_medium_12x12"
    sim = CraftSim(world, n_envs=40, device="cpu", pool_capacity=40)
    init = sim.generate_pool(40, seed=77, init_pos=True)
    from psketch_amd.cookbook import generator_primitives
    prims = generator_primitives(sim.cookbook)
    ws = [sim.cookbook.index["workshop%d" % i] for i in range(3)]
    grids, oinit, _ = oracle_mod.generate_scenarios(12, 12, sim.cookbook.index["boundary"], prims, 2, ws, 40, 77,
                                                    rng="splitmix", scenario_id0=0)
    np.testing.assert_array_equal(init.numpy(), oinit)
    sim.reset(np.arange(40, dtype=np.int32), oinit[:, 0], oinit[:, 1], np.zeros(40, np.int32),
              np.zeros(40, np.int32))
    np.testing.assert_array_equal(sim.get_state()["grid"].numpy(), grids)
    sim.check()


def test_cpu_errors_mirror_the_hip_library():
    """The same statuses as the HIP library: a bad action latches EBADACTION with its slot; a
    pool row with an open border is refused; a beyond-capacity load is ERANGE."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 4)
    sim = cpu_sim(world, 64, pool)
    sim.reset(*synthetic_specs(pool, 12, 12, 64, 0, seed=0, task_ids=[12]))
    acts = torch.zeros(64, dtype=torch.int32)
    acts[17] = 9
    sim.step(acts, tick=0)
    w = sim.error_word().tolist()
    assert w[0] == N.EBADACTION and w[2] == 17
    with pytest.raises(N.CraftError) as e:
        sim.check()
    assert e.value.status == N.EBADACTION
    sim.check()
    g = pool[:1].copy()
    g[0, 3] = 0
    with pytest.raises(N.CraftError) as e:
        sim.load_pool(g)
    assert e.value.status == N.EINVARIANT
    with pytest.raises(N.CraftError) as e:
        sim.load_pool(np.repeat(pool, 2, axis=0))
    assert e.value.status == N.ERANGE


def test_host_threads_knob_and_abi_version_cpu():
    """craft_sim_tune_host sets the CPU variant's worker threads (results identical for 1, 3 and
    the machine's); out-of-range values are refused in both libraries' way; both libraries report
    the binding's CRAFT_ABI_VERSION."""
    assert N.lib(cpu=True).craft_abi_version() == N.ABI_VERSION == 2
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    n = 5000
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=4, task_ids=[t.id for t in tm.dataset_tasks()])
    outs = []
    for threads in (1, 3, 0):
        s = cpu_sim(world, n, pool)
        s.tune_host(threads)
        s.reset(*specs)
        ring = torch.zeros((4, n, s.n_features))
        labels = torch.zeros((4, n), dtype=torch.int32)
        s.rollout_teach(4, seed=2, obs=ring, labels=labels)
        s.check()
        outs.append((ring, labels, s.stats()))
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)
    with pytest.raises(N.CraftError):
        s.tune_host(-1)
    with pytest.raises(N.CraftError):
        s.tune_host(4096)
    s.sync_table()                                   # (no table in this variant: a no-op)
