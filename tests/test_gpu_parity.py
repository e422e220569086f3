"""Parity of the HIP path (through the C ABI) against the reference fixtures and
the CPU oracle.  Bit-exact everywhere: every quantity is integer (features are
small integers in fp32)."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from psketch_amd import _native as N
from tests.helpers import make_tables, world_for

pytestmark = pytest.mark.gpu


def sim_with_pool(world, n, pool, **kw):
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=max(1, len(pool)), **kw)
    sim.load_pool(pool)
    return sim


def set_states(sim, grids_idx, agent, inv, task=None, dirs=None):
    """Slots 0..n-1 := (pool entry, x, y, dir, inventory)."""
    n = len(grids_idx)
    agent = np.asarray(agent, dtype=np.int32)
    task = np.zeros(n, dtype=np.int32) if task is None else np.asarray(task, dtype=np.int32)
    spec = np.stack([np.asarray(grids_idx), agent[:, 0], agent[:, 1], agent[:, 2], task], 1)
    ag = np.concatenate([agent[:, :3], np.full((n, 1), 40)], 1)
    K = sim.n_kinds
    iv = np.zeros((n, K), dtype=np.int32)
    inv = np.asarray(inv)
    iv[:, :inv.shape[1]] = inv[:, :K]
    sim.set_state(spec, ag, iv)


def host(t):
    return t.cpu().numpy()


def test_edge_kats(golden):
    cases = golden("kat_edges.json")
    pool = np.asarray([c["grid"] for c in cases], dtype=np.uint8)
    sim = sim_with_pool("craft_medium", len(cases), pool)
    set_states(sim, np.arange(len(cases)), [c["pos"] + [c["dir"]] for c in cases],
               [c["inv"] for c in cases])
    sim.transition(torch.tensor([c["action"] for c in cases], dtype=torch.int32, device="cuda"))
    st = sim.get_state()
    sim.check()
    for i, c in enumerate(cases):
        assert host(st["agent"][i, :3]).tolist() == c["post_pos"] + [c["post_dir"]], c["name"]
        assert host(st["inventory"][i]).tolist() == c["post_inv"], c["name"]
        assert host(st["grid"][i]).tolist() == c["post_grid"], c["name"]


@pytest.mark.parametrize("W", [8, 12])
def test_random_step_kats(golden, W):
    g = golden("kat_step.npz")
    p = f"w{W}_"
    n = len(g[p + "action"])
    sim = sim_with_pool(world_for(W, 3), n, g[p + "pre_grid"])
    set_states(sim, np.arange(n), g[p + "pre_agent"], g[p + "pre_inv"])
    obs = sim.empty_obs(n)
    sim.observe(obs=obs, n=n)
    np.testing.assert_array_equal(host(obs), g[p + "features"].astype(np.float32))
    sat = torch.empty(n, dtype=torch.int8, device="cuda")
    for t in range(g[p + "satisfies"].shape[1]):
        sim.observe(tasks=torch.full((n,), t, dtype=torch.int32, device="cuda"), sat=sat, n=n)
        np.testing.assert_array_equal(host(sat), g[p + "satisfies"][:, t], err_msg=f"task {t}")
    sim.transition(torch.as_tensor(g[p + "action"].astype(np.int32), device="cuda"))
    st = sim.get_state()
    sim.check()
    np.testing.assert_array_equal(host(st["agent"][:, :3]), g[p + "post_agent"])
    np.testing.assert_array_equal(host(st["inventory"]), g[p + "post_inv"])
    np.testing.assert_array_equal(host(st["grid"]), g[p + "post_grid"])


def test_copy_on_step_keeps_old_state(golden):
    g = golden("kat_step.npz")
    sim = sim_with_pool("craft_medium_12x12", 4, g["w12_pre_grid"][:2])
    set_states(sim, [0, 1, 0, 1], g["w12_pre_agent"][[0, 1, 0, 1]], g["w12_pre_inv"][[0, 1, 0, 1]])
    before = {k: host(v) for k, v in sim.get_state().items()}
    src = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    dst = torch.tensor([2, 3], dtype=torch.int32, device="cuda")
    acts = torch.as_tensor(g["w12_action"][:2].astype(np.int32), device="cuda")
    sim.transition(acts, src, dst)
    after = {k: host(v) for k, v in sim.get_state().items()}
    sim.check()
    for k in before:
        np.testing.assert_array_equal(after[k][:2], before[k][:2])
    np.testing.assert_array_equal(after["agent"][2:, :3], g["w12_post_agent"][:2])
    np.testing.assert_array_equal(after["grid"][2:], g["w12_post_grid"][:2])


@pytest.mark.parametrize("split", ["dev", "test"])
def test_replay_reference_demonstrations_on_gpu(golden, split):
    """The reference's committed demonstrations, replayed on the GPU: the GPU
    teacher reproduces every action and every episode ends satisfied."""
    g = golden("devtest.npz")
    n = len(g[f"{split}_task"])
    sim = sim_with_pool("craft_medium", n, g[f"{split}_grids"])
    pos = g[f"{split}_pos"].astype(np.int32)
    agent = np.concatenate([pos, np.zeros((n, 1), np.int32)], 1)
    set_states(sim, g[f"{split}_world"], agent, np.zeros((n, 1)), task=g[f"{split}_task"])
    acts = g[f"{split}_actions"].astype(np.int32)
    for t in range(acts.shape[1]):
        ta, _ = sim.teacher(n=n)
        ta = host(ta)
        live = acts[:, t] >= 0
        np.testing.assert_array_equal(ta[live], acts[live, t], err_msg=f"t={t}")
        step = np.where(live & (acts[:, t] != N.STOP), acts[:, t], -1).astype(np.int32)
        sim.transition(torch.as_tensor(step, device="cuda"))
    sat = torch.empty(n, dtype=torch.int8, device="cuda")
    sim.observe(sat=sat, n=n)
    sim.check()
    assert (host(sat) == 1).all()


def test_teacher_12x12(golden):
    g = golden("teacher_12x12.npz")
    n = len(g["grid"])
    sim = sim_with_pool("craft_medium_12x12", n, g["grid"])
    set_states(sim, np.arange(n), g["agent"], g["inv"])
    plen = torch.empty(n, dtype=torch.int32, device="cuda")
    n_tasks = g["action"].shape[1]
    for t in range(n_tasks):
        tasks = torch.full((n,), t, dtype=torch.int32, device="cuda")
        a, _ = sim.teacher(tasks=tasks, path_len_out=plen, n=n)
        np.testing.assert_array_equal(host(a), g["action"][:, t], err_msg=f"task {t}")
        ref = g["path_len"][:, t]
        if (ref != -3).all():
            np.testing.assert_array_equal(host(plen), ref, err_msg=f"task {t}")
        try:
            sim.check()
        except N.CraftError as e:
            assert e.status == N.ETEACHER and (g["action"][:, t] == -2).any()


@pytest.mark.parametrize("window", [3, 5])
def test_rollout_fixture(golden, window):
    g = golden(f"rollout_12x12_w{window}.npz")
    E = g["spec"].shape[0]
    sim = sim_with_pool(world_for(12, window), E, g["pool"])
    sp = g["spec"]
    sim.reset(sp[:, 0], sp[:, 1], sp[:, 2], sp[:, 3], sp[:, 4])
    obs = sim.empty_obs()
    rew = torch.empty(E, dtype=torch.float32, device="cuda")
    done = torch.empty(E, dtype=torch.uint8, device="cuda")
    succ = torch.empty(E, dtype=torch.int8, device="cuda")
    ticks = list(g["obs_ticks"])
    seed = int(g["seed"][0])
    for t in range(g["done"].shape[0]):
        sim.step(seed=seed, tick=t, obs=obs, reward=rew, done=done, success=succ)
        st = sim.get_state()
        np.testing.assert_array_equal(host(done), g["done"][t])
        np.testing.assert_array_equal(host(succ), g["success"][t])
        np.testing.assert_array_equal(host(rew), g["reward"][t].astype(np.float32))
        np.testing.assert_array_equal(host(st["agent"]), g["agent"][t])
        np.testing.assert_array_equal(host(st["inventory"]), g["inv"][t])
        np.testing.assert_array_equal(host(st["grid"]), g["grid"][t])
        if t in ticks:
            np.testing.assert_array_equal(host(obs), g["obs"][ticks.index(t)].astype(np.float32))
    sim.check()


def oracle_from_sim_specs(oracle_mod, cfg, pool, specs):
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*specs)
    return o, envs


@pytest.mark.parametrize("window,autoreset,policy", [(3, True, False), (5, True, False),
                                                     (3, False, True), (5, True, True)])
def test_lockstep_vs_oracle_4096(oracle_mod, window, autoreset, policy):
    """Config 2: 4096 12x12 envs, 100 ticks, bit-exact against the CPU oracle
    every tick (observation, done, success, reward; full state every 10 ticks)."""
    world = world_for(12, window)
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    n = 4096
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=11, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.reset(*specs)
    o, envs = oracle_from_sim_specs(oracle_mod, cfg, pool, specs)
    obs = sim.empty_obs()
    rew = torch.empty(n, dtype=torch.float32, device="cuda")
    done = torch.empty(n, dtype=torch.uint8, device="cuda")
    succ = torch.empty(n, dtype=torch.int8, device="cuda")
    rng = np.random.RandomState(window)
    stats = np.zeros(3, dtype=np.int64)
    T = 100 if autoreset else 50
    for t in range(T):
        acts = rng.randint(0, 6, size=n).astype(np.int32) if policy else None
        sim.step(None if acts is None else torch.as_tensor(acts, device="cuda"), seed=5, tick=t,
                 autoreset=autoreset, obs=obs, reward=rew, done=done, success=succ)
        rc, oobs, orew, odone, osucc = o.batch_tick(envs, 0, acts, 5, t, autoreset, True, stats)
        assert rc == 0
        np.testing.assert_array_equal(host(done), odone, err_msg=f"t={t}")
        np.testing.assert_array_equal(host(succ), osucc, err_msg=f"t={t}")
        np.testing.assert_array_equal(host(rew), orew, err_msg=f"t={t}")
        np.testing.assert_array_equal(host(obs), oobs, err_msg=f"t={t}")
        if t % 10 == 9:
            st = sim.get_state()
            np.testing.assert_array_equal(host(st["agent"]),
                                          np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1))
            np.testing.assert_array_equal(host(st["inventory"]), envs["inv"][:, :cfg.n_kinds])
            np.testing.assert_array_equal(host(st["grid"]), envs["grid"][:, :144])
    np.testing.assert_array_equal(host(sim.stats()), stats)
    sim.check()


def test_full_size_properties_and_sharding(oracle_mod):
    """Config 3 sizes (65536 envs, 12x12, w=3): determinism, shard invariance
    (two half-size sims with env_id_base == one full sim), episode accounting,
    observation invariants, and an oracle spot-check of 256 random envs."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 1024)
    n, T = 65536, 30
    tasks = [t.id for t in tm.dataset_tasks()]
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=0, task_ids=tasks)

    def run(base, count):
        sp = synthetic_specs(pool, 12, 12, count, base, seed=0, task_ids=tasks)
        sim = CraftSim(world, n_envs=count, device=0, env_id_base=base, pool_capacity=1024)
        sim.load_pool(pool)
        sim.reset(*sp)
        obs = sim.empty_obs()
        done = torch.empty(count, dtype=torch.uint8, device="cuda")
        total_done = torch.zeros(count, dtype=torch.int64, device="cuda")
        for t in range(T):
            sim.step(seed=1, tick=t, obs=obs, done=done)
            total_done += done
        st = sim.get_state()
        sim.check()
        return sim, obs, total_done, st

    sim, obs, total_done, st = run(0, n)
    _, obs2, _, _ = run(0, n)
    assert torch.equal(obs, obs2)
    _, oa, _, sa = run(0, n // 2)
    _, ob, _, sb = run(n // 2, n // 2)
    assert torch.equal(torch.cat([oa, ob]), obs)
    for k in st:
        assert torch.equal(torch.cat([sa[k], sb[k]]), st[k]), k
    s = host(sim.stats())
    assert s[2] == n * T and s[1] == int(total_done.sum())
    o = host(obs)
    L = 9 * 21
    assert (o[:, -1] == 0).all()
    assert (o[:, 2 * L + 21:2 * L + 25].sum(1) == 1).all()
    assert (o[:, :L].reshape(n, 9, 21).sum(2) <= 1).all()
    # oracle spot-check on random global ids
    ids = np.random.RandomState(0).choice(n, 256, replace=False)
    oc = oracle_mod.Oracle(cfg, pool)
    for gid in ids:
        env = oc.init_envs(*[a[gid:gid + 1] for a in specs])
        for t in range(T):
            rc, oobs, _, _, _ = oc.batch_tick(env, int(gid), None, 1, t, True)
        np.testing.assert_array_equal(o[gid], oobs[0], err_msg=str(gid))


def test_teacher_at_scale_vs_oracle(oracle_mod):
    """Config 5: the batched GPU teacher on 65536 envs mid-rollout, checked
    against the literal per-target BFS oracle on 2048 of them; the quad-lane
    variant (small batches) gives the same answers as the single-lane one."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 512)
    n = 65536
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=4, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.reset(*specs)
    for t in range(7):
        sim.step(seed=9, tick=t)
    plen = torch.empty(n, dtype=torch.int32, device="cuda")
    act, _ = sim.teacher(path_len_out=plen)              # one lane per query (large batch)
    half = torch.arange(n // 2, dtype=torch.int32, device="cuda")
    plen_q = torch.empty(n // 2, dtype=torch.int32, device="cuda")
    act_q, _ = sim.teacher(slots=half, path_len_out=plen_q)   # four lanes per query (small batch)
    st = {k: host(v) for k, v in sim.get_state().items()}
    sim.check()
    act, plen = host(act), host(plen)
    assert np.array_equal(host(act_q), act[:n // 2]) and np.array_equal(host(plen_q), plen[:n // 2])
    o = oracle_mod.Oracle(cfg, pool)
    for i in np.random.RandomState(1).choice(n, 2048, replace=False):
        x, y, d, _ = st["agent"][i]
        env = o.env(st["grid"][i], x, y, d, st["inventory"][i])
        rc, a = o.teacher(env, int(specs[4][i]))
        assert rc == 0 and a == act[i], i
        rc, _, ln = o.closest_resource(env, cfg.task[int(specs[4][i])].arg_kind)
        assert rc == 0 and ln == plen[i], i


def test_bad_action_latches_error():
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 8)
    sim = sim_with_pool(world, 64, pool)
    sim.reset(*synthetic_specs(pool, 12, 12, 64, 0, seed=0, task_ids=[12]))
    acts = torch.zeros(64, dtype=torch.int32, device="cuda")
    acts[17] = 9
    assert sim.error_word().cpu().tolist() == [0, 0, 0, 0]
    sim.step(acts, tick=0)
    w = sim.error_word().cpu().tolist()   # queued on the stream, read without craft_sim_check
    assert w[0] == N.EBADACTION and w[2] == 17
    with pytest.raises(N.CraftError) as e:
        sim.check()
    assert e.value.status == N.EBADACTION
    sim.check()   # cleared
    assert sim.error_word().cpu().tolist()[0] == 0


@pytest.mark.parametrize("border", ["open", "wood", "water", "workshop0", "boundary"])
def test_pool_border_ring(border):
    """craft_pool_load refuses a border cell that is empty, clearable by USE (a grabbable kind,
    water, stone) or a task's target (a workshop, wood), which the band-layout teacher BFS and
    the kernels cannot see or would walk past; the boundary ring of every make_data.py world
    (make_data.py:108-112) loads."""
    sim = CraftSim("craft_medium", n_envs=8, device=0, pool_capacity=2)
    idx = sim.cookbook.index
    g = np.zeros((8, 8), dtype=np.uint8)
    g[0, :] = g[-1, :] = g[:, 0] = g[:, -1] = idx["boundary"]
    if border != "boundary":
        g[0, 3] = 0 if border == "open" else idx[border]
    if border == "boundary":
        sim.load_pool(g.reshape(1, 64))
        return
    with pytest.raises(N.CraftError) as e:
        sim.load_pool(g.reshape(1, 64))
    assert e.value.status == N.EINVARIANT


@pytest.mark.parametrize("window", [3, 5])
def test_tuning_does_not_change_results(window):
    """craft_sim_tune changes only the kernel geometry: every tile size and
    residency cap gives bit-identical observations, states and statistics; the
    bf16 and u8 observation formats hold exactly the same values."""
    world = world_for(12, window)
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 128)
    n = 5000   # not a multiple of any tile: exercises the partial last tile
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    ref = None
    for tile, cap, pol, fmt in [(64, 0, 0, "f32"), (32, 0, 1, "f32"), (16, 0, 2, "f32"),
                                (16, 6, 0, "f32"), (32, 4, 2, "f32"), (64, 3, 1, "f32"),
                                (64, 0, 1, "bf16"), (16, 0, 0, "bf16"), (64, 0, 1, "u8"),
                                (32, 0, 2, "u8")]:
        sim = sim_with_pool(world, n, pool)
        sim.tune(tile, cap, pol)
        sim.set_obs_format(fmt)
        obs = sim.empty_obs()
        assert obs.dtype == {"f32": torch.float32, "bf16": torch.bfloat16, "u8": torch.uint8}[fmt]
        sim.reset(*specs, obs=obs)
        outs = [host(obs.float())]
        for t in range(12):
            sim.step(seed=4, tick=t, obs=obs)
            outs.append(host(obs.float()))
        o2 = sim.empty_obs()
        sim.observe(obs=o2, n=n)
        outs.append(host(o2.float()))
        st = {k: host(v) for k, v in sim.get_state().items()}
        stats = host(sim.stats())
        sim.check()
        if ref is None:
            ref = (outs, st, stats)
        else:
            for a, b in zip(outs, ref[0]):
                np.testing.assert_array_equal(a, b, err_msg=f"tile {tile} cap {cap} {fmt}")
            for k in st:
                np.testing.assert_array_equal(st[k], ref[1][k])
            np.testing.assert_array_equal(stats, ref[2])


@pytest.mark.parametrize("world,W", [("craft_medium", 8), ("craft_large", 10), ("craft_16x16_w7", 16)])
def test_lockstep_other_geometries(oracle_mod, world, W):
    """Other grid sizes / windows (row strides, pooled-window clipping, the
    w=5 and w=7 kernels, 16x16 = 256 cells): 1024 envs x 60 ticks bit-exact."""
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 7, 64)
    n = 1024
    specs = synthetic_specs(pool, W, W, n, 0, seed=5, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.reset(*specs)
    o, envs = oracle_from_sim_specs(oracle_mod, cfg, pool, specs)
    obs = sim.empty_obs()
    done = torch.empty(n, dtype=torch.uint8, device="cuda")
    succ = torch.empty(n, dtype=torch.int8, device="cuda")
    for t in range(60):
        sim.step(seed=8, tick=t, obs=obs, done=done, success=succ)
        rc, oobs, _, odone, osucc = o.batch_tick(envs, 0, None, 8, t, True, True)
        np.testing.assert_array_equal(host(obs), oobs, err_msg=f"t={t}")
        np.testing.assert_array_equal(host(done), odone)
        np.testing.assert_array_equal(host(succ), osucc)
    st = sim.get_state()
    np.testing.assert_array_equal(host(st["grid"]), envs["grid"][:, :W * W])
    np.testing.assert_array_equal(host(st["inventory"]), envs["inv"][:, :cfg.n_kinds])
    if 4 * W * W <= 1000:
        act, _ = sim.teacher()
        act = host(act)
        for i in range(0, n, 3):
            rc, a = o.teacher(envs[i:i + 1], int(specs[4][i]))
            assert (a if rc == 0 else -2) == act[i], i
    sim.check()


@pytest.mark.parametrize("world,W,tile,fmt,autoreset,given,chunk,R,threads", [
    ("craft_medium_12x12", 12, 0, "f32", True, False, 0, 3, 0),
    ("craft_medium_12x12", 12, 0, "f32", True, False, 0, 16, 256),
    ("craft_medium_12x12", 12, 0, "f32", True, False, 1, 3, 0),
    ("craft_medium_12x12", 12, 0, "f32", True, False, 1, 16, 0),
    ("craft_medium_12x12", 12, 0, "bf16", True, False, 2, 16, 256),
    ("craft_medium_12x12", 12, 16, "bf16", True, True, 2, 3, 0),
    ("craft_medium_12x12", 12, 32, "u8", False, True, 3, 16, 0),
    ("craft_medium_12x12", 12, 32, "f32", True, True, 0, 16, 128),
    ("craft_medium_12x12", 12, 32, "f32", True, False, 1, 3, 512),
    ("craft_medium_12x12", 12, 16, "bf16", False, True, 0, 16, 512),
    ("craft_medium_12x12", 12, 16, "f32", True, False, 0, 16, 256),
    ("craft_medium_12x12", 12, 16, "f32", True, False, 0, 16, 320),
    ("craft_medium_12x12", 12, 16, "u8", True, True, 2, 3, 384),
    ("craft_medium_12x12", 12, 32, "bf16", True, False, 1, 16, 320),
    ("craft_medium_12x12", 12, 32, "f32", False, False, 0, 3, 384),
    ("craft_medium_12x12_w5", 12, 16, "f32", True, False, 0, 3, 320),
    ("craft_16x16_w7", 16, 16, "f32", True, True, 3, 16, 384),
    ("craft_medium", 8, 16, "f32", True, False, 1, 9, 320),
    ("craft_medium_12x12_w5", 12, 0, "f32", True, False, 2, 3, 0),
    ("craft_medium_12x12_w5", 12, 0, "u8", True, False, 0, 3, 128),
    ("craft_16x16_w7", 16, 0, "f32", False, False, 0, 3, 0),
    ("craft_16x16_w7", 16, 32, "f32", True, False, 0, 3, 256),
    ("craft_medium", 8, 64, "f32", True, True, 1, 9, 0),
    ("craft_medium", 8, 64, "f32", True, True, 0, 9, 256),
    # chunk -1: the continuous pipeline (prefetched tile switches, deferred outputs)
    ("craft_medium_12x12", 12, 0, "f32", True, False, -1, 3, 0),
    ("craft_medium_12x12", 12, 0, "bf16", False, True, -1, 16, 0),
    ("craft_medium_12x12", 12, 0, "u8", True, True, -1, 9, 0)])
def test_multi_tick_rollout_equals_steps(world, W, tile, fmt, autoreset, given, chunk, R, threads):
    """craft_rollout(K ticks) == K craft_step calls: observation / reward / done /
    success rings, final states and episode statistics, bit for bit; several
    launches in a row (state written back and picked up again).  Small work
    units (chunk) hand each tile between workgroups several times per launch.
    Every workgroup width (2 to 16 threads per env) is covered, and the
    split-producer kernel (320 / 384 / 512 threads on 16- and 32-env tiles).
    With a ring (R = 3) shorter than a launch, slots are rewritten by later
    units that may run on another XCD (full release between units); with
    R >= the launch, only the state is handed over (write-through, no fence)."""
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    n = 5000                                   # a partial last tile
    specs = synthetic_specs(pool, W, W, n, 0, seed=3, task_ids=[t.id for t in tm.dataset_tasks()])
    chunks = [5, 1, 9]
    T = sum(chunks)
    rng = np.random.RandomState(4)
    acts = torch.as_tensor(rng.randint(0, 6, size=(T, n)).astype(np.int32), device="cuda")
    sims = []
    for _ in range(2):
        sim = sim_with_pool(world, n, pool)
        sim.tune(tile, 0, 1)
        sim.tune_rollout(chunk, threads)
        sim.set_obs_format(fmt)
        sim.reset(*specs)
        sims.append(sim)
    a, b = sims
    ring = lambda shape, dt: torch.zeros((R,) + shape, dtype=dt, device="cuda")  # noqa: E731
    oa, ob = ring((n, a.n_features), a.obs_dtype), ring((n, a.n_features), a.obs_dtype)
    outs = {k: (ring((n,), dt), ring((n,), dt)) for k, dt in
            (("reward", torch.float32), ("done", torch.uint8), ("success", torch.int8))}
    t0 = 0
    for K in chunks:
        a.rollout(K, seed=11, tick0=t0, actions=acts[t0:t0 + K] if given else None,
                  autoreset=autoreset, obs=oa, reward=outs["reward"][0], done=outs["done"][0],
                  success=outs["success"][0])
        for k in range(K):
            t = t0 + k
            b.step(acts[t] if given else None, seed=11, tick=t, autoreset=autoreset, obs=ob[t % R],
                   reward=outs["reward"][1][t % R], done=outs["done"][1][t % R],
                   success=outs["success"][1][t % R])
        t0 += K
        np.testing.assert_array_equal(host(oa.float()), host(ob.float()))
        for k, (x, y) in outs.items():
            np.testing.assert_array_equal(host(x), host(y), err_msg=k)
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            np.testing.assert_array_equal(host(sa[k]), host(sb[k]), err_msg=k)
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))
    a.check()
    b.check()
    assert host(b.stats())[2] > 0


def test_empty_and_single_env_calls(gpu):
    """Zero-length calls are no-ops (no launch, no error); a one-env simulator
    runs every entry point."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 4)
    sim = sim_with_pool(world, 1, pool)
    e32 = torch.empty(0, dtype=torch.int32, device="cuda")
    sim.teacher(slots=e32)
    sim.observe(slots=e32, obs=torch.empty((0, sim.n_features), device="cuda"))
    sim.transition(e32, src=e32, dst=e32)
    sim.rollout(0, obs=torch.empty((1, 1, sim.n_features), device="cuda"))
    sim.generate_pool(0)
    sim.get_state(slots=e32)
    sim.check()
    specs = synthetic_specs(pool, 12, 12, 1, 0, seed=0, task_ids=[t.id for t in tm.dataset_tasks()])
    obs = sim.empty_obs()
    sim.reset(*specs, obs=obs)
    for t in range(45):                                    # crosses an episode boundary
        sim.step(seed=1, tick=t, obs=obs)
    ring = torch.empty((4, 1, sim.n_features), device="cuda")
    sim.rollout(8, seed=1, tick0=45, obs=ring)
    act, _ = sim.teacher()
    assert int(act[0]) in range(6)
    stats = host(sim.stats())
    assert stats[2] == 53 and stats[1] >= 1
    sim.check()


@pytest.mark.parametrize("launches,R,chunk", [
    ((32,), 16, 0),          # the bench's default launch
    ((20, 13), 16, 0),       # the driver's --steps 20 launch, then a ragged one
    ((20, 3, 32), 16, -1),   # the continuous pipeline, incl. launches shorter than its prefetch
    ((32,), 32, 4),          # chunked units, ring >= launch: write-through state hand-off
    ((24,), 8, 3)])          # chunked units, ring < launch: full release between units
def test_bench_rollout_equals_steps_at_full_size(launches, R, chunk, oracle_mod):
    """BASELINE's single-GPU size (65536 envs, 12x12 craft_medium, w=3), the
    bench's own path: craft_rollout launches into a ring with the default
    workgroup shape, against one craft_step launch per tick.  Every
    observation, reward, done and success and the final states are identical
    (compared on the device), and the episode counters agree.  The chunked
    cases hand every tile between workgroups (possibly on other XCDs) several
    times per launch, at full size.  The rollout ring is also checked directly
    against the CPU oracle: 256 random global ids, every tick the ring keeps, and
    their agent states after each launch."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 1024)
    n = 65536
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=0, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.tune_rollout(chunk, 0)
    a.reset(*specs)
    b.reset(*specs)
    F = a.n_features
    ring = torch.empty((R, n, F), dtype=torch.float32, device="cuda")
    outs = {k: torch.empty((R, n), dtype=dt, device="cuda") for k, dt in
            (("reward", torch.float32), ("done", torch.uint8), ("success", torch.int8))}
    obs = torch.empty((n, F), dtype=torch.float32, device="cuda")
    one = {k: torch.empty(n, dtype=v.dtype, device="cuda") for k, v in outs.items()}
    # the oracle on a sample of global ids, one env per call (its hashed actions are keyed by id)
    gids = np.sort(np.random.RandomState(sum(launches) + R).choice(n, 256, replace=False))
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*[np.asarray(s)[gids] for s in specs])
    gid_d = torch.as_tensor(gids, device="cuda")
    t0 = 0
    for K in launches:
        a.rollout(K, seed=5, tick0=t0, obs=ring, **outs)
        ref = []
        for t in range(t0, t0 + K):
            b.step(seed=5, tick=t, obs=obs, **one)
            if t >= t0 + K - R:                  # the ring keeps the launch's last R ticks
                assert torch.equal(ring[t % R], obs), t
                for k in outs:
                    assert torch.equal(outs[k][t % R], one[k]), (k, t)
            step = [o.batch_tick(envs[j:j + 1], int(g), None, 5, t, True) for j, g in enumerate(gids)]
            assert all(s[0] == 0 for s in step)
            ref.append([np.concatenate([s[m] for s in step]) for m in range(1, 5)])
        for t in range(max(t0, t0 + K - R), t0 + K):
            r_obs, r_rew, r_done, r_succ = ref[t - t0]
            np.testing.assert_array_equal(ring[t % R][gid_d].cpu().numpy(), r_obs, err_msg=f"obs {t}")
            np.testing.assert_array_equal(outs["reward"][t % R][gid_d].cpu().numpy(), r_rew)
            np.testing.assert_array_equal(outs["done"][t % R][gid_d].cpu().numpy(), r_done)
            np.testing.assert_array_equal(outs["success"][t % R][gid_d].cpu().numpy(), r_succ)
        t0 += K
        sa, sb = a.get_state(), b.get_state()
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
        np.testing.assert_array_equal(sa["agent"][gid_d].cpu().numpy(),
                                      np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1))
        np.testing.assert_array_equal(sa["inventory"][gid_d].cpu().numpy(), envs["inv"][:, :cfg.n_kinds])
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))
    assert host(a.stats())[2] == n * sum(launches)
    a.check()
    b.check()


def test_rollout_fast_path_revalidates_resized_rings():
    """rollout() skips re-checking output rings it has seen unchanged; a ring resized
    (or re-pointed) in place since the last call is checked again and refused."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 16)
    n = 256
    sim = sim_with_pool(world, n, pool)
    sim.reset(*synthetic_specs(pool, 12, 12, n, 0, seed=1, task_ids=[t.id for t in tm.dataset_tasks()]))
    ring = torch.empty((4, n, sim.n_features), dtype=torch.float32, device="cuda")
    done = torch.empty((4, n), dtype=torch.uint8, device="cuda")
    sim.rollout(3, tick0=0, obs=ring, done=done)
    sim.rollout(3, tick0=3, obs=ring, done=done)          # the cached path
    ring.resize_(4, n // 2, sim.n_features)
    with pytest.raises(ValueError):
        sim.rollout(3, tick0=6, obs=ring, done=done)
    # re-strided in place to a non-contiguous view of the same storage: refused
    ring2 = torch.empty((4, n, sim.n_features), dtype=torch.float32, device="cuda")
    sim.rollout(3, tick0=6, obs=ring2, done=done)
    ring2.as_strided_((4, n, sim.n_features), (n * sim.n_features, 1, n))
    with pytest.raises(ValueError):
        sim.rollout(3, tick0=9, obs=ring2, done=done)
    # the cache holds no reference: a dropped ring is freed
    import weakref
    ring3 = torch.empty((4, n, sim.n_features), dtype=torch.float32, device="cuda")
    sim.rollout(3, tick0=9, obs=ring3, done=done)
    r = weakref.ref(ring3)
    del ring3
    assert r() is None
    sim.check()
    sim.close()
    assert sim._rollout_cache is None


def test_rollout_shape_reports_the_launched_kernel():
    """craft_sim_rollout_shape names what craft_rollout launches: the 3x3 default is the split
    kernel on 32-env tiles x 512 threads; 64-env tiles run 256 or 512 threads (a request for
    384 runs, and is reported as, 512); smaller tiles run 128, 256 or the split kernel at
    320 / 384 / 512."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 16)
    sim = sim_with_pool(world, 256, pool)
    assert sim.rollout_shape() == (32, 512, True)
    sim.tune(64, 0, 2)
    for req, want in ((256, (64, 256, False)), (384, (64, 512, False)), (512, (64, 512, False))):
        sim.tune_rollout(0, req)
        assert sim.rollout_shape() == want, req
    sim.tune(32, 0, 2)
    for req, want in ((128, (32, 128, False)), (256, (32, 256, False)), (320, (32, 320, True)),
                      (384, (32, 384, True))):
        sim.tune_rollout(0, req)
        assert sim.rollout_shape() == want, req


def test_rollout_graph_replay_and_eager_interleave():
    """A craft_rollout captured into a HIP graph (torch.cuda.graph) replays correctly any number
    of times, interleaved with eager launches of the same handle: every replay and launch equals
    the same launch run eagerly, and the episode counters grow by one launch's env-steps each
    time (the captured launch has its own work-unit counter, zeroed inside the graph)."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    n, K, R = 4096, 8, 8
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    ra, rb = (torch.empty((R, n, a.n_features), dtype=torch.float32, device="cuda") for _ in range(2))
    da, db = (torch.empty((R, n), dtype=torch.uint8, device="cuda") for _ in range(2))
    for s in (a, b):
        s.reset(*specs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.rollout(K, seed=4, tick0=0, obs=rb, done=db)
    for it in range(3):
        a.rollout(K, seed=4, tick0=0, obs=ra, done=da)        # eager reference
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(ra, rb) and torch.equal(da, db), it
        if it == 1:                                           # an eager launch on b in between
            a.rollout(K, seed=4, tick0=K, obs=ra, done=da)
            b.rollout(K, seed=4, tick0=K, obs=rb, done=db)
            assert torch.equal(ra, rb) and torch.equal(da, db)
    sa, sb = host(a.stats()), host(b.stats())
    np.testing.assert_array_equal(sa, sb)
    assert sb[2] == 4 * K * n                                 # env-steps: every env every tick
    for k, v in a.get_state().items():
        assert torch.equal(v, b.get_state()[k]), k
    a.check()
    b.check()
