"""Batched do_rollout (psketch_amd.rollout) against the reference's
ImitationTrainer.do_rollout (tests/golden/imitation_rollout.npz) and the oracle
restatement (oracle/rollout_oracle.py) at larger sizes."""
import numpy as np
import pytest
import torch

from tests.helpers import make_tables

pytestmark = pytest.mark.gpu


def torch_policy(W, bias, device):
    """fake_policy of make_golden.py on the device: exact (small integers in float64)."""
    Wd = torch.as_tensor(np.asarray(W, dtype=np.float64), device=device)
    bd = torch.as_tensor(np.asarray(bias, dtype=np.float64), device=device)

    def act(obs, t):
        return (obs.double() @ Wd[t % Wd.shape[0]] * 8 + bd).argmax(dim=1).to(torch.int32)
    return act


@pytest.mark.parametrize("case", ["dev8", "w12"])
@pytest.mark.parametrize("mode,fused,lookahead", [("train", True, False), ("train", False, False),
                                                  ("eval", True, False), ("train", True, True),
                                                  ("eval", True, True)])
def test_do_rollout_matches_reference_fixture(golden, gpu, case, mode, fused, lookahead):
    """fused: the teacher labels come from each step's launch (craft_step_teach); else from
    craft_teacher on a side stream.  lookahead: tick t + 1 is queued before tick t's all(done)
    flag is read; the result, every receive() call included, must not change."""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout
    fx = golden("imitation_rollout.npz")
    world = {"dev8": "craft_medium", "w12": "craft_medium_12x12"}[case]
    pool, spec = fx[f"{case}_pool"], fx[f"{case}_spec"]
    key = f"{case}_{mode}"
    sim = CraftSim(world, n_envs=len(spec), device=gpu.index, pool_capacity=len(pool))
    sim.load_pool(pool)
    received = []
    info = do_rollout(sim, tuple(spec.T), torch_policy(fx[f"{case}_W"], fx[f"{case}_bias"], gpu),
                      mode == "eval", behavior_clone=fx[key + "_bc"],
                      receive=lambda r: received.append(r.cpu().numpy()), fused_teacher=fused,
                      lookahead=lookahead)
    ref = info.to_reference()
    A = fx[key + "_action_seqs"]
    assert ref["action_seqs"] == [[int(a) for a in row if a >= 0] for row in A]
    assert ref["success"] == [bool(s) for s in fx[key + "_success"]]
    assert ref["distances"] == fx[key + "_distances"].tolist()
    assert [ref["num_interactions"], ref["num_steps"]] == fx[key + "_counts"].tolist()
    R = fx[key + "_received"]
    assert np.array_equal(np.asarray(received, dtype=np.int8).reshape(R.shape), R)


@pytest.mark.parametrize("world,n", [("craft_medium_12x12", 2048), ("craft_medium_12x12_w5", 512)])
def test_do_rollout_vs_oracle(golden, gpu, oracle_mod, world, n):
    """Random policy-mix rollouts on sampled 12x12 worlds, with every observation the
    student saw (keep_obs) checked against the oracle's features()."""
    from oracle import rollout_oracle
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout
    from psketch_amd.sim import synthetic_specs
    sc = golden("scenarios_seed123.npz")
    pool = sc["w12_grids"]
    _, _, tm, cfg = make_tables(world)
    tasks = [t.id for t in tm.dataset_tasks()]
    spec = np.stack(synthetic_specs(pool, 12, 12, n, seed=5, task_ids=tasks), axis=1)
    spec[:, 3] = np.arange(n) % 4                   # non-default initial directions too
    rng = np.random.RandomState(9)
    bc = rng.binomial(1, 0.5, size=n)
    W = rng.randint(-3, 4, size=(3, cfg.n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, -40])
    seen = []

    def act_cpu(obs, t):
        seen.append(obs.copy())
        return rollout_oracle.fake_policy(W, bias)(obs, t)

    expect = rollout_oracle.do_rollout(oracle_mod.Oracle(cfg, pool), spec, act_cpu, False,
                                       bc_mask=bc)
    sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    sim.load_pool(pool)
    received = []
    info = do_rollout(sim, tuple(spec.T), torch_policy(W, bias, gpu), False, behavior_clone=bc,
                      receive=lambda r: received.append(r.cpu().numpy()), keep_obs=True)
    got = info.to_reference()
    for k in ["action_seqs", "success", "distances", "num_interactions", "num_steps"]:
        assert got[k] == expect[k], k
    assert np.array_equal(np.asarray(received), np.asarray(expect["received"]))
    assert info.ticks == len(seen)
    obs = info.obs.cpu().numpy()
    for t in range(info.ticks):
        assert np.array_equal(obs[t], seen[t]), t


def test_imitation_rollout_replays_dataset(golden, gpu):
    """Dataset batches (data/dataset.py) through ImitationRollout in eval mode, the
    student replaying the reference's demonstrations: every episode succeeds, the
    recorded sequences are the demonstrations, get-task distances are 0."""
    from psketch_amd.dataset import Dataset
    from psketch_amd.rollout import ImitationRollout
    from tests.test_host import devtest_as_json
    fx = golden("devtest.npz")
    _, cb, tm, _ = make_tables("craft_medium")
    ds = Dataset(devtest_as_json(fx, "dev", tm, cb.n_kinds), "dev", tm,
                 random=np.random.RandomState(1), batch_size=500)
    runner = ImitationRollout("craft_medium", ds.pool_array(), device=gpu.index)
    total = 0
    for batch in ds.iterate_batches():
        A = np.full((40, len(batch)), 5, dtype=np.int32)
        for i, it in enumerate(batch):
            A[:len(it["ref_actions"]), i] = it["ref_actions"]
        Ad = torch.as_tensor(A, device=gpu)
        info = runner.do_rollout(batch, lambda obs, t: Ad[t], is_eval=True)
        ref = info.to_reference()
        assert ref["action_seqs"] == [list(it["ref_actions"]) for it in batch]
        assert all(ref["success"])
        assert ref["distances"] == [0] * sum(it["task"].goal_name == "get" for it in batch)
        total += len(batch)
    assert total == len(ds)
    # last batch has a different size: a second simulator was created for it
    assert len(runner._sims) == 2


@pytest.mark.parametrize("is_eval,keep_obs,bc_rate,stop_at", [(False, False, 0.0, 6),
                                                              (True, True, 0.0, 9),
                                                              (False, False, 0.5, None)])
def test_lookahead_equals_sync_loop_full_size(gpu, is_eval, keep_obs, bc_rate, stop_at):
    """Config 3/5 size (65,536 envs): the lookahead loop gives the synchronous loop's result
    bit for bit: action_seqs, success, distances, counters, every receive() call, ticks and
    (keep_obs) every observation.  With stop_at the policy answers STOP from that tick on, so the
    loop ends before the timer and the discarded speculative tick is exercised; with cloning the
    teacher's episodes run to the timer."""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout
    from psketch_amd.sim import sample_scenarios, synthetic_specs
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    n = 65536
    spec = synthetic_specs(pool, 12, 12, n, seed=3, task_ids=[t.id for t in tm.dataset_tasks()])
    rng = np.random.RandomState(4)
    W = rng.randint(-3, 4, size=(4, cfg.n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, 0])
    bc = rng.binomial(1, bc_rate, size=n)
    base = torch_policy(W, bias, gpu)

    def act(obs, t):
        a = base(obs, t)
        return torch.full_like(a, 5) if stop_at is not None and t >= stop_at else a

    outs = []
    for lookahead in (False, True):
        sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
        sim.load_pool(pool)
        received = []
        info = do_rollout(sim, spec, act, is_eval, behavior_clone=bc,
                          receive=lambda r: received.append(r.cpu().numpy()), keep_obs=keep_obs,
                          lookahead=lookahead)
        outs.append((info, received))
    (a, ra), (b, rb) = outs
    assert a.ticks == b.ticks
    assert a.ticks == (stop_at + 1 if stop_at is not None else cfg.max_timesteps)
    for k in ("action_seqs", "n_actions", "success", "distances"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert (a.num_interactions, a.num_steps) == (b.num_interactions, b.num_steps)
    assert len(ra) == len(rb) == (0 if is_eval else a.ticks)
    for x, y in zip(ra, rb):
        assert np.array_equal(x, y)
    if keep_obs:
        assert torch.equal(a.obs, b.obs)
    assert sim._live_dev != 0                  # the flags were stored into mapped host memory


def test_host_flag_pointer(gpu):
    """craft_host_flag_pointer maps torch's page-locked memory (the any-live flags) and refuses
    pageable memory."""
    import ctypes
    from psketch_amd import _native as N
    p = ctypes.c_void_p()
    pinned = torch.zeros(8, dtype=torch.int32, pin_memory=True)
    assert N.lib().craft_host_flag_pointer(pinned.data_ptr(), ctypes.byref(p)) == 0 and p.value
    plain = torch.zeros(8, dtype=torch.int32)
    assert N.lib().craft_host_flag_pointer(plain.data_ptr(), ctypes.byref(p)) == N.EINVAL


@pytest.mark.parametrize("is_eval,bc_rate,stop_at,G,fused", [(False, 0.5, None, 8, True), (False, 0.0, 6, 7, True),
                                                             (True, 0.0, 9, 40, True), (False, 0.0, 17, 1, True),
                                                             (False, 0.5, None, 8, False), (False, 1.0, 13, 5, False)])
def test_graph_rollout_equals_sync_loop(gpu, is_eval, bc_rate, stop_at, G, fused):
    """do_rollout(graph=G) (HIP graphs of G ticks, captured once per simulator and act, replayed
    by later rollouts) gives the synchronous loop's result bit for bit at 65,536 envs: two
    rollouts on different specs and cloning masks through the same graphs, early stops inside
    and at the end of a chunk, every receive() call; fused=False: the teacher forked beside the
    student inside the graphs (against the fused synchronous loop)."""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout
    from psketch_amd.sim import sample_scenarios, synthetic_specs
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    n = 65536
    rng = np.random.RandomState(4)
    W = rng.randint(-3, 4, size=(4, cfg.n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, 0])
    base = torch_policy(W, bias, gpu)

    def act(obs, t):
        a = base(obs, t)
        return torch.full_like(a, 5) if stop_at is not None and t >= stop_at else a

    ref_sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    ref_sim.load_pool(pool)
    g_sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    g_sim.load_pool(pool)
    for rep in range(2):
        spec = synthetic_specs(pool, 12, 12, n, seed=3 + rep, task_ids=[t.id for t in tm.dataset_tasks()])
        bc = rng.binomial(1, bc_rate, size=n)
        outs = []
        for sim, graph in ((ref_sim, 0), (g_sim, G)):
            received = []
            info = do_rollout(sim, spec, act, is_eval, behavior_clone=bc,
                              receive=lambda r: received.append(r.cpu().numpy()), graph=graph,
                              fused_teacher=fused or not graph)
            outs.append((info, received))
        (a, ra), (b, rb) = outs
        assert a.ticks == b.ticks
        if bc_rate < 1:                              # (every env cloning: the student's STOP is never taken)
            assert a.ticks == (stop_at + 1 if stop_at is not None else cfg.max_timesteps)
        for k in ("action_seqs", "n_actions", "success", "distances", "is_get"):
            assert torch.equal(getattr(a, k), getattr(b, k)), (rep, k)
        assert (a.num_interactions, a.num_steps) == (b.num_interactions, b.num_steps)
        assert len(ra) == len(rb) == (0 if is_eval else a.ticks)
        for x, y in zip(ra, rb):
            assert np.array_equal(x, y)
    assert len(g_sim._graph_state["graphs"]) == (cfg.max_timesteps + G - 1) // G


def test_rollout_distances_two_lane_path_vs_oracle(golden, gpu, oracle_mod):
    """craft_rollout_distances above 16,384 envs (2 BFS lanes per env): after a 32,768-env
    eval rollout, a 384-env sample's distances equal the oracle's find_closest_resources length
    on the env's initial grid at its final pose (imitation.py:83-89), its is_get the task's goal
    and its action count the action record's; the env states are left as the rollout ended."""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout
    from psketch_amd.sim import synthetic_specs
    sc = golden("scenarios_seed123.npz")
    pool = sc["w12_grids"]
    world = "craft_medium_12x12"
    _, _, tm, cfg = make_tables(world)
    n = 32768
    tasks = [t.id for t in tm.dataset_tasks()]
    spec = np.stack(synthetic_specs(pool, 12, 12, n, seed=8, task_ids=tasks), axis=1)
    spec[:, 3] = np.arange(n) % 4
    rng = np.random.RandomState(4)
    W = rng.randint(-3, 4, size=(3, cfg.n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, -40])
    sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    sim.load_pool(pool)
    info = do_rollout(sim, tuple(spec.T), torch_policy(W, bias, gpu), True)
    agent = sim.get_state(fields=("agent",))["agent"].cpu().numpy()
    dist, succ = info.distances.cpu().numpy(), info.success.cpu().numpy()
    is_get, nact = info.is_get.cpu().numpy(), info.n_actions.cpu().numpy()
    seqs = info.action_seqs.cpu().numpy()
    o = oracle_mod.Oracle(cfg, pool)
    get_ids = {t.id for t in tm.tasks if t.goal_name == "get"}
    ids = np.random.RandomState(1).choice(n, 384, replace=False)
    probed = 0
    for i in ids:
        tk = int(spec[i, 4])
        assert bool(is_get[i]) == (tk in get_ids), i
        assert nact[i] == int((seqs[:, i] >= 0).sum()), i
        if tk not in get_ids:
            assert dist[i] == -1, i
        elif succ[i]:
            assert dist[i] == 0, i
        else:
            e = o.env(pool[spec[i, 0]], agent[i, 0], agent[i, 1], agent[i, 2])
            rc, _, ln = o.closest_resource(e, cfg.task[tk].arg_kind)
            assert rc == 0 and dist[i] == ln, (i, dist[i], ln)
            probed += 1
    assert probed > 20
    sim.check()


@pytest.mark.parametrize("case", ["none_success", "no_target", "unreachable"])
def test_do_rollout_raises_where_the_reference_raises(golden, gpu, case):
    """trainers/imitation.py's failures at the end of a rollout, through the summary's
    flags: satisfies() is None for a finished episode (a `use` task: the assert at :68), and a
    failed get task whose initial grid holds none of its target, or only a target walled in by
    boundary cells (find_closest_resources returns None in both cases, and the reference raises
    the same TypeError, len(None), at :88-89).  Every env stops at tick 0 (a STOP-only
    student)."""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import RolloutError, do_rollout
    sc = golden("scenarios_seed123.npz")
    pool = np.array(sc["w12_grids"][:4], dtype=np.uint8)
    world = "craft_medium_12x12"
    _, cb, tm, _ = make_tables(world)
    task = {t.id: str(t) for t in tm.tasks}
    if case == "none_success":
        tid = next(i for i, s in task.items() if s == "use none")
    else:
        tid = next(i for i, s in task.items() if s == "get wood")
        pool[0][pool[0] == cb.index["wood"]] = 0          # row 0 (the only one used) loses its wood
        if case == "unreachable":                         # one wood, no free neighbour
            g = pool[0].reshape(12, 12)
            g[5, 5] = cb.index["wood"]
            for x, y in ((4, 5), (6, 5), (5, 4), (5, 6)):
                g[x, y] = cb.index["boundary"]
    n = 300
    free = [c for c in range(144) if pool[0][c] == 0 and 1 <= c // 12 <= 10 and 1 <= c % 12 <= 10]
    cells = np.asarray(free)[np.arange(n) % len(free)]
    spec = (np.zeros(n, np.int32), (cells // 12).astype(np.int32), (cells % 12).astype(np.int32),
            np.zeros(n, np.int32), np.full(n, tid, np.int32))
    sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    sim.load_pool(pool)
    stop = torch.full((n,), 5, dtype=torch.int32, device=gpu)
    with pytest.raises(RolloutError, match="None" if case == "none_success" else "len\\(None\\)"):
        do_rollout(sim, spec, lambda obs, t: stop, True)
    sim.check()                                           # nothing latched besides the flags


def test_graph_rollout_student_reallocates_weights(gpu):
    """A student that replaces its weight tensor (a new allocation, as an optimizer that
    rebinds parameters does) between rollouts: with graph_key naming the allocation the graphs
    are captured anew and the rollout equals the synchronous loop's with the new weights; with
    the key unchanged, drop_graphs(sim) does the same.  (A replay of the old capture would read
    the old tensor.)"""
    from psketch_amd import CraftSim
    from psketch_amd.rollout import do_rollout, drop_graphs
    from psketch_amd.sim import sample_scenarios, synthetic_specs
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 128)
    n = 8192
    rng = np.random.RandomState(9)

    class Student:
        def __init__(self):
            self.W = torch.as_tensor(rng.randint(-3, 4, size=(cfg.n_features, 6)).astype(np.float64), device=gpu)

        def act(self, obs, t):
            return (obs.double() @ self.W).argmax(dim=1).to(torch.int32)

    st = Student()
    spec = synthetic_specs(pool, 12, 12, n, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    bc = rng.binomial(1, 0.5, size=n)
    ref_sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    g_sim = CraftSim(world, n_envs=n, device=gpu.index, pool_capacity=len(pool))
    for s in (ref_sim, g_sim):
        s.load_pool(pool)

    def both(key, before=None):
        a = do_rollout(ref_sim, spec, st.act, False, behavior_clone=bc)
        if before:
            before()
        b = do_rollout(g_sim, spec, st.act, False, behavior_clone=bc, graph=8, graph_key=key)
        for k in ("action_seqs", "n_actions", "success", "distances"):
            assert torch.equal(getattr(a, k), getattr(b, k)), k
        return g_sim._graph_state["graphs"]

    g0 = both((st.W.data_ptr(),))
    keep = st.W                                     # the old allocation stays alive (no reuse)
    st.W = torch.flip(keep, dims=[1]).contiguous()  # new weights in a new tensor
    g1 = both((st.W.data_ptr(),))
    assert g1 is not g0                             # captured anew for the new key
    st.W = torch.roll(keep, 1, dims=1).contiguous()
    g2 = both(None, before=lambda: drop_graphs(g_sim))
    assert g2 is not g1
    assert both(None) is g2                         # same act and key: the graphs are reused
    del keep
