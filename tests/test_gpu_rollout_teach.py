"""craft_rollout_teach on the GPU (csrc/craft_rollout_teach.h): K ticks and the
DemonstrationTeacher's label of every env's new state per tick in one launch.  Checked tick by
tick against craft_step_teach (itself pinned to craft_teacher, the oracle and the reference's 4400
demonstrations), against the CPU variant of the ABI, against the oracle on sampled global ids at
config 5's size, and by regenerating the reference's demonstrations (make_data.py:146-152) in
20-tick launches."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from tests.helpers import make_tables
from tests.test_gpu_parity import host, set_states, sim_with_pool

pytestmark = pytest.mark.gpu


def _rings(sim, ring):
    n, dev = sim.n_envs, sim.device
    return dict(obs=torch.zeros((ring, n, sim.n_features), dtype=sim.obs_dtype, device=dev),
                done=torch.zeros((ring, n), dtype=torch.uint8, device=dev),
                success=torch.zeros((ring, n), dtype=torch.int8, device=dev),
                reward=torch.zeros((ring, n), dtype=torch.float32, device=dev),
                labels=torch.zeros((ring, n), dtype=torch.int32, device=dev),
                action_record=torch.zeros((ring, n), dtype=torch.int32, device=dev))


def _setup(world, W, n, pool_n=256, seed=6, base=0):
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, pool_n)
    specs = synthetic_specs(pool, W, W, n, base, seed=seed, task_ids=[t.id for t in tm.dataset_tasks()])
    return cfg, pool, specs


# mode: policy = the hashed draw; given = an action table (USE raised: cells cleared, recipes);
# bc = behaviour cloning on half the envs; label = every env acts on its label (demonstrations)
@pytest.mark.parametrize("world,W,n,T,K,ring,mode,autoreset", [
    ("craft_medium_12x12", 12, 65536, 40, 20, 40, "policy", True),   # config 5's size
    ("craft_medium_12x12", 12, 65536, 40, 40, 8, "given", True),     # ring < K: slots rewritten
    ("craft_medium_12x12", 12, 20000, 40, 13, 40, "bc", True),
    ("craft_medium_12x12", 12, 5000, 40, 40, 40, "label", False),    # partial tile, frozen envs
    ("craft_medium_12x12", 12, 4099, 30, 10, 30, "bc", False),
    ("craft_medium", 8, 3000, 30, 15, 30, "given", True),            # 8x8: two words per cell set
    ("craft_large", 10, 1500, 25, 25, 25, "policy", True),           # 10x10, 5x5 windows
    ("craft_medium_12x12_w5", 12, 2048, 25, 25, 25, "given", True),
    ("craft_medium_12x12", 12, 8192, 30, 15, 30, "given_bc", True)])      # action table + cloning
def test_rollout_teach_equals_step_teach(world, W, n, T, K, ring, mode, autoreset):
    cfg, pool, specs = _setup(world, W, n)
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.reset(*specs)
    b.reset(*specs)
    rng = np.random.RandomState(11)
    acts = (rng.choice(6, size=(T, n), p=[.18, .18, .18, .18, .26, .02]).astype(np.int32)
            if mode in ("given", "given_bc") else None)
    bc = (rng.rand(n) < 0.5).astype(np.uint8) if mode in ("bc", "given_bc") else None
    src = (torch.ones(n, dtype=torch.uint8, device="cuda") if mode == "label"
           else (torch.as_tensor(bc, device="cuda") if bc is not None else None))
    cur = b.teacher()[0].clone()                                  # labels of the reset states
    out = _rings(a, ring)
    lab_in = cur.clone()
    F = a.n_features
    ob = torch.empty((n, F), dtype=torch.float32, device="cuda")
    db, rb = torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.float32, device="cuda")
    sb, recb = torch.empty(n, dtype=torch.int8, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda")
    lb = torch.empty(n, dtype=torch.int32, device="cuda")
    for t0 in range(0, T, K):
        k = min(K, T - t0)
        a.rollout_teach(k, seed=3, tick0=t0,
                        actions=None if acts is None else torch.as_tensor(acts[t0:t0 + k], device="cuda"),
                        autoreset=autoreset, label_in=lab_in if src is not None else None,
                        behavior_clone=None if bc is None else torch.as_tensor(bc, device="cuda"),
                        label_actions=mode == "label", **out)
        lab_in = out["labels"][(t0 + k - 1) % ring].clone()
        for t in range(t0, t0 + k):
            b.step(None if acts is None else torch.as_tensor(acts[t], device="cuda"), seed=3, tick=t,
                   autoreset=autoreset, obs=ob, reward=rb, done=db, success=sb, action_record=recb,
                   ref_actions=cur if src is not None else None, behavior_clone=src, labels=lb)
            cur = lb.clone()
            if t >= T - ring or ring >= T:                       # slots not rewritten later
                r = t % ring
                assert torch.equal(out["obs"][r], ob), t
                for key, ref in (("done", db), ("success", sb), ("reward", rb), ("action_record", recb),
                                 ("labels", lb)):
                    assert torch.equal(out[key][r], ref), (key, t)
    sa, sb2 = a.get_state(), b.get_state()
    for key in sa:
        assert torch.equal(sa[key], sb2[key]), key
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))
    if mode == "label" and not autoreset:
        assert bool((lb == -1).all())                             # every demonstration ended
    a.check()
    b.check()


def _hip_vs_cpu(world, W, n, T, mode, seed=2, pool_n=256):
    cfg, pool, specs = _setup(world, W, n, seed=seed, pool_n=pool_n)
    g = sim_with_pool(world, n, pool)
    c = CraftSim(world, n_envs=n, device="cpu", pool_capacity=len(pool))
    c.load_pool(pool)
    g.reset(*specs)
    c.reset(*specs)
    bc = (np.random.RandomState(4).rand(n) < 0.5).astype(np.uint8)
    kw = {}
    if mode == "bc":
        kw = dict(behavior_clone=bc)
    elif mode == "label":
        kw = dict(label_actions=True)
    outs = []
    for s in (g, c):
        r = _rings(s, T)
        if mode != "policy":
            kw["label_in"] = s.teacher()[0].clone()
        s.rollout_teach(T, seed=9, autoreset=mode != "label", **{k: (torch.as_tensor(v, device=s.device)
                                                                    if isinstance(v, np.ndarray) else v)
                                                                 for k, v in kw.items()}, **r)
        s.check()
        outs.append({k: v.cpu() for k, v in r.items()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
    return outs[0]


@pytest.mark.parametrize("mode", ["policy", "bc", "label"])
def test_rollout_teach_hip_equals_cpu_variant(mode):
    _hip_vs_cpu("craft_medium_12x12", 12, 2048, 35, mode)


def _world(W, win, prims=2):
    return dict(WIDTH=W, HEIGHT=W, WINDOW_WIDTH=win, WINDOW_HEIGHT=win, N_WORKSHOPS=3, N_PRIMITIVES=prims,
                N_WORLDS=100)


# The instantiations no BASELINE config runs: 7x7 windows (rollout_teach_kernel<7, 16, 4>, whose LDS
# carve passes 64 KiB: the table words' LDS-DMA target stays first in it) and 15x15 grids (8 BFS
# words: <3, 32, 8> and <7, 16, 8>, the variants with scratch spills)
@pytest.mark.parametrize("W,win,prims,mode", [(12, 7, 2, "policy"), (12, 7, 2, "label"), (15, 3, 4, "policy"),
                                              (15, 7, 4, "bc")])
def test_rollout_teach_wide_instantiations_equal_cpu_variant(W, win, prims, mode):
    out = _hip_vs_cpu(_world(W, win, prims), W, 1024, 30, mode, pool_n=128)
    if mode == "label":                                        # demonstrations: actions, then -1 once ended
        assert bool((out["labels"] >= -1).all()) and bool((out["labels"][0] >= 0).all())
    else:
        assert (out["labels"] >= 0).float().mean() > 0.5       # labels are mostly actions, not -1/-2


def test_rollout_teach_long_launch():
    """A 1200-tick launch (the teacher wave's bounded waits count per wait, not per launch: no
    error latches however long the launch) equals the same ticks in 4 launches."""
    world, W, n, T = "craft_medium_12x12", 12, 1024, 1200
    cfg, pool, specs = _setup(world, W, n, seed=3)
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.reset(*specs)
    b.reset(*specs)
    ra, rb = _rings(a, 8), _rings(b, 8)
    a.rollout_teach(T, seed=7, **ra)
    a.check()
    for t0 in range(0, T, 300):
        b.rollout_teach(300, seed=7, tick0=t0, **rb)
    b.check()
    for k in ra:
        assert torch.equal(ra[k], rb[k]), k
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))


def test_rollout_teach_capture_right_after_pool_load():
    """A launch captured into a graph straight after load_pool: the capture refuses to build the
    new rows' teacher-table entries (they would be rebuilt on every replay); after sync_table the
    captured launch replays equal to an eager one."""
    from psketch_amd._native import CraftError
    world, W, n, T = "craft_medium_12x12", 12, 4096, 10
    cfg, pool, specs = _setup(world, W, n, seed=5)
    a = sim_with_pool(world, n, pool)
    a.reset(*specs)
    ra = _rings(a, T)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(CraftError, match="sync_table"):
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                a.rollout_teach(T, seed=1, **ra)
    torch.cuda.synchronize()
    b = sim_with_pool(world, n, pool)
    b.reset(*specs)
    b.sync_table()
    rb = _rings(b, T)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g2, stream=s):
            b.rollout_teach(T, seed=1, **rb)
    g2.replay()
    torch.cuda.synchronize()
    b.check()
    c = sim_with_pool(world, n, pool)
    c.reset(*specs)
    rc = _rings(c, T)
    c.rollout_teach(T, seed=1, **rc)
    c.check()
    for k in rb:
        assert torch.equal(rb[k], rc[k]), k


@pytest.mark.parametrize("world,mode", [("craft_medium_12x12", "policy"), ("craft_medium_12x12_w5", "policy"),
                                        ("craft_medium_12x12", "bc"), ("craft_medium_12x12", "label")])
def test_rollout_teach_vs_oracle_full_size(oracle_mod, world, mode):
    """Config 5's launch (65,536 envs, 40 ticks of hashed actions with auto-reset, every env
    labelled every tick), with 3x3 and 5x5 windows, against the literal oracle on 256 sampled
    global ids, run from their initial states with their own ids: labels, actions, done, success
    and every tick's observation rows; bc: half the envs act on their labels (the transition
    wave's own lookup), the label of the first tick from the oracle; label: every env does
    (make_data's demonstrations, auto-reset after each episode)."""
    from oracle import rollout_oracle
    W, n, T, base = 12, 65536, 40, 65536
    cfg, pool, specs = _setup(world, W, n, pool_n=1024, seed=0, base=base)
    sim = sim_with_pool(world, n, pool, env_id_base=base)
    sim.reset(*specs)
    out = _rings(sim, T)
    kw, bc, lab = {}, None, None
    if mode == "bc":
        bc = (np.random.RandomState(2).rand(n) < 0.5).astype(np.uint8)
        kw = dict(behavior_clone=torch.as_tensor(bc, device="cuda"))
    elif mode == "label":
        bc = np.ones(n, dtype=np.uint8)
        kw = dict(label_actions=True)
    if bc is not None:
        lab = sim.teacher()[0].clone()
    sim.rollout_teach(20, seed=5, tick0=0, label_in=lab, **kw, **out)
    sim.rollout_teach(20, seed=5, tick0=20, label_in=None if lab is None else out["labels"][19].clone(), **kw, **out)
    sim.check()
    pick = np.sort(np.random.RandomState(1).choice(n, 256, replace=False))
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*[np.asarray(x)[pick] for x in specs])
    extra = {} if bc is None else dict(label_in=host(lab)[pick], label_src=bc[pick])
    ref = rollout_oracle.teach_rollout(o, envs, base + pick, T, seed=5, want_obs=True, **extra)
    for k in ("labels", "action_record", "done", "success"):
        np.testing.assert_array_equal(host(out[k])[:, pick], ref[k], err_msg=k)
    ob = out["obs"][:, torch.as_tensor(pick, device="cuda")].cpu().numpy()
    for t in range(T):
        np.testing.assert_array_equal(ob[t], ref["obs"][t], err_msg=f"observations, tick {t}")
    assert (ref["labels"] >= 0).mean() > 0.9


@pytest.mark.parametrize("split", ["dev", "test"])
def test_demonstrations_regenerated_on_gpu(golden, split):
    """make_data.get_reference_actions (make_data.py:146-152) for every committed instance, on
    the GPU in 20-tick launches: every env acts on its label until STOP.  The action record is
    the reference's ref_actions and every episode ends satisfied."""
    g = golden("devtest.npz")
    n = len(g[f"{split}_task"])
    sim = sim_with_pool("craft_medium", n, g[f"{split}_grids"])
    pos = g[f"{split}_pos"].astype(np.int32)
    agent = np.concatenate([pos, np.zeros((n, 1), np.int32)], 1)
    set_states(sim, g[f"{split}_world"], agent, np.zeros((n, 1)), task=g[f"{split}_task"])
    ref = g[f"{split}_actions"].astype(np.int32)
    label_in = sim.teacher()[0].clone()
    rec = []
    for tick0 in (0, 20):
        out = _rings(sim, 20)
        sim.rollout_teach(20, tick0=tick0, label_in=label_in, label_actions=True, autoreset=False, **out)
        rec.append(host(out["action_record"]))
        label_in = out["labels"][19].clone()
    sim.check()
    rec = np.concatenate(rec)
    L = ref.shape[1]
    np.testing.assert_array_equal(rec[:L].T, ref)
    assert (rec[L:] == -1).all()
    sat = torch.empty(n, dtype=torch.int8, device="cuda")
    sim.observe(sat=sat, n=n)
    assert (host(sat) == 1).all()


@pytest.mark.parametrize("mode", ["given", "label"])
def test_rollout_teach_with_and_without_table(mode):
    """The teacher table (pristine grids answered at pool load) against every query running the
    BFS (craft_sim_tune_teach table = 2): identical labels.  With label actions the transition
    wave looks labels up itself (table) or waits for every go label's BFS answer (no table)."""
    world, W, n, T = "craft_medium_12x12", 12, 32768, 40
    cfg, pool, specs = _setup(world, W, n, seed=3)
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    b.tune_teach(0, 0, 2)
    rng = np.random.RandomState(7)
    acts = torch.as_tensor(rng.choice(6, size=(T, n), p=[.18, .18, .18, .18, .26, .02]).astype(np.int32),
                           device="cuda")
    outs = []
    for s in (a, b):
        s.reset(*specs)
        r = _rings(s, T)
        if mode == "label":
            s.rollout_teach(T, label_in=s.teacher()[0].clone(), label_actions=True, **r)
        else:
            s.rollout_teach(T, actions=acts, **r)
        s.check()
        outs.append(r)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_rollout_teach_graph_replay():
    """A launch captured into a HIP graph (its own zeroed work counter) replays like eager
    launches, interleaved with them."""
    world, W, n, K = "craft_medium_12x12", 12, 8192, 8
    cfg, pool, specs = _setup(world, W, n, seed=5)
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.reset(*specs)
    b.reset(*specs)
    ra, rb = _rings(a, K), _rings(b, K)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a.rollout_teach(K, seed=1, tick0=0, **ra)                # warm (eager)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        a.rollout_teach(K, seed=1, tick0=K, **ra)
    b.rollout_teach(K, seed=1, tick0=0, **rb)
    for rep in range(3):
        g.replay()                                                # ticks K..2K-1 each time (same tick0)
        torch.cuda.synchronize()
        b.rollout_teach(K, seed=1, tick0=K, **rb)
        for k in ra:
            assert torch.equal(ra[k], rb[k]), (k, rep)
        a.rollout_teach(K, seed=1, tick0=0, **ra)                # eager between replays
        b.rollout_teach(K, seed=1, tick0=0, **rb)
    a.check()
    b.check()


@pytest.mark.parametrize("mode", ["policy", "label"])
def test_rollout_teach_hint_walk_fallback(mode):
    """A hint tree with more satisfies() predicates than the tabulated walk takes (make[ladder]
    over bed, axe and shears: 15) keeps the walk itself; mixed with tabulated tasks in one tile,
    labels equal craft_step_teach's (teach_env's walk) tick by tick.  With label actions such a
    config keeps the row-synchronous mode (every item's row complete before the next tick)."""
    import copy
    from psketch_amd import gamedef
    hints = copy.deepcopy(gamedef.HINTS)
    hints["make[ladder]"] = ["make[bed]", "make[axe]", "make[shears]", "makeat[workshop2]"]
    world, W, n, T = "craft_medium_12x12", 12, 4096, 30
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    a = CraftSim(world, n_envs=n, device=0, pool_capacity=len(pool), hints=hints)
    b = CraftSim(world, n_envs=n, device=0, pool_capacity=len(pool), hints=hints)
    for s in (a, b):
        s.load_pool(pool)
    ids = [t.id for t in a.task_manager.dataset_tasks()]
    ladder = a.task_manager["make[ladder]"].id
    specs = synthetic_specs(pool, W, W, n, 0, seed=4, task_ids=[ladder, ladder] + ids)
    a.reset(*specs)
    b.reset(*specs)
    out = _rings(a, T)
    label = mode == "label"
    cur = b.teacher()[0].clone()
    a.rollout_teach(T, seed=2, label_in=cur.clone() if label else None, label_actions=label, **out)
    ob = torch.empty((n, a.n_features), dtype=torch.float32, device="cuda")
    lb = torch.empty(n, dtype=torch.int32, device="cuda")
    src = torch.ones(n, dtype=torch.uint8, device="cuda") if label else None
    for t in range(T):
        b.step(None, seed=2, tick=t, obs=ob, labels=lb, ref_actions=cur if label else None, behavior_clone=src)
        assert torch.equal(out["labels"][t], lb), t
        cur = lb.clone()
    if not label:
        assert (host(out["labels"])[:, np.asarray(specs[4]) == ladder] >= 0).mean() > 0.5
    a.check()
    b.check()


@pytest.mark.parametrize("table", [1, 2])
def test_rollout_teach_late_episode_vs_oracle(oracle_mod, table):
    """Config 5's size through a whole 40-tick episode in rollout_teach launches ending at ticks
    9, 25 and 38, USE raised so that cleared cells and crafted inventories are common late in the
    episode; 1024 envs' labels of those ticks against the literal BFS oracle on the state the
    launch left, with the teacher table read (1) and off (2)."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 512)
    n, T = 65536, 40
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=12, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.tune_teach(0, 0, table)
    sim.reset(*specs)
    rng = np.random.RandomState(21)
    acts = torch.as_tensor(rng.choice(6, size=(T, n), p=[.15, .15, .15, .15, .38, .02]).astype(np.int32),
                           device="cuda")
    o = oracle_mod.Oracle(cfg, pool)
    pick = np.random.RandomState(4).choice(n, 1024, replace=False)
    out = _rings(sim, 16)
    checked, t0 = 0, 0
    for t1 in (10, 26, 39, 40):
        sim.rollout_teach(t1 - t0, seed=5, tick0=t0, actions=acts[t0:t1], autoreset=False, **out)
        t = t1 - 1
        t0 = t1
        if t not in (9, 25, 38):
            continue
        st = {k: host(v) for k, v in sim.get_state().items()}
        sim.check()
        lh = host(out["labels"][t % 16])
        cleared = (st["grid"][pick] != pool[st["spec"][pick, 0]]).any(1)
        if t >= 25:
            assert cleared.mean() > 0.2 and (st["inventory"][pick][:, 12:].sum(1) > 0).any(), t
        for i in pick:
            x, y, d, _ = st["agent"][i]
            if lh[i] == -1:                                              # frozen: the episode ended
                continue
            env = o.env(st["grid"][i], x, y, d, st["inventory"][i])
            rc, act = o.teacher(env, int(specs[4][i]))
            assert (rc == 0 and act == lh[i]) or (rc != 0 and lh[i] == -2), (t, i)
            checked += 1
    assert checked > 1024


def test_rollout_teach_refusals_on_the_gpu():
    """The HIP library refuses what the CPU variant refuses (tests/test_rollout_teach_cpu.py):
    labels feeding actions without label_in, a ring shorter than one slot, negative ticks; a
    refused call launches nothing and leaves the states as they were."""
    from psketch_amd import _native as N
    world, W, n = "craft_medium_12x12", 12, 256
    cfg, pool, specs = _setup(world, W, n, pool_n=16)
    sim = sim_with_pool(world, n, pool)
    sim.reset(*specs)
    before = {k: v.clone() for k, v in sim.get_state().items()}
    with pytest.raises(N.CraftError):
        sim.rollout_teach(4, label_actions=True)
    with pytest.raises(N.CraftError):
        sim.rollout_teach(4, behavior_clone=torch.ones(n, dtype=torch.uint8, device="cuda"))
    with pytest.raises(N.CraftError):
        sim.rollout_teach(4, tick0=-1)
    with pytest.raises(N.CraftError):
        sim.tune_teach(0, 3, 0)
    after = sim.get_state()
    for k in before:
        assert torch.equal(before[k], after[k]), k
    sim.check()


@pytest.mark.parametrize("n,mode", [(1, "policy"), (7, "policy"), (33, "policy"), (95, "policy"),
                                    (7, "label"), (33, "label"), (33, "bc"), (95, "bc")])
def test_rollout_teach_tiny_batches_equal_cpu_variant(n, mode):
    """Fewer envs than one tile, one env past a tile, three tiles minus one: the persistent grid
    sizes itself to the tiles and the tail tile's idle lanes store nothing (label / bc: the LA
    kernel, whose transition wave publishes labels for the tail tile's live lanes only)."""
    world, W, T = "craft_medium_12x12", 12, 30
    cfg, pool, specs = _setup(world, W, n, pool_n=16, seed=n)
    g = sim_with_pool(world, n, pool)
    c = CraftSim(world, n_envs=n, device="cpu", pool_capacity=len(pool))
    c.load_pool(pool)
    outs = []
    bc = (np.random.RandomState(n).rand(n) < 0.5).astype(np.uint8)
    for s in (g, c):
        s.reset(*specs)
        r = _rings(s, 8)
        kw = {}
        if mode != "policy":
            kw["label_in"] = s.teacher()[0].clone()
            if mode == "label":
                kw["label_actions"] = True
            else:
                kw["behavior_clone"] = torch.as_tensor(bc, device=s.device)
        s.rollout_teach(T, seed=4, autoreset=True, **kw, **r)
        s.check()
        outs.append(({k: v.cpu() for k, v in r.items()}, {k: v.cpu() for k, v in s.get_state().items()}))
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("fmt", ["bf16", "u8"])
def test_rollout_teach_obs_formats(fmt):
    """The narrower observation formats hold the same exact values (craft_sim_set_obs_format):
    the teacher rollout's ring in bf16 / u8 equals its fp32 ring, labels and states unchanged."""
    world, W, n, T = "craft_medium_12x12", 12, 4096, 24
    cfg, pool, specs = _setup(world, W, n, seed=8)
    outs = []
    for f in ("f32", fmt):
        s = sim_with_pool(world, n, pool)
        s.set_obs_format(f)
        s.reset(*specs)
        r = _rings(s, T)
        s.rollout_teach(T, seed=6, **r)
        s.check()
        outs.append(({k: v.float() if k == "obs" else v for k, v in r.items()}, s.get_state()))
    (a, sa), (b, sb) = outs
    for k in a:
        assert torch.equal(a[k], b[k]), k
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_rollout_teach_label_actions_after_many_cleared_cells():
    """Label actions from states with more than three cells cleared this episode (the transition
    wave's lookup then reads the grid instead of its cleared-cell list) and with fewer: 60 ticks of
    USE-heavy given actions with an axe and bridges in hand (grabs, stone and water cleared), then
    20 ticks acting on labels in one launch, tick by tick against craft_step_teach fed its own
    labels (no auto-reset: cleared cells stay)."""
    world, W, n, T0, T = "craft_medium_12x12", 12, 32768, 60, 20
    cfg, pool, specs = _setup(world, W, n, seed=8)
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    ix = a.cookbook.index
    inv = np.zeros((n, a.n_kinds), dtype=np.int32)
    inv[:, ix["axe"]] = 1
    inv[:, ix["bridge"]] = 4
    agent = np.stack([specs[1], specs[2], specs[3]], 1)
    acts = torch.as_tensor(np.random.RandomState(5).choice(6, size=(T0, n), p=[.125, .125, .125, .125, .5, 0])
                           .astype(np.int32), device="cuda")
    for s in (a, b):
        set_states(s, specs[0], agent, inv, task=specs[4])
        s.rollout(T0, actions=acts, autoreset=False)
    cur = b.teacher()[0].clone()
    st = a.get_state(fields=("grid", "spec"))
    g, sp = host(st["grid"]), host(st["spec"])
    cleared = ((np.asarray(pool)[sp[:, 0]] != 0) & (g == 0)).sum(1)
    assert (cleared >= 4).sum() >= 20 and (cleared <= 3).mean() > 0.2, np.bincount(cleared)   # (~0.14 % past 3)
    out = _rings(a, T)
    a.rollout_teach(T, tick0=T0, label_in=cur.clone(), label_actions=True, autoreset=False, **out)
    ob = torch.empty((n, a.n_features), dtype=torch.float32, device="cuda")
    lb = torch.empty(n, dtype=torch.int32, device="cuda")
    recb = torch.empty(n, dtype=torch.int32, device="cuda")
    src = torch.ones(n, dtype=torch.uint8, device="cuda")
    for t in range(T):
        b.step(None, tick=T0 + t, autoreset=False, obs=ob, labels=lb, action_record=recb, ref_actions=cur,
               behavior_clone=src)
        assert torch.equal(out["labels"][t], lb), t
        assert torch.equal(out["action_record"][t], recb), t
        assert torch.equal(out["obs"][t], ob), t
        cur = lb.clone()
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    a.check()
    b.check()
