"""craft_step_teach (config 5's tick): one launch that steps every env and labels
its new state with the DemonstrationTeacher (teachers/demonstration.py:9-30,
teachers/base.py:10-87), checked against craft_step_ex followed by the
standalone craft_teacher (itself pinned by the reference's 4400
demonstrations) and, on a sample, against the per-target BFS oracle."""
import numpy as np
import pytest
import torch

from psketch_amd import sample_scenarios, synthetic_specs
from tests.helpers import make_tables
from tests.test_gpu_parity import host, sim_with_pool

pytestmark = pytest.mark.gpu


# kernel: 0 the library's choice (the two-tile kernel for 3x3 windows from 32768 envs), 1 the
# one-tile kernel (craft_tile.h), 2 the two-tile kernel (craft_tick2.h; the one-tile kernel for
# other windows)
@pytest.mark.parametrize("world,W,n,T,autoreset,given,kernel", [
    ("craft_medium_12x12", 12, 65536, 45, True, False, 0),  # config 5's size, across episode ends
    ("craft_medium_12x12", 12, 5000, 45, False, True, 2),   # frozen envs (label -1), a partial tile
    ("craft_medium_12x12", 12, 5000, 45, False, True, 1),
    ("craft_medium_12x12", 12, 40000, 45, False, True, 2),  # partial last workgroup
    ("craft_medium_12x12", 12, 70001, 12, True, True, 0),
    ("craft_medium_12x12", 12, 4000, 30, True, True, 0),
    ("craft_medium", 8, 3000, 30, True, True, 2),           # 8x8: two words per cell set
    ("craft_medium", 8, 3000, 30, True, True, 1),
    ("craft_medium_12x12_w5", 12, 2048, 20, True, False, 2),  # w = 5: always the one-tile kernel
    ("craft_large", 10, 1024, 20, True, False, 2),          # 10x10: four words per cell set
    ("craft_large", 10, 1024, 20, True, False, 1)])
def test_step_teach_equals_step_then_teacher(world, W, n, T, autoreset, given, kernel):
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    specs = synthetic_specs(pool, W, W, n, 0, seed=6, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.tune_teach(kernel)
    a.reset(*specs)
    b.reset(*specs)
    F = a.n_features
    rng = np.random.RandomState(2)
    oa, ob = (torch.empty((n, F), dtype=torch.float32, device="cuda") for _ in range(2))
    da, db = (torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2))
    la = torch.empty(n, dtype=torch.int32, device="cuda")
    for t in range(T):
        acts = (torch.as_tensor(rng.randint(0, 6, size=n).astype(np.int32), device="cuda")
                if given else None)
        a.step(acts, seed=3, tick=t, autoreset=autoreset, obs=oa, done=da, labels=la)
        b.step(acts, seed=3, tick=t, autoreset=autoreset, obs=ob, done=db)
        lb, _ = b.teacher()
        assert torch.equal(oa, ob), t
        assert torch.equal(da, db), t
        assert torch.equal(la, lb), t
    if not autoreset:
        assert bool((la == -1).any())                     # frozen envs are labelled -1
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))
    a.check()
    b.check()


# The one-tile kernel on 32-env tiles (5x5 / 7x7 windows, tile_kernel<WIN, 0, 32, 2, NW>): 192 tick
# threads beside the teacher pairs, each env's teacher word and the deferred BFS list in row
# padding, task_sub as bytes (craft_tile.h).  table 2: every go leaf is a deferred BFS, so the
# list fills; USE raised in the given actions, so cells are cleared and recipes run.
@pytest.mark.parametrize("world,W,n,T,table,given", [
    ("craft_medium_12x12_w5", 12, 65536, 10, 0, False),   # config 5's size: four workgroups per CU
    ("craft_medium_12x12_w5", 12, 5000, 30, 2, True),     # the deferred list full; a partial tile
    ("craft_large", 10, 4000, 25, 2, True),
    (dict(WIDTH=12, HEIGHT=12, WINDOW_WIDTH=7, WINDOW_HEIGHT=7, N_WORKSHOPS=3, N_PRIMITIVES=2, N_WORLDS=100),
     12, 3000, 25, 2, True)])
def test_step_teach_wide_windows_equal_step_then_teacher(world, W, n, T, table, given):
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    specs = synthetic_specs(pool, W, W, n, 0, seed=11, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = sim_with_pool(world, n, pool), sim_with_pool(world, n, pool)
    a.tune_teach(1, 0, table)
    kname, envs, lanes = a.step_shape(teach=True)
    assert (envs, lanes) == (32, 2), (kname, envs, lanes)
    a.reset(*specs)
    b.reset(*specs)
    F = a.n_features
    rng = np.random.RandomState(5)
    oa, ob = (torch.empty((n, F), dtype=torch.float32, device="cuda") for _ in range(2))
    la = torch.empty(n, dtype=torch.int32, device="cuda")
    for t in range(T):
        acts = (torch.as_tensor(rng.choice(6, size=n, p=[.15, .15, .15, .15, .38, .02]).astype(np.int32),
                                device="cuda") if given else None)
        a.step(acts, seed=3, tick=t, autoreset=not given, obs=oa, labels=la)
        b.step(acts, seed=3, tick=t, autoreset=not given, obs=ob)
        lb, _ = b.teacher()
        assert torch.equal(oa, ob), t
        assert torch.equal(la, lb), t
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    if given:                                             # cells were cleared (deferred BFS queries)
        assert bool((sa["grid"].cpu().numpy() != pool[sa["spec"].cpu().numpy()[:, 0]]).any())
    a.check()
    b.check()


def test_step_teach_vs_oracle(oracle_mod):
    """The fused labels of 65536 mid-rollout envs against the literal BFS oracle
    on 1024 of them."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 512)
    n = 65536
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=8, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.reset(*specs)
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    for t in range(9):
        sim.step(seed=5, tick=t, labels=lab)
    st = {k: host(v) for k, v in sim.get_state().items()}
    sim.check()
    lab = host(lab)
    o = oracle_mod.Oracle(cfg, pool)
    for i in np.random.RandomState(3).choice(n, 1024, replace=False):
        x, y, d, _ = st["agent"][i]
        env = o.env(st["grid"][i], x, y, d, st["inventory"][i])
        rc, act = o.teacher(env, int(specs[4][i]))
        assert rc == 0 and act == lab[i], i


def test_step_teach_rejects_oversized_worlds():
    """4*W*H > 1000 overflows the reference's fixed BFS queue (teachers/base.py:42):
    refused before any launch, as craft_teacher does."""
    from psketch_amd import _native as N
    world = "craft_16x16_w7"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 8)
    sim = sim_with_pool(world, 64, pool)
    sim.reset(*synthetic_specs(pool, 16, 16, 64, 0, seed=0, task_ids=[t.id for t in tm.dataset_tasks()]))
    lab = torch.empty(64, dtype=torch.int32, device="cuda")
    with pytest.raises(N.CraftError):
        sim.step(seed=0, tick=0, labels=lab)


@pytest.mark.parametrize("table,obs_mode", [(0, "reused"), (0, "null"), (2, "ring")])
def test_step_teach_late_episode_vs_oracle(oracle_mod, table, obs_mode):
    """A whole 40-tick episode at config 5's size with USE raised, so cleared cells and crafted
    inventories are common late in the episode, and 1024 envs checked against the literal BFS
    oracle at ticks 9, 25 and 38 (teachers/base.py:10-87): with the teacher table read (auto mode
    reads it when obs is NULL or one buffer is rewritten every tick) and with it off (table 2),
    observations going to a fresh ring slot every tick."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 512)
    n = 65536
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=12, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    sim.tune_teach(0, 0, table)
    sim.reset(*specs)
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    F = sim.n_features
    ring = [torch.empty((n, F), dtype=torch.float32, device="cuda") for _ in range(2 if obs_mode == "ring" else 1)]
    rng = np.random.RandomState(21)
    o = oracle_mod.Oracle(cfg, pool)
    pick = np.random.RandomState(4).choice(n, 1024, replace=False)
    checked = 0
    for t in range(40):
        acts = torch.as_tensor(rng.choice(6, size=n, p=[.15, .15, .15, .15, .38, .02]).astype(np.int32),
                               device="cuda")
        obs = None if obs_mode == "null" else ring[t % len(ring)]
        sim.step(acts, seed=5, tick=t, autoreset=False, obs=obs, labels=lab)
        if t in (9, 25, 38):
            st = {k: host(v) for k, v in sim.get_state().items()}
            sim.check()
            lh = host(lab)
            cleared = (st["grid"][pick] != pool[st["spec"][pick, 0]]).any(1)
            crafted = st["inventory"][pick][:, 12:].sum(1) > 0           # planks and later products
            if t >= 25:
                assert cleared.mean() > 0.2 and crafted.any(), (t, cleared.mean())
            for i in pick:
                x, y, d, _ = st["agent"][i]
                if lh[i] == -1:                                          # frozen: the episode ended
                    continue
                env = o.env(st["grid"][i], x, y, d, st["inventory"][i])
                rc, act = o.teacher(env, int(specs[4][i]))
                assert (rc == 0 and act == lh[i]) or (rc != 0 and lh[i] == -2), (t, i)
                checked += 1
    assert checked > 1024
