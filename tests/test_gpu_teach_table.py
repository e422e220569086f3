"""The teacher table (craft_teach.h): find_closest_resources answered ahead of time for every
pool row's pristine grid, read by every teacher query whose env has cleared no cell.  It is the
same function evaluated earlier, so every label, path length and summary must equal the BFS's
(craft_sim_tune_teach(.., table=2) keeps every teacher off the table; table=1 makes the fused tick +
teacher kernels read it on every launch, which these tests set explicitly).  The reference fixtures of
tests/test_gpu_parity.py (teacher_12x12.npz with its raising calls, the 4400 demonstrations) run
through the table path too: their states are set with set_state, i.e. pristine grids."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from tests.helpers import make_tables, world_for

pytestmark = pytest.mark.gpu


def _pair(world, n, pool, kernel=0):
    """Two simulators: every teacher on the table (table=1), and none (table=2)."""
    out = []
    for table in (1, 2):
        s = CraftSim(world, n_envs=n, device=0, pool_capacity=len(pool))
        s.load_pool(pool)
        s.tune_teach(kernel, 0, table)
        out.append(s)
    return out


@pytest.mark.parametrize("world,W,n,teach_kernel", [("craft_medium_12x12", 12, 65536, 0),
                                                    ("craft_medium_12x12", 12, 3000, 1),
                                                    ("craft_medium_12x12_w5", 12, 5000, 0),
                                                    ("craft_medium", 8, 4096, 0),
                                                    ("craft_16x16_w7", 16, 2000, 0)])
def test_step_teach_labels_with_and_without_table(world, W, n, teach_kernel):
    params, cb, tm, cfg = make_tables(world)
    if 4 * W * W > 1000:
        pytest.skip("4*W*H > 1000: no teacher (teachers/base.py:42)")
    pool, _, _ = sample_scenarios(params, cb, 123, 128)
    specs = synthetic_specs(pool, W, W, n, 0, seed=9, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = _pair(world, n, pool, teach_kernel)
    for s in (a, b):
        s.reset(*specs)
    rng = np.random.RandomState(n)
    labels = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
    for t in range(45):                        # envs grab (masks fill) and restart (masks clear)
        acts = torch.as_tensor(rng.choice(6, size=n, p=[.2, .2, .2, .2, .18, .02]).astype(np.int32), device="cuda")
        for s, lab in zip((a, b), labels):
            s.step(acts, seed=1, tick=t, autoreset=True, labels=lab)
        assert torch.equal(labels[0], labels[1]), t
    plen = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
    acts = [s.teacher(path_len_out=p)[0] for s, p in zip((a, b), plen)]
    assert torch.equal(acts[0], acts[1]) and torch.equal(plen[0], plen[1])
    # without path lengths the standalone teacher defers its BFS queries to a dense pass
    dense = [s.teacher()[0] for s in (a, b)]
    assert torch.equal(dense[0], acts[0]) and torch.equal(dense[1], acts[0])
    assert torch.equal(labels[0], acts[0])            # the last tick's labels are these states' labels
    a.check()
    b.check()


def test_rollout_summary_with_and_without_table():
    """craft_rollout_distances always searches the initial (pool) grid: with the table it never
    runs the BFS; distances, is_get and the raise flags are the BFS's."""
    from psketch_amd.rollout import do_rollout
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    n = 20000
    spec = synthetic_specs(pool, 12, 12, n, 0, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = _pair(world, n, pool)
    W = torch.as_tensor(np.random.RandomState(3).randint(-3, 4, size=(cfg.n_features, 6)), dtype=torch.float32,
                        device="cuda")

    def act(obs, t):
        return (obs @ W).argmax(1).to(torch.int32)
    infos = [do_rollout(s, spec, act, True) for s in (a, b)]
    for k in ("action_seqs", "n_actions", "success", "distances", "is_get"):
        assert torch.equal(getattr(infos[0], k), getattr(infos[1], k)), k
    assert (infos[0].distances > 0).any()


def test_table_rows_loaded_piecewise_and_reloaded():
    """Pool rows loaded in pieces (out of order, one row alone, a row replaced by another grid)
    and generated on the device: the table entries are built lazily by the next launch that
    reads the table, so every teacher answers as the table-off BFS does, including for the
    replaced row."""
    world, W, n = "craft_medium_12x12", 12, 8192
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 96)
    other, _, _ = sample_scenarios(params, cb, 7, 1)
    sims = []
    for table in (1, 2):
        s = CraftSim(world, n_envs=n, device=0, pool_capacity=128)
        s.tune_teach(0, 0, table)
        s.load_pool(pool[40:96], first=40)
        s.load_pool(pool[:1], first=0)
        s.load_pool(pool[1:40], first=1)
        sims.append(s)
    specs = synthetic_specs(pool, W, W, n, 0, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    for s in sims:
        s.reset(*specs)
    first = [s.teacher()[0].clone() for s in sims]
    assert torch.equal(first[0], first[1])
    pool2 = pool.copy()
    pool2[5] = other[0]
    specs = synthetic_specs(pool2, W, W, n, 0, seed=2, task_ids=[t.id for t in tm.dataset_tasks()])
    for s in sims:                                     # row 5 replaced: its entries rebuilt
        s.load_pool(other, first=5)
        s.reset(*specs)
    second = [s.teacher()[0].clone() for s in sims]
    assert torch.equal(second[0], second[1])
    rows5 = torch.as_tensor(np.asarray(specs[0]) == 5, device="cuda")
    assert not torch.equal(first[0][rows5], second[0][rows5])    # (the new grid answers differently)
    for s in sims:
        s.check()
