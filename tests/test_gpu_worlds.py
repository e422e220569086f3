"""The drop-in CraftWorld/CraftState surface (psketch_amd.worlds) on the GPU,
driven the way the reference's per-env trainer loop and teachers drive it, and
checked against the reference's demonstrations and the CPU oracle."""
from types import SimpleNamespace as NS

import numpy as np
import pytest

from psketch_amd import worlds
from psketch_amd.cookbook import Task
from tests.helpers import make_tables

pytestmark = pytest.mark.gpu


def make_config(world="craft_medium"):
    return NS(recipes="resources/craft/recipes.yaml",        # absent on the box: built-in table
              world=NS(name="CraftWorld", config=world),
              student=NS(model=NS()), teacher=NS(name="DemonstrationTeacher"),
              trainer=NS(hints="resources/craft/hints.hierarchy.yaml", max_timesteps=40),
              random=np.random.RandomState(0))


def onehot(ids, W, H, K=21):
    g = np.zeros((W, H, K))
    ids = np.asarray(ids).reshape(W, H)
    for k in range(1, K):
        g[..., k] = ids == k
    return g


def test_world_surface_and_config_side_effects():
    cfg = make_config()
    w = worlds.load(cfg)
    assert cfg.student.model.input_size == w.n_features == 404
    assert cfg.student.model.n_actions == w.n_actions == 6
    assert [a.index for a in w.action_space] == list(range(6))
    assert w.actions.LEFT.coord_change == (-1, 0) and w.actions.UP.coord_change == (0, 1)
    assert w.grabbable_indices == [0] + list(range(7, 21))
    assert w.workshop_indices == [2, 3, 4] and (w.water_index, w.stone_index) == (5, 6)


@pytest.mark.parametrize("split", ["dev"])
def test_shim_replays_reference_demonstrations(golden, oracle_mod, split):
    """init_state + step through the reference's ref_actions; features() equals
    the oracle's at every state, the final state satisfies the task, earlier
    states stay unchanged (immutability), teacher-facing helpers agree."""
    g = golden("devtest.npz")
    cfg = make_config()
    w = worlds.load(cfg)
    _, cb, tm, ocfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(ocfg)
    rng = np.random.RandomState(0)
    for i in rng.choice(len(g[f"{split}_task"]), 40, replace=False):
        ids = g[f"{split}_grids"][g[f"{split}_world"][i]]
        x, y = (int(v) for v in g[f"{split}_pos"][i])
        task = tm.tasks[int(g[f"{split}_task"][i])]
        s0 = w.init_state(onehot(ids, 8, 8), (x, y))
        env = o.env(ids, x, y, 0)
        state = s0
        for a in g[f"{split}_actions"][i]:
            if a < 0 or a == 5:
                break
            np.testing.assert_array_equal(state.features(), o.features(env).astype(np.float64))
            nav = state.make_navigation_grid()
            np.testing.assert_array_equal(nav, (env["grid"][0, :64].reshape(8, 8) > 0).astype(float))
            _, state = state.step(int(a))
            o.step(env, int(a))
            assert state.pos == (int(env["x"][0]), int(env["y"][0])) and state.dir == int(env["dir"][0])
            np.testing.assert_array_equal(state.inventory, env["inv"][0, :21].astype(np.float64))
        assert state.satisfies(Task(f"{task.goal_name}[{task.goal_arg}]")) is True
        assert s0.pos == (x, y) and s0.dir == 0 and not s0.inventory.any()
        for arg in ("wood", "iron", "workshop0"):
            kind = cb.index[arg]
            ref = [tuple(p) for p in np.argwhere(env["grid"][0, :64].reshape(8, 8) == kind)]
            assert [tuple(map(int, p)) for p in state.find_resource_positions(arg)] == ref


def test_shim_errors_mirror_reference():
    cfg = make_config()
    w = worlds.load(cfg)
    ids = np.zeros((8, 8), dtype=np.uint8)
    ids[0, :] = ids[-1, :] = ids[:, 0] = ids[:, -1] = 1
    s = w.init_state(onehot(ids, 8, 8), (3, 3))
    with pytest.raises(Exception, match="Unexpected action"):
        s.step(9)
    bad = onehot(ids, 8, 8)
    bad[3, 4, 7] = bad[3, 4, 8] = 1
    with pytest.raises(AssertionError):
        w.init_state(bad, (3, 3))
    assert s.satisfies(Task("makeat[workshop0]")) is None
    assert s.satisfies(Task("get[wood]")) is False


def test_shim_slots_recycle():
    cfg = make_config()
    w = worlds.CraftWorld(cfg, capacity=8)
    ids = np.zeros((8, 8), dtype=np.uint8)
    ids[0, :] = ids[-1, :] = ids[:, 0] = ids[:, -1] = 1
    s = w.init_state(onehot(ids, 8, 8), (3, 3))
    for t in range(50):                       # only a handful alive at any time
        _, s = s.step(t % 4)
    assert 1 <= s.pos[0] <= 6
