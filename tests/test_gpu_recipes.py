"""A recipe table longer than the reference's (13 recipes: 39 recipe words, more than a tile's
lanes) with a 3-env tail tile, so that recipe words sit in lanes that hold no env: every kernel
family reads the words by v_readlane from a register loaded while every lane was active
(transition<RCV>, csrc/craft_device.h).  Rich inventories and raised USE make crafting common;
HIP equals the CPU variant (itself pinned to the oracle) state for state, tick by tick."""
import copy

import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, gamedef, sample_scenarios, synthetic_specs
from tests.helpers import make_tables
from tests.test_gpu_parity import set_states

pytestmark = pytest.mark.gpu

WORLD, W = "craft_medium_12x12", 12


def long_recipes():
    r = copy.deepcopy(gamedef.RECIPES)
    r["recipes"].update({
        "ingot": {"iron": 2, "_at": "workshop2"},
        "torch": {"stick": 1, "grass": 1, "_at": "workshop1"},
        "crown": {"iron": 1, "wood": 2, "_at": "workshop0", "_yield": 2},
        "boat": {"plank": 2, "_at": "workshop2"},
    })
    return r


def _sims(n, pool, recipes):
    out = []
    for dev in ("cuda:0", "cpu"):
        s = CraftSim(WORLD, n_envs=n, device=dev, pool_capacity=len(pool), recipes=recipes)
        s.load_pool(pool)
        out.append(s)
    return out


def _start(sims, pool, n, seed):
    params, cb, tm, cfg = make_tables(WORLD)
    specs = synthetic_specs(pool, W, W, n, 0, seed=seed, task_ids=[t.id for t in tm.dataset_tasks()])
    rng = np.random.RandomState(seed)
    ix = sims[0].cookbook.index
    inv = np.zeros((n, sims[0].n_kinds), dtype=np.int32)
    for k in ("wood", "iron", "grass", "stick", "plank"):
        inv[:, ix[k]] = rng.randint(0, 6, size=n)
    agent = np.stack([specs[1], specs[2], specs[3]], 1)
    for s in sims:
        set_states(s, specs[0], agent, inv, task=specs[4])
    return specs


def _same_state(a, b, what):
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert torch.equal(sa[k].cpu(), sb[k].cpu()), (what, k)


def chained_recipes():
    """Still three recipes per workshop with at most two ingredients (the compact per-workshop
    table, SimView::wsr), but with an output that is also its own ingredient (stick) and a
    recipe whose ingredient an earlier one at the same workshop makes (axe from plank)."""
    r = copy.deepcopy(gamedef.RECIPES)
    r["recipes"]["stick"] = {"wood": 1, "stick": 1, "_at": "workshop1", "_yield": 3}
    r["recipes"]["axe"] = {"plank": 1, "iron": 1, "_at": "workshop0"}
    return r


def triple_recipes():
    """A recipe with three ingredients, which the compact table cannot hold either."""
    r = copy.deepcopy(gamedef.RECIPES)
    r["recipes"]["bed"] = {"plank": 1, "grass": 1, "stick": 1, "_at": "workshop1"}
    return r


@pytest.mark.parametrize("recipes,n", [("long", 35), ("long", 4099), ("chained", 4099), ("triple", 4099)])
def test_long_recipe_table_every_kernel(recipes, n):
    """(long: a workshop with four recipes, triple: a recipe with three ingredients, which the
    compact table cannot hold: every kernel's general recipe loop; chained: the compact table's
    two-round-trip path with its forwarding)"""
    recipes = {"long": long_recipes, "chained": chained_recipes, "triple": triple_recipes}[recipes]()
    assert len(recipes["recipes"]) in (13, 9)
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    g, c = _sims(n, pool, recipes)
    T = 24
    acts = np.random.RandomState(3).choice(6, size=(T, n), p=[.14, .14, .14, .14, .42, .02]).astype(np.int32)
    # one tick per launch (tile kernel), with the teacher (one-tile or two-tile kernel)
    _start((g, c), pool, n, 1)
    for t in range(T):
        for s in (g, c):
            s.step(torch.as_tensor(acts[t], device=s.device), tick=t, autoreset=True)
    _same_state(g, c, "step")
    if len(recipes["recipes"]) == 13:
        crafted = g.get_state()["inventory"].cpu().numpy()[:, 21:].sum()
        assert crafted > 0                                # the added recipes fired
    _start((g, c), pool, n, 2)
    lab = [torch.empty(n, dtype=torch.int32, device=s.device) for s in (g, c)]
    for t in range(T):
        for s, lb in zip((g, c), lab):
            s.step(torch.as_tensor(acts[t], device=s.device), tick=t, autoreset=True, labels=lb)
        assert torch.equal(lab[0].cpu(), lab[1]), t
    _same_state(g, c, "step_teach")
    # K ticks per launch: the rollout kernel and the teacher-labelled rollout
    for kind in ("rollout", "rollout_teach"):
        _start((g, c), pool, n, 3)
        outs = []
        for s in (g, c):
            r = dict(done=torch.zeros((T, n), dtype=torch.uint8, device=s.device),
                     success=torch.zeros((T, n), dtype=torch.int8, device=s.device))
            a = torch.as_tensor(acts, device=s.device)
            if kind == "rollout":
                s.rollout(T, actions=a, **r)
            else:
                r["labels"] = torch.zeros((T, n), dtype=torch.int32, device=s.device)
                s.rollout_teach(T, actions=a, **r)
            outs.append({k: v.cpu() for k, v in r.items()})
        for k in outs[0]:
            assert torch.equal(outs[0][k], outs[1][k]), (kind, k)
        _same_state(g, c, kind)
    g.check()
    c.check()
