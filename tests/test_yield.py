"""Recipes with `_yield` > 1 (craft.py:394 `n_inventory[output] += yld`).  The inventory is u8
on the device, so a count that would pass 255 saturates and latches CRAFT_ERANGE instead of
wrapping (the reference's float inventory never overflows; no recipe of the reference's own
recipes.yaml yields more than 1, so these are synthetic recipes).  Checked on the oracle, the CPU
variant and the HIP library: a known-answer USE, a 40-tick lockstep rollout with raised USE and
rich inventories against the oracle, and the overflow latch."""
import copy

import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from psketch_amd import _native as N
from psketch_amd import gamedef
from tests.helpers import make_tables
from tests.test_gpu_parity import set_states

WORLD, W = "craft_medium_12x12", 12


def yield_recipes(plank=2, stick=3, rope=1):
    r = copy.deepcopy(gamedef.RECIPES)
    r["recipes"]["plank"]["_yield"] = plank
    r["recipes"]["stick"]["_yield"] = stick
    r["recipes"]["rope"]["_yield"] = rope
    return r


def _sim(device, n, pool, recipes):
    s = CraftSim(WORLD, n_envs=n, device=device, pool_capacity=len(pool), recipes=recipes)
    s.load_pool(pool)
    return s


def _facing(pool, kind):
    """(pool row, x, y, dir) with the agent on a free interior cell facing a cell of `kind`."""
    for p, g in enumerate(pool.reshape(len(pool), W, W)):
        for x in range(1, W - 1):
            for y in range(1, W - 1):
                if g[x, y] != 0:
                    continue
                for d, (dx, dy) in enumerate(((0, -1), (0, 1), (-1, 0), (1, 0))):   # DOWN UP LEFT RIGHT
                    if g[x + dx, y + dy] == kind:
                        return p, x, y, d
    raise AssertionError("no such cell")


def _kat(device):
    recipes = yield_recipes()
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 16)
    sim = _sim(device, 2, pool, recipes)
    ix = sim.cookbook.index
    p0, x0, y0, d0 = _facing(pool, ix["workshop0"])
    p1, x1, y1, d1 = _facing(pool, ix["workshop1"])
    inv = np.zeros((2, sim.n_kinds), dtype=np.int32)
    inv[0, ix["wood"]] = 3                        # plank (yield 2) at workshop0
    inv[1, ix["wood"]] = 1                        # stick (yield 3) at workshop1
    inv[1, ix["plank"]] = 1
    inv[1, ix["grass"]] = 1                       # then bed (plank 1, grass 1) chains
    set_states(sim, [p0, p1], [[x0, y0, d0], [x1, y1, d1]], inv)
    sim.transition(torch.full((2,), 4, dtype=torch.int32, device=sim.device))   # USE
    sim.check()
    got = sim.get_state()["inventory"].cpu().numpy()
    exp = inv.copy()
    exp[0, ix["wood"]], exp[0, ix["plank"]] = 2, 2
    exp[1, ix["wood"]], exp[1, ix["stick"]] = 0, 3
    exp[1, ix["plank"]], exp[1, ix["grass"]], exp[1, ix["bed"]] = 0, 0, 1
    np.testing.assert_array_equal(got, exp)
    return sim, pool


def _lockstep(device, oracle_mod, n=600, T=40):
    recipes = yield_recipes()
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    sim = _sim(device, n, pool, recipes)
    specs = synthetic_specs(pool, W, W, n, 0, seed=3, task_ids=[t.id for t in tm.dataset_tasks()])
    rng = np.random.RandomState(8)
    inv = np.zeros((n, sim.n_kinds), dtype=np.int32)
    for k in ("wood", "iron", "grass"):
        inv[:, sim.cookbook.index[k]] = rng.randint(0, 12, size=n)
    agent = np.stack([specs[1], specs[2], specs[3]], 1)
    set_states(sim, specs[0], agent, inv, task=specs[4])
    o = oracle_mod.Oracle(sim.config, pool)
    envs = o.init_envs(*specs)
    envs["inv"][:, :sim.n_kinds] = inv
    dev = sim.device
    obs, rew = sim.empty_obs(), torch.empty(n, dtype=torch.float32, device=dev)
    done, succ = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int8, device=dev)
    stats = np.zeros(3, dtype=np.int64)
    made = 0
    for t in range(T):
        acts = rng.choice(6, size=n, p=[.15, .15, .15, .15, .38, .02]).astype(np.int32)
        sim.step(torch.as_tensor(acts, device=dev), seed=5, tick=t, autoreset=False, obs=obs, reward=rew,
                 done=done, success=succ)
        rc, oobs, orew, odone, osucc = o.batch_tick(envs, 0, acts, 5, t, False, True, stats)
        assert rc == 0
        np.testing.assert_array_equal(done.cpu().numpy(), odone, err_msg=f"t={t}")
        np.testing.assert_array_equal(succ.cpu().numpy(), osucc, err_msg=f"t={t}")
        np.testing.assert_array_equal(obs.float().cpu().numpy(), oobs, err_msg=f"t={t}")
        st = sim.get_state()
        np.testing.assert_array_equal(st["inventory"].cpu().numpy(), envs["inv"][:, :sim.n_kinds], err_msg=f"t={t}")
        made = max(made, int(envs["inv"][:, sim.cookbook.index["stick"]].max()))
    assert made >= 6                              # two stick crafts somewhere: yield 3 exercised
    np.testing.assert_array_equal(sim.get_state()["grid"].cpu().numpy(), envs["grid"][:, :W * W])
    sim.check()


def _overflow(device):
    """A count that would pass 255 saturates at 255 and latches CRAFT_ERANGE with the slot."""
    recipes = yield_recipes(rope=200)
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 16)
    sim = _sim(device, 4, pool, recipes)
    ix = sim.cookbook.index
    p, x, y, d = _facing(pool, ix["workshop0"])
    inv = np.zeros((4, sim.n_kinds), dtype=np.int32)
    inv[:, ix["grass"]] = 2
    inv[2, ix["rope"]] = 100                      # 100 + 200 > 255
    set_states(sim, [p] * 4, [[x, y, d]] * 4, inv)
    use = torch.full((4,), 4, dtype=torch.int32, device=sim.device)
    sim.transition(use)
    w = sim.error_word().tolist()
    assert w[0] == N.ERANGE and w[2] == 2
    with pytest.raises(N.CraftError) as e:
        sim.check()
    assert e.value.status == N.ERANGE
    got = sim.get_state()["inventory"].cpu().numpy()
    assert got[2, ix["rope"]] == 255 and got[0, ix["rope"]] == 200 and got[0, ix["grass"]] == 1
    sim.transition(use)                           # slot 0: 200 + 200 -> 255, latched again
    assert sim.get_state()["inventory"].cpu().numpy()[0, ix["rope"]] == 255
    with pytest.raises(N.CraftError):
        sim.check()


def test_yield_refused_outside_range():
    params, cb, tm, cfg = make_tables(WORLD)
    for bad in (0, 256):
        with pytest.raises(N.CraftError):
            CraftSim(WORLD, n_envs=4, device="cpu", pool_capacity=1, recipes=yield_recipes(plank=bad))


def test_yield_oracle_kat(oracle_mod):
    """The oracle's own known answer: USE at workshop0 with wood 3 and plank yield 2."""
    recipes = yield_recipes()
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 16)
    sim = CraftSim(WORLD, n_envs=1, device="cpu", pool_capacity=1, recipes=recipes)
    ix = sim.cookbook.index
    p, x, y, d = _facing(pool, ix["workshop0"])
    o = oracle_mod.Oracle(sim.config, pool)
    envs = o.init_envs(np.array([p], np.int32), np.array([x], np.int32), np.array([y], np.int32),
                       np.array([d], np.int32), np.zeros(1, np.int32))
    envs["inv"][0, ix["wood"]] = 3
    rc, *_ = o.batch_tick(envs, 0, np.array([4], np.int32), 0, 0, False, False, np.zeros(3, np.int64))
    assert rc == 0
    assert envs["inv"][0, ix["wood"]] == 2 and envs["inv"][0, ix["plank"]] == 2


def test_yield_kat_cpu():
    _kat("cpu")


def test_yield_lockstep_vs_oracle_cpu(oracle_mod):
    _lockstep("cpu", oracle_mod)


def test_yield_overflow_latch_cpu():
    _overflow("cpu")


@pytest.mark.gpu
def test_yield_kat_gpu():
    _kat("cuda:0")


@pytest.mark.gpu
def test_yield_lockstep_vs_oracle_gpu(oracle_mod):
    _lockstep("cuda:0", oracle_mod, n=4099)


@pytest.mark.gpu
def test_yield_overflow_latch_gpu():
    _overflow("cuda:0")


@pytest.mark.gpu
def test_yield_rollouts_hip_equal_cpu_variant():
    """The multi-tick rollouts (split pipeline and teacher-labelled) with yield recipes: HIP ==
    the CPU variant, labels included."""
    recipes = yield_recipes()
    params, cb, tm, cfg = make_tables(WORLD)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    n, T = 2048, 30
    specs = synthetic_specs(pool, W, W, n, 0, seed=9, task_ids=[t.id for t in tm.dataset_tasks()])
    acts = np.random.RandomState(2).choice(6, size=(T, n), p=[.15, .15, .15, .15, .38, .02]).astype(np.int32)
    outs = []
    for dev in ("cuda:0", "cpu"):
        s = _sim(dev, n, pool, recipes)
        s.reset(*specs)
        r = dict(obs=torch.zeros((T, n, s.n_features), dtype=torch.float32, device=dev),
                 done=torch.zeros((T, n), dtype=torch.uint8, device=dev),
                 success=torch.zeros((T, n), dtype=torch.int8, device=dev),
                 reward=torch.zeros((T, n), dtype=torch.float32, device=dev),
                 labels=torch.zeros((T, n), dtype=torch.int32, device=dev),
                 action_record=torch.zeros((T, n), dtype=torch.int32, device=dev))
        s.rollout_teach(T, actions=torch.as_tensor(acts, device=dev), **r)
        s.check()
        st = s.get_state()
        outs.append(({k: v.cpu() for k, v in r.items()}, {k: v.cpu() for k, v in st.items()}))
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_primitives_for_divides_by_yield():
    """Cookbook.primitives_for (cookbook.py:28-52): an intermediate is made ceil(count/_yield)
    times.  axe needs 4 sticks; stick yields 3 from 1 wood -> 2 wood."""
    from psketch_amd.cookbook import Cookbook
    cb = Cookbook()
    ix = cb.index
    assert cb.primitives_for(ix["axe"]) == {ix["wood"]: 1, ix["iron"]: 1}
    assert cb.primitives_for(ix["ladder"]) == {ix["wood"]: 2}
    r = yield_recipes()
    r["recipes"]["axe"]["stick"] = 4
    cb = Cookbook(r)
    assert cb.primitives_for(ix["axe"]) == {ix["wood"]: 2, ix["iron"]: 1}
    assert cb.primitives_for(ix["ladder"]) == {ix["wood"]: 2}        # plank 1/2 -> 1, stick 1/3 -> 1
    assert cb.primitives_for(ix["bed"]) == {ix["wood"]: 1, ix["grass"]: 1}
