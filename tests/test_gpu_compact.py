"""Compact observation staging of the tile kernel (craft_obs.h, 5x5 / 7x7 windows): each env
stages local / pooled kind masks and the row's tail bytes instead of a u8 features() row
(craft.py:296-330), and E reads every group of 4 features off them.  Checked against the u8-row
staging (the default; CRAFT_COMPACT=1 at creation selects compact records) on every output of every entry point that observes, for
every observation format, tile size and a partial last tile; and at BASELINE's size (65,536 envs,
12x12, w = 5, one round of 64-env workgroups) against the CPU oracle."""
import numpy as np
import pytest
import torch

from psketch_amd import sample_scenarios, synthetic_specs
from tests.helpers import make_tables
from tests.test_gpu_parity import host, sim_with_pool

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, world, n, pool):
    monkeypatch.setenv("CRAFT_COMPACT", "1")
    a = sim_with_pool(world, n, pool)                       # compact records
    monkeypatch.delenv("CRAFT_COMPACT")
    b = sim_with_pool(world, n, pool)                       # u8 rows (the default)
    return a, b


@pytest.mark.parametrize("world,W,n,tile,fmt", [
    ("craft_medium_12x12_w5", 12, 70001, 0, "f32"),
    ("craft_medium_12x12_w5", 12, 5000, 16, "bf16"),
    ("craft_medium_12x12_w5", 12, 3001, 32, "u8"),
    ("craft_medium_12x12_w5", 12, 4099, 64, "bf16"),
    ("craft_large", 10, 2050, 0, "f32"),
    ("craft_large", 10, 999, 64, "u8"),
    ("craft_16x16_w7", 16, 1500, 0, "f32"),
    ("craft_16x16_w7", 16, 777, 16, "bf16")])
def test_compact_equals_u8_rows(monkeypatch, world, W, n, tile, fmt):
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 96)
    specs = synthetic_specs(pool, W, W, n, 0, seed=5, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = _pair(monkeypatch, world, n, pool)
    for s in (a, b):
        if tile:
            s.tune(tile, 0, 2)
        s.set_obs_format(fmt)
    assert a.tile_shape()[0] == (tile or (64 if cfg.window_width == 5 else 32))
    dev = "cuda"
    oa, ob = a.empty_obs(), b.empty_obs()
    for s, o in ((a, oa), (b, ob)):
        s.reset(*specs, obs=o)                               # MODE_RESET's observation
    assert torch.equal(oa, ob)
    rng = np.random.RandomState(n)
    for t in range(30):                                      # crosses episode restarts
        acts = None if t % 3 == 0 else torch.as_tensor(rng.randint(0, 6, size=n).astype(np.int32), device=dev)
        outs = []
        for s, o in ((a, oa), (b, ob)):
            code = torch.empty(n, dtype=torch.int8, device=dev)
            done = torch.empty(n, dtype=torch.uint8, device=dev)
            s.step(acts, seed=9, tick=t, autoreset=t % 2 == 0, obs=o, done=done, transition_code=code)
            outs.append((done, code))
        assert torch.equal(oa, ob), f"obs differ at tick {t}"
        assert all(torch.equal(x, y) for x, y in zip(*outs)), t
    # MODE_TRANSITION (copy-on-step into other slots), then MODE_OBSERVE over a slot list
    # (repeated and reversed slots)
    m = min(200, n // 2)
    src = torch.arange(m, dtype=torch.int32, device=dev)
    ta = torch.as_tensor(rng.randint(0, 6, size=m).astype(np.int32), device=dev)
    for s in (a, b):
        s.transition(ta, src=src, dst=src + m)
    slots = torch.as_tensor(np.r_[np.arange(n)[::-7], [0, 0, n - 1]].astype(np.int32), device=dev)
    pa = torch.empty((len(slots), a.n_features), dtype=a.obs_dtype, device=dev)
    pb = torch.empty_like(pa)
    a.observe(slots=slots, obs=pa)
    b.observe(slots=slots, obs=pb)
    assert torch.equal(pa, pb)
    for k, v in a.get_state().items():
        assert torch.equal(v, b.get_state()[k]), k
    np.testing.assert_array_equal(host(a.stats()), host(b.stats()))
    a.check()
    b.check()


def test_compact_full_size_vs_oracle(oracle_mod, monkeypatch):
    """65,536 12x12 envs with 5x5 windows (the 64-env compact tiles: 1024 workgroups, one
    round), one craft_step per tick with auto-reset: 256 random global ids against the oracle
    every tick (observation, done, success, reward) and their states at the end."""
    world = "craft_medium_12x12_w5"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 1024)
    n, T = 65536, 45
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=1, task_ids=[t.id for t in tm.dataset_tasks()])
    monkeypatch.setenv("CRAFT_COMPACT", "1")
    sim = sim_with_pool(world, n, pool)
    monkeypatch.delenv("CRAFT_COMPACT")
    assert sim.tile_shape()[0] == 64
    sim.reset(*specs)
    gids = np.sort(np.random.RandomState(7).choice(n, 256, replace=False))
    gid_d = torch.as_tensor(gids, device="cuda")
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*[np.asarray(s)[gids] for s in specs])
    obs = sim.empty_obs()
    outs = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
            (("reward", torch.float32), ("done", torch.uint8), ("success", torch.int8))}
    for t in range(T):
        sim.step(seed=2, tick=t, obs=obs, **outs)
        step = [o.batch_tick(envs[j:j + 1], int(g), None, 2, t, True) for j, g in enumerate(gids)]
        assert all(s[0] == 0 for s in step)
        ref = [np.concatenate([s[m] for s in step]) for m in range(1, 5)]
        np.testing.assert_array_equal(obs[gid_d].cpu().numpy(), ref[0], err_msg=f"obs {t}")
        np.testing.assert_array_equal(outs["reward"][gid_d].cpu().numpy(), ref[1])
        np.testing.assert_array_equal(outs["done"][gid_d].cpu().numpy(), ref[2])
        np.testing.assert_array_equal(outs["success"][gid_d].cpu().numpy(), ref[3])
    st = sim.get_state()
    np.testing.assert_array_equal(st["agent"][gid_d].cpu().numpy(),
                                  np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1))
    np.testing.assert_array_equal(st["inventory"][gid_d].cpu().numpy(), envs["inv"][:, :cfg.n_kinds])
    sim.check()
