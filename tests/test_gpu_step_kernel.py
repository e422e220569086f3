"""The one-launch-per-tick kernel (craft_tile.h): config 3's streamed tick (student actions,
behaviour cloning, action record, any-live flag) at 65,536 envs against the CPU oracle
(trainers/imitation.py:43-73 per env)."""
import numpy as np
import pytest
import torch

from psketch_amd import sample_scenarios, synthetic_specs
from tests.helpers import make_tables
from tests.test_gpu_parity import host, sim_with_pool

pytestmark = pytest.mark.gpu


def _outputs(sim, n, with_code=True):
    dev = "cuda"
    return {"obs": sim.empty_obs(), "reward": torch.empty(n, dtype=torch.float32, device=dev),
            "done": torch.empty(n, dtype=torch.uint8, device=dev),
            "success": torch.empty(n, dtype=torch.int8, device=dev),
            "action_record": torch.empty(n, dtype=torch.int32, device=dev),
            "any_live": torch.zeros(1, dtype=torch.int32, device=dev),
            "transition_code": torch.empty(n, dtype=torch.int8, device=dev) if with_code else None}


def test_step_ex_streamed_tick_full_size_vs_oracle(oracle_mod):
    """Config 3's tick as do_rollout issues it (trainers/imitation.py:43-73): 65,536 envs,
    student actions, behaviour cloning from teacher-style labels, the action record and the
    any-live flag, no auto-reset (done envs freeze), 40 ticks = one whole episode; every output
    of 256 envs checked each tick against the oracle run on the same effective actions."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 1024)
    n, T = 65536, 40
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=12, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = sim_with_pool(world, n, pool)
    assert sim.step_shape() == ("tile_kernel", 64, 0)                 # the default
    sim.reset(*specs)
    out = _outputs(sim, n, with_code=False)
    ids = np.sort(np.random.RandomState(5).choice(n, 256, replace=False))
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*[x[ids] for x in specs])
    rng = np.random.RandomState(6)
    bc = (rng.rand(n) < 0.5).astype(np.uint8)               # config.random.binomial(1, mix, n)
    bc_d = torch.as_tensor(bc, device="cuda")
    frozen = np.zeros(n, dtype=bool)
    for t in range(T):
        student = rng.randint(0, 6, size=n).astype(np.int32)
        ref = rng.randint(0, 6, size=n).astype(np.int32)
        out["any_live"].zero_()
        sim.step(torch.as_tensor(student, device="cuda"), tick=t, autoreset=False,
                 ref_actions=torch.as_tensor(ref, device="cuda"), behavior_clone=bc_d, **out)
        eff = np.where(bc == 1, ref, student)
        pre_frozen = envs["frozen"].copy()
        rc, oobs, orew, odone, osucc = o.batch_tick(envs, 0, eff[ids], 0, t, False)
        assert rc == 0
        np.testing.assert_array_equal(host(out["obs"])[ids], oobs, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(host(out["done"])[ids], odone, err_msg=f"done t={t}")
        np.testing.assert_array_equal(host(out["success"])[ids], osucc, err_msg=f"success t={t}")
        np.testing.assert_array_equal(host(out["reward"])[ids], orew, err_msg=f"reward t={t}")
        rec = host(out["action_record"])
        np.testing.assert_array_equal(rec[ids], np.where(pre_frozen != 0, -1, eff[ids]), err_msg=f"rec t={t}")
        np.testing.assert_array_equal(rec, np.where(frozen, -1, eff), err_msg=f"rec (all) t={t}")
        done = host(out["done"]).astype(bool)
        frozen |= done
        assert int(out["any_live"].item()) == int((~done).any()), t
    assert frozen.all()                                     # timer 40: every episode has ended
    st = {k: host(v) for k, v in sim.get_state(slots=torch.as_tensor(ids, dtype=torch.int32,
                                                                         device="cuda")).items()}
    np.testing.assert_array_equal(st["agent"], np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1))
    np.testing.assert_array_equal(st["inventory"], envs["inv"][:, :cfg.n_kinds])
    np.testing.assert_array_equal(st["grid"], envs["grid"][:, :144])
    sim.check()
