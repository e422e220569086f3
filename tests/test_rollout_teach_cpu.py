"""craft_rollout_teach (the teacher-labelled K-tick rollout: config 5's DAgger labels and
make_data.get_reference_actions' demonstrations) through the CPU variant of the C ABI, checked on
the CPU against the oracle's restatement (oracle/rollout_oracle.py teach_rollout) and against the
reference's own 4400 demonstrations (data/craft_medium_{dev,test}.json, tests/golden/devtest.npz).
tests/test_gpu_rollout_teach.py checks the HIP kernel against this and against craft_step_teach."""
import numpy as np
import pytest
import torch

from psketch_amd import sample_scenarios, synthetic_specs
from psketch_amd import _native as N
from tests.helpers import make_tables
from tests.test_cpu_variant import cpu_sim
from tests.test_gpu_parity import set_states


def _run(sim, T, ring, **kw):
    n = sim.n_envs
    out = dict(obs=torch.zeros((ring, n, sim.n_features), dtype=torch.float32),
               done=torch.zeros((ring, n), dtype=torch.uint8),
               success=torch.zeros((ring, n), dtype=torch.int8),
               reward=torch.zeros((ring, n), dtype=torch.float32),
               labels=torch.zeros((ring, n), dtype=torch.int32),
               action_record=torch.zeros((ring, n), dtype=torch.int32))
    sim.rollout_teach(T, **kw, **out)
    return out


# mode: the action source (policy = hashed draw, given = an action table, bc = behaviour cloning on
# half the envs, label = every env acts on its label: make_data's demonstrations)
@pytest.mark.parametrize("mode,autoreset", [("policy", True), ("given", True), ("bc", True),
                                            ("label", False), ("label", True), ("bc", False),
                                            ("given_bc", True)])
def test_rollout_teach_cpu_vs_oracle(oracle_mod, mode, autoreset):
    from oracle import rollout_oracle
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 64)
    n, T, base, seed = 160, 45, 1000, 7
    specs = synthetic_specs(pool, 12, 12, n, base, seed=4, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = cpu_sim(world, n, pool, env_id_base=base)
    sim.reset(*specs)
    rng = np.random.RandomState(5)
    acts = (rng.choice(6, size=(T, n), p=[.2, .2, .2, .2, .18, .02]).astype(np.int32)
            if mode in ("given", "given_bc") else None)
    bc = (rng.rand(n) < 0.5).astype(np.uint8) if mode in ("bc", "given_bc") else None
    lsrc = mode in ("bc", "label", "given_bc")
    label_in = sim.teacher()[0].clone() if lsrc else None
    out = _run(sim, T, T, seed=seed, actions=None if acts is None else torch.as_tensor(acts),
               autoreset=autoreset, label_in=label_in, behavior_clone=None if bc is None else torch.as_tensor(bc),
               label_actions=mode == "label")
    sim.check()
    o = oracle_mod.Oracle(cfg, pool)
    envs = o.init_envs(*specs)
    src = np.ones(n, bool) if mode == "label" else (bc.astype(bool) if bc is not None else None)
    ref = rollout_oracle.teach_rollout(o, envs, np.arange(base, base + n), T, seed=seed, actions=acts,
                                       autoreset=autoreset, label_in=None if label_in is None else label_in.numpy(),
                                       label_src=src)
    for k in ("labels", "action_record", "done", "success"):
        np.testing.assert_array_equal(out[k].numpy(), ref[k], err_msg=k)
    if mode == "label" and not autoreset:
        assert (out["labels"].numpy()[-1] == -1).all()      # every demonstration ended with STOP
    st = sim.get_state()
    np.testing.assert_array_equal(st["agent"][:, 0].numpy(), envs["x"])
    np.testing.assert_array_equal(st["agent"][:, 1].numpy(), envs["y"])
    np.testing.assert_array_equal(st["inventory"].numpy(), envs["inv"][:, :sim.n_kinds])
    # the observation ring holds each tick's features (the same tick kernel as craft_rollout)
    assert out["obs"].sum() > 0


def test_rollout_teach_cpu_ring_wraps():
    """ring < n_ticks: each output slot holds the last tick that wrote it."""
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    n, T = 96, 23
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=1, task_ids=[t.id for t in tm.dataset_tasks()])
    a, b = cpu_sim(world, n, pool), cpu_sim(world, n, pool)
    a.reset(*specs)
    b.reset(*specs)
    full = _run(a, T, T, seed=3)
    wrap = _run(b, T, 5, seed=3)
    for k in full:
        for t in range(T - 5, T):
            np.testing.assert_array_equal(wrap[k][t % 5].numpy(), full[k][t].numpy(), err_msg=f"{k} {t}")


@pytest.mark.parametrize("split", ["dev", "test"])
def test_demonstrations_cpu(golden, split):
    """make_data.get_reference_actions on every committed instance: each env acts on its own
    label until STOP; two launches of 20 ticks, the second continuing from the first's last
    labels.  The action record equals the reference's ref_actions and every episode ends
    satisfied."""
    g = golden("devtest.npz")
    n = len(g[f"{split}_task"])
    sim = cpu_sim("craft_medium", n, g[f"{split}_grids"])
    pos = g[f"{split}_pos"].astype(np.int32)
    agent = np.concatenate([pos, np.zeros((n, 1), np.int32)], 1)
    set_states(sim, g[f"{split}_world"], agent, np.zeros((n, 1)), task=g[f"{split}_task"])
    ref = g[f"{split}_actions"].astype(np.int32)
    label_in = sim.teacher()[0].clone()
    rec = []
    for tick0 in (0, 20):
        out = _run(sim, 20, 20, tick0=tick0, label_in=label_in, label_actions=True, autoreset=False)
        rec.append(out["action_record"].numpy())
        label_in = out["labels"][19].clone()
    sim.check()
    rec = np.concatenate(rec)                       # [40, n]
    L = ref.shape[1]
    np.testing.assert_array_equal(rec[:L].T, ref)
    assert (rec[L:] == -1).all()
    sat = torch.empty(n, dtype=torch.int8)
    sim.observe(sat=sat, n=n)
    assert (sat.numpy() == 1).all()


def test_rollout_teach_cpu_refuses():
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 4)
    sim = cpu_sim(world, 8, pool)
    with pytest.raises(N.CraftError):
        sim.rollout_teach(4, label_actions=True)    # labels feed actions: label_in required
    with pytest.raises(N.CraftError):
        sim.tune_teach(0, 3, 0)
