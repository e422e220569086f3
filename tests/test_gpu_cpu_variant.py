"""The HIP library and its CPU variant (libpsketch_craft_cpu.so) side by side on
the same inputs: every output of the fused tick + teacher, the K-tick rollout, the standalone
teacher with path lengths, the rollout summary and on-device scenario generation agree bit for
bit."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
from tests.helpers import make_tables, world_for

pytestmark = pytest.mark.gpu


def _pair(world, n, pool):
    out = []
    for dev in (0, "cpu"):
        s = CraftSim(world, n_envs=n, device=dev, pool_capacity=len(pool))
        s.load_pool(pool)
        out.append(s)
    return out


@pytest.mark.parametrize("window", [3, 5])
def test_step_teach_and_rollout_gpu_equals_cpu(window):
    world = world_for(12, window)
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    n = 9000
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=6, task_ids=[t.id for t in tm.dataset_tasks()])
    g, c = _pair(world, n, pool)
    for s in (g, c):
        s.reset(*specs)
    rng = np.random.RandomState(window)
    for t in range(50):                                   # past the 40-tick episodes (auto-reset)
        acts = rng.randint(0, 6, size=n).astype(np.int32)
        res = []
        for s, dev in ((g, "cuda"), (c, "cpu")):
            o = {"obs": s.empty_obs(), "reward": torch.empty(n, device=dev),
                 "done": torch.empty(n, dtype=torch.uint8, device=dev),
                 "success": torch.empty(n, dtype=torch.int8, device=dev),
                 "action_record": torch.empty(n, dtype=torch.int32, device=dev),
                 "transition_code": torch.empty(n, dtype=torch.int8, device=dev),
                 "labels": torch.empty(n, dtype=torch.int32, device=dev)}
            s.step(torch.as_tensor(acts, device=dev), seed=3, tick=t, autoreset=t % 7 != 3, **o)
            res.append({k: v.cpu() for k, v in o.items()})
        for k in res[0]:
            assert torch.equal(res[0][k], res[1][k]), (t, k)
    R = 4
    rings = [torch.empty((R, n, g.n_features), device=d) for d in ("cuda", "cpu")]
    dones = [torch.empty((R, n), dtype=torch.uint8, device=d) for d in ("cuda", "cpu")]
    for s, r, d in ((g, rings[0], dones[0]), (c, rings[1], dones[1])):
        s.rollout(9, seed=8, tick0=50, obs=r, done=d)
    assert torch.equal(rings[0].cpu(), rings[1]) and torch.equal(dones[0].cpu(), dones[1])
    plen = [torch.empty(n, dtype=torch.int32, device=d) for d in ("cuda", "cpu")]
    acts = [s.teacher(path_len_out=p)[0].cpu() for s, p in ((g, plen[0]), (c, plen[1]))]
    assert torch.equal(acts[0], acts[1]) and torch.equal(plen[0].cpu(), plen[1])
    for k, v in g.get_state().items():
        assert torch.equal(v.cpu(), c.get_state()[k]), k
    assert torch.equal(g.stats().cpu(), c.stats())
    g.check()
    c.check()


def test_rollout_distances_and_pool_generate_gpu_equals_cpu():
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    n, T = 5000, 6
    g = CraftSim(world, n_envs=n, device=0, pool_capacity=300)
    c = CraftSim(world, n_envs=n, device="cpu", pool_capacity=300)
    init = [s.generate_pool(300, seed=21, init_pos=True).cpu() for s in (g, c)]
    assert torch.equal(init[0], init[1])
    tasks = [t.id for t in tm.dataset_tasks()]
    spec = (np.arange(n) % 300, init[0][np.arange(n) % 300, 0].numpy(), init[0][np.arange(n) % 300, 1].numpy(),
            np.arange(n) % 4, np.asarray(tasks)[np.arange(n) % len(tasks)])
    for s in (g, c):
        s.reset(*spec)
        for t in range(T):
            s.step(seed=2, tick=t, autoreset=False)
    out = []
    for s, dev in ((g, "cuda"), (c, "cpu")):
        seqs = torch.as_tensor(np.random.RandomState(0).randint(-1, 6, size=(T, n)).astype(np.int32), device=dev)
        task = torch.as_tensor(spec[4].astype(np.int32), device=dev)
        succ = torch.zeros(n, dtype=torch.int8, device=dev)
        d = torch.empty(n, dtype=torch.int32, device=dev)
        ig = torch.empty(n, dtype=torch.uint8, device=dev)
        na = torch.empty(n, dtype=torch.int32, device=dev)
        fl = torch.empty(2, dtype=torch.int32, device=dev)
        s._check(s._L.craft_rollout_distances(s._h, task.data_ptr(), succ.data_ptr(), seqs.data_ptr(), T,
                                              d.data_ptr(), ig.data_ptr(), na.data_ptr(), fl.data_ptr(),
                                              s._stream()), "craft_rollout_distances")
        out.append([x.cpu() for x in (d, ig, na, fl)])
    for a, b in zip(*out):
        assert torch.equal(a, b)
    g.check()
    c.check()
