"""Step-by-step probe of craft_rollout_teach (diagnostic): each call synchronised and timed, so a
hang names its step.  python tools/rt_probe.py [n] [ticks]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402
from tests.helpers import make_tables  # noqa: E402


def step(name, fn):
    t0 = time.perf_counter()
    try:
        r = fn()
        torch.cuda.synchronize()
    except Exception as e:                       # a latched kernel error: report it and go on
        print(f"{name}: {e}", flush=True)
        import re
        m = re.search(r"slot/item (-?\d+)", str(e))
        if m:
            x = int(m.group(1)) & (2**64 - 1)
            print(f"   wait {x >> 60} item {(x >> 32) & 0xfffffff} state {x & 0xffffffff:#010x}", flush=True)
        return None
    print(f"{name}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
    return r


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    world = "craft_medium_12x12"
    params, cb, tm, cfg = make_tables(world)
    pool, _, _ = sample_scenarios(params, cb, 123, 256)
    specs = synthetic_specs(pool, 12, 12, n, 0, seed=6, task_ids=[t.id for t in tm.dataset_tasks()])
    sim = step("create", lambda: CraftSim(world, n_envs=n, device=0, pool_capacity=len(pool)))
    step("load_pool (+ teacher table)", lambda: sim.load_pool(pool))
    step("reset", lambda: sim.reset(*specs))
    lab = step("teacher", lambda: sim.teacher()[0])
    step("check", sim.check)
    labels = torch.zeros((T, n), dtype=torch.int32, device="cuda")
    for mode in ("bfs", "table"):
        sim.tune_teach(0, 0, 1 if mode == "table" else 2)
        sim.reset(*specs)
        step(f"rollout_teach {mode} (no obs)", lambda: sim.rollout_teach(T, seed=1, labels=labels))
        step("check", sim.check)
        obs = torch.zeros((T, n, sim.n_features), dtype=torch.float32, device="cuda")
        step(f"rollout_teach {mode} (obs)", lambda: sim.rollout_teach(T, seed=1, tick0=T, obs=obs, labels=labels))
        step("check", sim.check)
    print("labels", np.bincount(labels.cpu().numpy().ravel() + 2), flush=True)


if __name__ == "__main__":
    main()
