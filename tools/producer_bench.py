"""Diagnostic: launch time of craft_rollout with and without observations, per
tile / threads configuration (product build, HIP events).  Without observations
only the producer's transitions run, so the difference isolates the observation
half.  Prints us per tick.

  python tools/producer_bench.py [envs] [K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
R = 16
ring = torch.empty((R, n, 404), dtype=torch.float32, device="cuda")
for tile, threads in [(32, 384), (64, 512), (32, 256), (16, 256), (16, 320)]:
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.tune(tile, 0, 0)
    sim.tune_rollout(0, threads)
    sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
    res = []
    for obs in (None, ring):
        tick = 0
        for _ in range(3):
            sim.rollout(K, tick0=tick, obs=obs)
            tick += K
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(8):
            sim.rollout(K, tick0=tick, obs=obs)
            tick += K
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / (8 * K))
    sim.check()
    print(f"tile {tile:3d} threads {threads:3d}: no obs {res[0]:6.2f} us/tick   obs {res[1]:6.2f} us/tick",
          flush=True)
