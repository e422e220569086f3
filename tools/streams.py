"""Diagnostic: the bench workload (65536 envs) split into S sims of 65536/S envs
on S streams, ticked K at a time (K = 1: craft_step, K > 1: craft_rollout).
Kernels of different streams overlap, so one stream's launch tail (its slowest
workgroups) runs alongside another stream's next launch.

  python tools/streams.py [K ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402


def run(world, S, K, n=65536, ticks=1024, ring=16):
    sims, rings, streams = [], [], []
    g = None
    for i in range(S):
        m = n // S
        sim = CraftSim(world, n_envs=m, device=0, env_id_base=i * m, pool_capacity=1024)
        if g is None:
            g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
        sim.load_pool(g)
        sim.tune(0, 0, 1 if K == 1 else 0)
        sim.reset(*synthetic_specs(g, sim.width, sim.height, m, i * m, 0,
                                   [t.id for t in sim.task_manager.dataset_tasks()]))
        sims.append(sim)
        rings.append(torch.empty((ring, m, sim.n_features), device="cuda"))
        streams.append(torch.cuda.Stream() if S > 1 else torch.cuda.current_stream())
    torch.cuda.synchronize()
    st = {"t": 0}

    def launch():
        t = st["t"]
        for i in range(S):
            with torch.cuda.stream(streams[i]):
                if K == 1:
                    sims[i].step(seed=0, tick=t, obs=rings[i][t % ring])
                else:
                    sims[i].rollout(K, seed=0, tick0=t, obs=rings[i])
        st["t"] += K

    for _ in range(max(1, 64 // K)):
        launch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(ticks // K):
        launch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / ticks
    for s in sims:
        s.check()
    return round(dt * 1e6, 2)


out = {}
for K in [int(k) for k in sys.argv[1:]] or [1, 32]:
    out[f"K{K}"] = {f"S{S}": run("craft_medium_12x12", S, K) for S in (1, 2, 4)}
    print(json.dumps({f"K{K}": out[f"K{K}"]}), flush=True)
