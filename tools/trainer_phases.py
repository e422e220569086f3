"""Diagnostic: the trainer line's rollout (bench.py --workload trainer: do_rollout with graphs of
8 ticks, 65,536 envs) split into do_rollout's own phases (timing=): setup (reset, the initial
labels, buffer fills), the tick loop, and the summary (distances kernel + one read-back), host
wall microseconds per rollout and per tick.

    python tools/trainer_phases.py [--graph 8] [--reps 6]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402
from psketch_amd.rollout import do_rollout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--graph", type=int, default=8)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    n = args.envs
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(grids)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = [torch.as_tensor(a, device=sim.device) for a in synthetic_specs(grids, 12, 12, n, 0, seed=0, task_ids=tasks)]
    act, _, _ = bench.trainer_policy(sim.n_features, sim.device, seed=7)
    bc = torch.as_tensor(np.random.RandomState(0).binomial(1, 0.5, size=n), device=sim.device)
    rows = []
    for rep in range(args.reps):
        timing = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = do_rollout(sim, specs, act, False, behavior_clone=bc, receive=lambda r: None, lookahead=True,
                          graph=args.graph, timing=timing)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if rep == 0:
            continue                                   # the capture
        rows.append({"wall_us": wall * 1e6, "ticks": info.ticks,
                     **{k: v * 1e6 for k, v in timing.items() if k != "ticks"}})
    mean = {k: float(np.mean([r[k] for r in rows])) for k in rows[0]}
    mean["per_tick"] = {k: mean[k] / mean["ticks"] for k in ("wall_us", "setup", "loop", "summary")}
    print(json.dumps(mean))


if __name__ == "__main__":
    main()
