"""Diagnostic: multi-tick rollout speed vs the observation ring's allocation.

Allocates several observation rings in one process (each at a new address) and
times K-tick craft_rollout launches into each; prints microseconds per tick and
the ring's base address.  Used to separate address-dependent behaviour from
run-to-run noise."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402


def main():
    n, R, K = 65536, 16, int(sys.argv[1]) if len(sys.argv) > 1 else 32
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(grids)
    sim.tune(int(sys.argv[2]) if len(sys.argv) > 2 else 64, 0, int(sys.argv[3]) if len(sys.argv) > 3 else 0)
    sim.reset(*synthetic_specs(grids, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
    keep = []
    tick = 0
    for i in range(6):
        ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
        keep.append(ring)
        for _ in range(4):
            sim.rollout(K, tick0=tick, obs=ring)
            tick += K
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(40):
            sim.rollout(K, tick0=tick, obs=ring)
            tick += K
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (40 * K)
        ring.fill_(1.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            ring.fill_(0.0)
        torch.cuda.synchronize()
        fill = ring.numel() * 4 * 10 / (time.perf_counter() - t0) / 1e12
        print(f"ring {i} base {ring.data_ptr():#x}: rollout {dt * 1e6:.2f} us/tick, "
              f"fill_ {fill:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
