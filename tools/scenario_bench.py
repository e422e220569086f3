"""Scenario generation throughput: craft_pool_generate (GPU, one lane per world)
vs the host generator craft_sample_scenarios (C++, numpy's MT19937 stream, one
thread) on 12x12 craft_medium.

  python tools/scenario_bench.py [--count 524288]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=524288)
    ap.add_argument("--world", default="craft_medium_12x12")
    args = ap.parse_args()
    sim = CraftSim(args.world, n_envs=64, device=0, pool_capacity=args.count)
    sim.generate_pool(1024, seed=1)                    # warm-up (module load)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for rep in range(3):
        ev[0].record()
        sim.generate_pool(args.count, seed=100 + rep)
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    sim.check()
    gpu = args.count / min(times)
    t0 = time.perf_counter()
    sample_scenarios(sim.params, sim.cookbook, 123, 2000, dedup=False)
    cpu = 2000 / (time.perf_counter() - t0)
    print(json.dumps({"world": args.world, "gpu_scenarios_per_s": gpu, "gpu_ms": 1e3 * min(times),
                      "count": args.count, "host_mt19937_scenarios_per_s_1_thread": cpu,
                      "ratio": gpu / cpu}), flush=True)


if __name__ == "__main__":
    main()
