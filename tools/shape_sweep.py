"""Launch-shape sweep for one world (bench.py's rollout and one-tick lines): craft_rollout over
(tile, threads, chunk) and craft_step over (tile, obs store), at 65,536 envs with a 16-slot ring,
each shape timed with HIP events over back-to-back launches after a warm pass, two alternating
passes.  Prints one JSON line per pass with µs per launch and GB/s (SURVEY §8(d) bytes).

  python tools/shape_sweep.py --world craft_medium_12x12_w5 [--ticks 20] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", default="craft_medium_12x12_w5")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ring", type=int, default=16)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--rollout", default="16:128:0,16:256:0,16:320:0,16:384:0,16:512:0,32:256:0,"
                                          "32:320:0,32:384:0,32:512:0,64:256:0,64:512:0,32:512:-1,"
                                          "16:512:-1,0:0:0")
    ap.add_argument("--step", default="16:2,32:2,64:2,64:1,0:2")
    args = ap.parse_args()
    n, R = args.envs, args.ring
    sim = CraftSim(args.world, n_envs=n, device=0, pool_capacity=1024)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(grids)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    sim.reset(*synthetic_specs(grids, sim.width, sim.height, n, 0, seed=0, task_ids=tasks))
    F = sim.n_features
    dev = sim.device
    ring = torch.empty((R, n, F), dtype=torch.float32, device=dev)
    rew = torch.empty((R, n), dtype=torch.float32, device=dev)
    done = torch.empty((R, n), dtype=torch.uint8, device=dev)
    succ = torch.empty((R, n), dtype=torch.int8, device=dev)
    bps = bench.bytes_per_env_step(sim.width, sim.height, sim.params["WINDOW_WIDTH"], F)
    ceiling, slot_us = bench.fill_ceiling([ring[r] for r in range(R)], reps=4)
    tick = [0]

    def roll():
        sim.rollout(args.ticks, seed=1, tick0=tick[0], obs=ring, reward=rew, done=done, success=succ)
        tick[0] += args.ticks

    def step():
        r = tick[0] % R
        sim.step(None, seed=1, tick=tick[0], obs=ring[r], reward=rew[r], done=done[r], success=succ[r])
        tick[0] += 1

    for p in range(args.passes):
        out = {"world": args.world, "envs": n, "ring": R, "pass": p, "bytes_per_env_step": bps,
               "fill_gbs": round(ceiling, 1), "fill_slot_us": round(slot_us, 2)}
        for spec in args.rollout.split(","):
            tile, thr, chunk = (int(x) for x in spec.split(":"))
            try:
                sim.tune(tile, 0, 2)
                sim.tune_rollout(chunk, thr)
                shape = sim.rollout_shape()
                us = timed(roll, args.reps)
            except Exception as e:          # a shape the library refuses (LDS, threads)
                out[f"rollout_{spec}"] = {"error": str(e)[:120]}
                continue
            out[f"rollout_{spec}"] = {"shape": shape, "us": round(us, 1),
                                      "gbs": round(bps * n * args.ticks / us / 1e3, 1)}
        sim.tune_rollout(0, 0)
        for spec in args.step.split(","):
            tile, store = (int(x) for x in spec.split(":"))
            try:
                sim.tune(tile, 0, store)
                us = timed(step, args.reps * args.ticks)
            except Exception as e:
                out[f"step_{spec}"] = {"error": str(e)[:120]}
                continue
            out[f"step_{spec}"] = {"shape": sim.tile_shape(), "us": round(us, 2),
                                   "gbs": round(bps * n / us / 1e3, 1)}
        sim.tune(0, 0, 2)
        sim.check()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
