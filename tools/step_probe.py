"""Diagnostic: one tick per launch at 65,536 envs, HIP events over back-to-back launches
(µs per launch), for each kernel craft_step / craft_step_teach can run, beside the in-situ
write ceiling of the same observation buffers (torch zero_ of one slot per launch).

    python tools/step_probe.py [--world craft_medium_12x12] [--envs 65536] [--ring 16] [--iters 200]

ring 16: every launch writes a fresh 106 MB slot (1.7 GB cycled, 6.6x the Infinity Cache);
ring 1: the same buffer every tick, as a trainer's obs tensor (do_rollout) is."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--world", default="craft_medium_12x12")
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--ring", type=int, nargs="+", default=[16, 1])
    p.add_argument("--iters", type=int, default=200)
    p.add_argument("--teacher", action="store_true")
    p.add_argument("--tiles", type=int, nargs="+", default=[0],
                   help="envs per tile workgroup to time the tick kernel at (0 = the handle's default)")
    p.add_argument("--caps", type=int, nargs="+", default=[0],
                   help="resident workgroups per CU (craft_sim_tune; 0 = as many as fit)")
    p.add_argument("--obs-store", type=int, nargs="+", default=[1],
                   help="observation store policies to time (craft_sim_tune: 0 wb, 1 nt, 2 sc1)")
    args = p.parse_args()
    n = args.envs
    sim = CraftSim(args.world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n,
                               task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
    F = sim.n_features
    st = {"t": 0}

    def timeit(fn, iters):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3

    for R in args.ring:
        ring = torch.empty((R, n, F), dtype=torch.float32, device="cuda")
        rew = torch.empty((R, n), dtype=torch.float32, device="cuda")
        done = torch.empty((R, n), dtype=torch.uint8, device="cuda")
        succ = torch.empty((R, n), dtype=torch.int8, device="cuda")
        lab = torch.empty((R, n), dtype=torch.int32, device="cuda")

        def fill():
            ring[st["t"] % R].zero_()
            st["t"] += 1

        def step():
            r = st["t"] % R
            sim.step(seed=0, tick=st["t"], obs=ring[r], reward=rew[r], done=done[r], success=succ[r])
            st["t"] += 1

        def teach():
            r = st["t"] % R
            sim.step(seed=0, tick=st["t"], obs=ring[r], reward=rew[r], done=done[r], success=succ[r],
                     labels=lab[r])
            st["t"] += 1

        res = {"world": args.world, "envs": n, "ring": R, "fill_us": round(timeit(fill, args.iters), 2)}
        for pol in args.obs_store:
            for tl in args.tiles:
                for cap in args.caps:
                    sim.tune(tl, cap, pol)
                    key = "tile" + (f"{tl}" if tl else "") + (f"_cap{cap}" if cap else "")
                    res[f"{key}_p{pol}_us"] = round(timeit(step, args.iters), 2)
        sim.tune(0, 0, 2)
        if args.teacher:
            for pol in args.obs_store:
                for tl in args.tiles:
                    sim.tune(tl, 0, pol)
                    for k, name in ((2, "teach_tick2"), (1, "teach_tile")):
                        sim.tune_teach(k)
                        res[f"{name}{tl or ''}_p{pol}_us"] = round(timeit(teach, args.iters), 2)
            sim.tune(0, 0, 2)
            sim.tune_teach(0)
        print(json.dumps(res), flush=True)
        del ring, rew, done, succ, lab
    sim.check()


if __name__ == "__main__":
    main()
