"""Where the trainer loop's per-tick time goes (bench.py --workload trainer): device time per
tick of back-to-back sequences queued without any host wait, so that only the kernels and the
gaps between them count:

  policy   the stand-in student alone (addmm + argmax + int32 cast), 40 ticks
  step     craft_step_teach alone (student actions precomputed), 40 ticks
  step_plain / teacher   craft_step_ex and craft_teacher alone
  both     policy then step per tick, 40 ticks (one do_rollout's device work)
  side_teacher   craft_teacher on a side stream beside the policy, then craft_step_ex
  graph    `both` captured as one HIP graph and replayed

    python tools/loop_probe.py [--envs 65536] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n, T = args.envs, 40
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(grids)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, 12, 12, n, 0, seed=0, task_ids=tasks)
    act, _, _ = bench.trainer_policy(sim.n_features, sim.device)
    obs = sim.empty_obs()
    labels = torch.empty((T + 1, n), dtype=torch.int32, device=sim.device)
    acts = torch.randint(0, 5, (n,), dtype=torch.int32, device=sim.device)

    def policy(t):
        return act(obs, t)

    def step(t, a):
        sim.step(a, tick=t, autoreset=True, obs=obs, labels=labels[t + 1])

    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    ev = [torch.cuda.Event() for _ in range(T)]

    def step_plain(t, a):
        sim.step(a, tick=t, autoreset=True, obs=obs)

    def side_tick(t):
        # the teacher's labels of the current states on a side stream, beside the student
        side.wait_stream(main)
        with torch.cuda.stream(side):
            sim.teacher(action_out=labels[t])
        ev[t].record(side)
        a = policy(t)
        main.wait_event(ev[t])
        step_plain(t, a)

    seqs = {
        "policy": lambda: [policy(t) for t in range(T)],
        "step": lambda: [step(t, acts) for t in range(T)],
        "step_plain": lambda: [step_plain(t, acts) for t in range(T)],
        "teacher": lambda: [sim.teacher(action_out=labels[t]) for t in range(T)],
        "both": lambda: [step(t, policy(t)) for t in range(T)],
        "side_teacher": lambda: [side_tick(t) for t in range(T)],
    }
    sim.reset(*specs)
    for f in seqs.values():
        f()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        seqs["both"]()
    seqs["graph"] = g.replay
    out = {"envs": n, "ticks": T}
    for name, f in seqs.items():
        us = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            us.append(e0.elapsed_time(e1) * 1e3 / T)
        out[name + "_us_per_tick"] = round(min(us), 2)
    out["policy_kernels_us"] = bench.profiled_kernel_us(lambda: policy(0), 8, "Cijk")
    sim.check()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
