"""Configs 3 and 5 end to end: batched do_rollout (psketch_amd.rollout) at
65536 envs with a stand-in student (one linear layer over the device features,
argmax) — eval (config 3: features + reward streamed to the student) and
train with the GPU DemonstrationTeacher labelling every live env each tick and
policy mix 0.5 (config 5, DAgger).

  python tools/rollout_bench.py [--envs 65536] [--world craft_medium_12x12] [--reps 5]

Prints one JSON line per mode: rollouts timed, ticks, env-ticks/s (envs x ticks
processed per second, done envs included, as the reference loop also visits
them) and live env-steps/s (transitions actually taken)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from psketch_amd import CraftSim, synthetic_specs  # noqa: E402
from psketch_amd.rollout import do_rollout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--world", default="craft_medium_12x12")
    ap.add_argument("--pool", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--obs-format", default="f32", choices=["f32", "bf16", "u8"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sim = CraftSim(args.world, n_envs=args.envs, device=0, pool_capacity=args.pool)
    sim.set_obs_format(args.obs_format)
    grids, _ = sim.sample_pool(args.pool, seed=123)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    spec = synthetic_specs(grids, sim.width, sim.height, args.envs, seed=1, task_ids=tasks)
    spec = tuple(torch.as_tensor(a, device=dev) for a in spec)
    gen = torch.Generator(device=dev).manual_seed(0)
    Wt = torch.randn(sim.n_features, 6, device=dev, generator=gen).to(torch.bfloat16)

    def act(obs, t):
        x = obs if obs.dtype == torch.bfloat16 else obs.to(torch.bfloat16)
        return (x @ Wt).argmax(dim=1).to(torch.int32)

    bc = np.random.RandomState(0).binomial(1, 0.5, size=args.envs)
    for mode in ["train", "train_side_stream", "eval"]:
        is_eval = mode == "eval"
        fused = mode != "train_side_stream"
        warm = do_rollout(sim, spec, act, is_eval, behavior_clone=bc, fused_teacher=fused)   # warm-up
        int((warm.n_actions - 1).clamp(min=0).sum())
        torch.cuda.synchronize()
        ticks = steps = 0
        phases = {}
        t0 = time.perf_counter()
        for _ in range(args.reps):
            info = do_rollout(sim, spec, act, is_eval, behavior_clone=bc, timing=phases,
                              fused_teacher=fused)
            ticks += info.ticks
            steps += int((info.n_actions - 1).clamp(min=0).sum())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({
            "mode": mode, "config": "3 (eval)" if is_eval else "5 (teacher, mix 0.5)",
            "teacher": None if is_eval else ("fused into the step" if fused else "side stream"),
            "world": args.world, "obs_format": args.obs_format, "envs": args.envs, "rollouts": args.reps, "ticks": ticks,
            "ms_per_rollout": 1e3 * dt / args.reps, "us_per_tick": 1e6 * dt / ticks,
            "env_ticks_per_s": args.envs * ticks / dt, "live_env_steps_per_s": steps / dt,
            "success_rate": float((info.success > 0).float().mean()),
            "phase_ms_per_rollout": {k: round(1e3 * v / args.reps, 3) for k, v in phases.items()
                                     if k != "ticks"}}), flush=True)


if __name__ == "__main__":
    main()
