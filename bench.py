"""Throughput benchmark: env-steps/s of the batched CraftWorld on MI355X.

One "step" = one rollout tick of every env on every GPU: the do_rollout body,
step(), satisfies() and the full features() observation, with auto-reset.
This is BASELINE.json's metric on 12x12 craft_medium with 65536 envs per GPU
(configs[2]); configs[3] is the 8-GPU sharding of the same.

Actions are the hashed random draw (the random-rollout workload), so ticks are
launched K = 32 at a time through craft_rollout. Every tick still does all of
its work and writes its full observation, reward, done and success to HBM; the
envs just stay on chip between ticks. --ticks-per-launch 1 times one craft_step
launch per tick instead.

Inputs (scenario pool, env states) are resident in HBM before the timed region.
Observations stream into a ring of R = 16 device buffers (1.7 GB, 6.6x the
256 MB Infinity Cache), as a trainer's per-tick feature tensors would.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints one JSON line (see the contract in the task description).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def bytes_per_env_step(W, H, window, F):
    """Algorithmic HBM bytes per env-step: 57 B of step state
    (action 1 + agent state r/w 48 + facing/target cells 2 + cell write 1 +
    reward 4 + done 1) + the fp32 observation row F*4 + the pooled window's
    grid cells min(w^2, W) * min(w^2, H)."""
    ww = window * window
    return 57 + 4 * F + min(ww, W) * min(ww, H)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1024)
    p.add_argument("--warmup", type=int, default=64)
    p.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--world", default="craft_medium_12x12")
    p.add_argument("--pool", type=int, default=1024)
    p.add_argument("--ring", type=int, default=16,
                   help="observation buffers cycled per tick (16 x 106 MB: 6.6x the Infinity Cache)")
    p.add_argument("--tile", type=int, default=0, help="envs per workgroup (0 = default)")
    p.add_argument("--obs-store", type=int, default=-1,
                   help="0 write-back, 1 nontemporal, 2 sc1; -1: the measured best for the path "
                        "(nontemporal for craft_step, write-back for craft_rollout)")
    p.add_argument("--ticks-per-launch", type=int, default=32,
                   help="K > 1: craft_rollout runs K ticks per launch (the same work per tick); "
                        "1: one craft_step launch per tick")
    p.add_argument("--rollout-threads", type=int, default=0,
                   help="craft_rollout threads per tile workgroup (0 = 8 per env: 7 streaming waves)")
    p.add_argument("--rollout-chunk", type=int, default=0,
                   help="craft_rollout ticks per dynamically scheduled work unit (0 = the whole launch)")
    p.add_argument("--obs-only", action="store_true",
                   help="diagnostic: skip the reward/done/success rings (not a bench line)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def cpu_baseline(sim, grids, specs, seconds):
    """The CPU oracle (C restatement) on a bounded sample of the same workload,
    one thread per host core given to this job (OMP_NUM_THREADS; 16 on the GPU
    box), each on its own slice of envs; env-steps/s.  ctypes releases the GIL
    around every oracle call, so the threads run in parallel."""
    import threading
    import oracle
    n = 4096
    cores = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    o = oracle.Oracle(sim.config, grids)
    envs = o.init_envs(*[a[:n] for a in specs])
    parts = [envs[i::cores].copy() for i in range(cores)]
    steps = [0] * cores
    t0 = time.perf_counter()
    deadline = t0 + seconds

    def work(i):
        while time.perf_counter() < deadline:
            steps[i] += o.bench(parts[i], 20, seed=1)

    threads = [threading.Thread(target=work, args=(i,)) for i in range(cores)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    dt = time.perf_counter() - t0
    total = sum(steps)
    return {"value": total / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n} envs x {total // n} ticks ({dt:.1f} s) of the same workload "
                      "(12x12 craft_medium, hashed actions, auto-reset): step + satisfies + "
                      f"full features() per env-step, oracle/craft_oracle.c, {cores} threads "
                      "on disjoint env slices"}


def main():
    args = parse()
    from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
    from psketch_amd import distributed as D

    rank, world_size, local_rank = D.world()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    D.init(device=dev)                        # RCCL process group when WORLD_SIZE > 1

    env_base, n = D.env_shard(rank, args.envs)
    sim = CraftSim(args.world, n_envs=n, device=local_rank, env_id_base=env_base,
                   pool_capacity=args.pool)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, args.pool)
    sim.load_pool(grids)
    K = max(1, args.ticks_per_launch)
    obs_store = args.obs_store if args.obs_store >= 0 else (1 if K == 1 else 0)
    sim.tune(args.tile, 0, obs_store)
    sim.tune_rollout(args.rollout_chunk, args.rollout_threads)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, sim.width, sim.height, n, env_base, seed=args.seed,
                            task_ids=tasks)
    sim.reset(*specs)
    F = sim.n_features
    R = args.ring
    if args.steps % K or args.warmup % K:
        raise SystemExit("--steps and --warmup must be multiples of --ticks-per-launch")
    ring = torch.empty((R, n, F), dtype=sim.obs_dtype, device=dev)     # one tick's obs per slot
    reward = torch.empty((R, n), dtype=torch.float32, device=dev)
    done = torch.empty((R, n), dtype=torch.uint8, device=dev)
    success = torch.empty((R, n), dtype=torch.int8, device=dev)

    tick = 0

    def launch():
        """K ticks: one craft_step (K = 1) or one craft_rollout launch."""
        nonlocal tick
        if K == 1:
            r = tick % R
            sim.step(seed=args.seed, tick=tick, obs=ring[r], reward=reward[r], done=done[r],
                     success=success[r])
        else:
            if args.obs_only:
                sim.rollout(K, seed=args.seed, tick0=tick, obs=ring)
            else:
                sim.rollout(K, seed=args.seed, tick0=tick, obs=ring, reward=reward, done=done,
                            success=success)
        tick += K

    for _ in range(args.warmup // K):
        launch()
    sim.check()

    def barrier():
        D.barrier()
        torch.cuda.synchronize()

    # ---- timed region: K ticks, barrier + synchronize on both sides ------------------
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps // K):
        launch()
    barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, dev)

    # ---- per-launch kernel duration, HIP events on the launch stream --------------------
    kstream = torch.cuda.current_stream(dev)
    m = max(1, min(args.steps // K, 400))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(m)]
    torch.cuda.synchronize()
    for a, b in evs:
        a.record(kstream)
        launch()
        b.record(kstream)
    torch.cuda.synchronize()
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))     # per launch (K ticks)

    # ---- scalar episode summary: one RCCL all-reduce of int64[3] --------------------------
    stats = D.reduce_episode_stats(sim.stats()).cpu().tolist()
    sim.check()

    if rank == 0:
        total_steps = n * world_size * args.steps
        value = total_steps / elapsed
        bps = bytes_per_env_step(sim.width, sim.height, sim.params["WINDOW_WIDTH"], F)
        win = sim.params["WINDOW_WIDTH"]
        if K > 1 and not args.rollout_threads and win == 3:
            tile, threads = 32, 512                      # craft_rollout's default shape (split producer)
        else:
            tile = args.tile or {3: 64, 5: 32}.get(win, 16)
            threads = args.rollout_threads or 8 * tile
        achieved = bps * n * K / (kernel_ms * 1e-3) / 1e9
        traffic = None
        workload = f"{args.world}_w{sim.params['WINDOW_WIDTH']}_B{n}_random_rollout_full_features"
        if K > 1:
            workload += f"_K{K}"
        if os.path.exists(args.traffic):
            try:
                tj = json.load(open(args.traffic))
                if tj.get("workload") == workload:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "env-steps/sec (whole node), 12x12 craft_medium, batch=65536",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: 1024 make_data.sample_scenario worlds (RandomState(123)), "
                    "per-env init keyed by global id, splitmix64 actions",
            "config": {"workload": workload, "world": args.world, "envs_per_gpu": n,
                       "global_batch": n * world_size, "window": sim.params["WINDOW_WIDTH"],
                       "n_features": F, "obs_dtype": "fp32", "obs_ring": args.ring,
                       "pool": args.pool, "parallelism": f"env-shard x{world_size}",
                       "max_timesteps": sim.config.max_timesteps, "ticks_per_launch": K,
                       "tile": tile, "rollout_threads": threads,
                       "rollout_chunk": args.rollout_chunk or K, "obs_store": ["write-back", "nontemporal", "sc1"][obs_store]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": (f"tile_kernel<{sim.params['WINDOW_WIDTH']}, MODE_TICK, {tile}>"
                                    if K == 1 else
                                    (f"rollout_split_kernel<{win}, {tile}, {threads}>"
                                     if tile <= 32 and threads >= 320
                                     else f"rollout_kernel<{win}, {tile}, {threads}>")),
                         "kernel_us": kernel_ms * 1e3, "ticks_per_launch": K,
                         "bytes_per_launch": bps * n * K, "bytes_per_env_step": bps},
            "episodes": {"successes": stats[0], "episodes": stats[1], "env_steps": stats[2]},
        }
        if world_size == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(sim, grids, specs, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
