"""Throughput benchmark: env-steps/s of the batched CraftWorld on MI355X.

One "step" = one rollout tick of every env on every GPU: the do_rollout body,
step(), satisfies() and the full features() observation, with auto-reset.
This is BASELINE.json's metric on 12x12 craft_medium with 65536 envs per GPU
(configs[2]); configs[3] is the 8-GPU sharding of the same.

Actions are the hashed random draw (the random-rollout workload), so ticks are
launched up to K = 32 at a time through craft_rollout: `--steps S` runs S // K
launches of K ticks plus one launch of the remainder.  Every tick still does
all of its work and writes its full observation, reward, done and success to
HBM; the envs just stay on chip between ticks.  --ticks-per-launch 1 times
one craft_step launch per tick instead.

--workload teacher is configs[4]: every tick also runs the on-GPU
DemonstrationTeacher (teachers/demonstration.py) for every env, the DAgger
label of the next tick's state, in the same launch: up to K ticks per
craft_rollout_teach launch (labels into a ring beside the observations), or with
--ticks-per-launch 1 one craft_step_teach launch per tick (--teacher-mode
separate: craft_teacher + craft_step as two launches).

Inputs (scenario pool, env states) are resident in HBM before the timed region.
Observations stream into a ring of R = 16 device buffers (1.7 GB, 6.6x the
256 MB Infinity Cache), as a trainer's per-tick feature tensors would.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

`--gpus N > 1` without torchrun's environment starts N rank processes itself
(python -m torch.distributed.run) before touching the GPU.  Rank 0 prints one
JSON line (see the contract in the task description).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def bytes_per_env_step(W, H, window, F, teacher=False, obs_bytes=4):
    """Algorithmic HBM bytes per env-step: 57 B of step state
    (action 1 + agent state r/w 48 + facing/target cells 2 + cell write 1 +
    reward 4 + done 1) + the fp32 observation row F*4 + the pooled window's
    grid cells min(w^2, W) * min(w^2, H); the teacher adds the W*H navigation
    grid + the 2 B task id, and its 4 B label ("C5 adds the
    teacher reads").  obs_bytes: bytes per observation element (4 fp32, 2 bf16,
    1 u8: the same exact values, craft_sim_set_obs_format)."""
    ww = window * window
    b = 57 + obs_bytes * F + min(ww, W) * min(ww, H)
    if teacher:
        b += W * H + 2 + 4
    return b


def plan_launches(steps, k):
    """Launch sizes (ticks per launch) covering `steps` ticks: steps // k
    launches of k ticks, then one of the remainder."""
    if steps < 0 or k < 1:
        raise ValueError("need steps >= 0 and ticks-per-launch >= 1")
    full, rem = divmod(steps, k)
    return [k] * full + ([rem] if rem else [])


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1024)
    p.add_argument("--warmup", type=int, default=64)
    p.add_argument("--workload", choices=("rollout", "teacher", "trainer"), default="rollout",
                   help="rollout: configs[2] (random rollout, full features); "
                        "teacher: configs[4] (+ the BFS DemonstrationTeacher label every tick); "
                        "trainer: configs[2]/[4] closed loop, psketch_amd.rollout.do_rollout "
                        "(train mode, fused teacher labels, a fixed on-device student); "
                        "--steps counts rollouts")
    p.add_argument("--rollout-graph", type=int, default=8,
                   help="trainer workload: ticks per captured HIP graph in do_rollout (0 = the "
                        "eager lookahead loop: 2.9-3.2 ms per 40-tick rollout against 2.80-2.91 "
                        "with graphs of 8 ticks, whose loop does not depend on the host's speed)")
    p.add_argument("--trainer-teacher", choices=("fused", "side"), default="fused",
                   help="trainer workload: the teacher fused into the tick (craft_step_teach labels "
                        "the next tick's ref_actions) or forked beside the student's act() on a side "
                        "stream inside the captured graphs (craft_teacher, then craft_step_ex)")
    p.add_argument("--teacher-mode", choices=("fused", "separate"), default="fused",
                   help="teacher workload: one craft_step_teach launch per tick, or craft_teacher "
                        "then craft_step")
    p.add_argument("--teacher-actions", choices=("policy", "label", "mix"), default="policy",
                   help="teacher workload, K-tick launches: the hashed policy (DAgger labels of a "
                        "scripted policy's states), every env acting on its own label "
                        "(make_data.get_reference_actions' demonstrations at scale, auto-reset), or "
                        "behaviour cloning on a fixed half of the envs (imitation.py:56-57)")
    p.add_argument("--teach-table", choices=("auto", "always", "never"), default="auto",
                   help="teacher workload: which teachers read the teacher table (craft_sim_tune_teach "
                        "table 0 / 1 / 2); results are identical")
    p.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--world", default="craft_medium_12x12")
    p.add_argument("--pool", type=int, default=1024)
    p.add_argument("--ring", type=int, default=16,
                   help="observation buffers cycled per tick (16 x 106 MB: 6.6x the Infinity Cache)")
    p.add_argument("--tile", type=int, default=0, help="envs per workgroup (0 = default)")
    p.add_argument("--obs-store", type=int, default=-1,
                   help="0 write-back, 1 nontemporal, 2 sc1; -1: the library default (write-through, "
                        "sc1: the measured best for craft_rollout and for craft_step on a reused buffer; "
                        "nontemporal for craft_rollout_teach)")
    p.add_argument("--ticks-per-launch", type=int, default=32,
                   help="K > 1: craft_rollout runs up to K ticks per launch (the same work per "
                        "tick); 1: one craft_step launch per tick")
    p.add_argument("--rollout-threads", type=int, default=0,
                   help="craft_rollout threads per tile workgroup (0 = the library's default shape)")
    p.add_argument("--rollout-chunk", type=int, default=0,
                   help="craft_rollout ticks per dynamically scheduled work unit (0 = the whole "
                        "launch; -1 = one continuous pipeline per workgroup)")
    p.add_argument("--obs-only", action="store_true",
                   help="diagnostic: skip the reward/done/success rings (not a bench line)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI)")
    p.add_argument("--one-device", action="store_true",
                   help="rehearsal: every rank on cuda:0 (a 1-GPU box; use --dist-backend gloo)")
    p.add_argument("--cpu-seconds", type=float, default=8.0,
                   help="wall seconds of each cpu_baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-profiler", action="store_true",
                   help="price one-tick kernels by HIP events only (for runs under rocprofv3, "
                        "whose tracer the torch profiler would share)")
    p.add_argument("--obs-format", choices=("f32", "bf16", "u8"), default="f32",
                   help="observation element type (the same exact values in each; the metric's "
                        "line is f32, what students/imitation.py:73 feeds the model)")
    p.add_argument("--traffic", default=None,
                   help="PMC traffic JSON (tools/pmc_summary.py); default profiles/pmc_traffic*.json")
    args = p.parse_args(argv)
    # everything is validated here, before any process is started or any GPU call is made
    if args.gpus < 1:
        p.error("--gpus must be >= 1")
    if args.steps < 1 or args.warmup < 0:
        p.error("--steps must be >= 1 and --warmup >= 0")
    if args.ticks_per_launch < 1:
        p.error("--ticks-per-launch must be >= 1")
    if args.envs < 1 or args.pool < 1 or args.ring < 1:
        p.error("--envs, --pool and --ring must be >= 1")
    if args.tile not in (0, 16, 32, 64):
        p.error("--tile must be 0, 16, 32 or 64")
    if args.workload == "teacher" and args.teacher_mode == "separate":
        args.ticks_per_launch = 1                 # craft_teacher + craft_step: one tick per launch pair
    if args.teacher_actions != "policy" and (args.workload != "teacher" or args.ticks_per_launch < 2):
        p.error("--teacher-actions label / mix: the teacher workload's K-tick launches only")
    return args


def world_check(args, env=None):
    """What to do about the process topology: "spawn" (no torchrun environment
    and --gpus > 1: start the ranks), "run", or an error message when
    WORLD_SIZE disagrees with --gpus."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if args.gpus > 1 else "run"
    if int(ws) != args.gpus:
        return f"WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a different node size"
    return "run"


def spawn_ranks(args, argv):
    """Start one rank per GPU with torch.distributed.run as a CHILD process (this
    process has not touched the GPU) and return its exit code."""
    import torch
    have = torch.cuda.device_count()          # counts devices without initialising HIP
    if have < args.gpus and not args.one_device:
        print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---- CPU baseline ----------------------------------------------------------------------------
def _cores():
    n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_baseline_c(cfg, grids, specs, env_id_base, seed, seconds, teacher=False, ring=16):
    """The C restatement (oracle/craft_oracle.c oracle_bench) on a bounded sample of the same
    workload, one thread per host core given to this job, each on its own contiguous slice of
    global env ids, every env writing its own observation row into ring slot tick % ring of a
    per-thread ring (16 slots x 256 envs x 1616 B = 6.6 MB per thread, 106 MB over 16 threads:
    past the threads' cache share, so the stores reach DRAM as the GPU's do); with `teacher`
    (configs[4]) the DemonstrationTeacher labels every env's new state every tick, as
    craft_step_teach does.  env-steps/s.  ctypes releases the GIL around each call."""
    import threading
    import oracle
    oracle.build()
    n = 4096
    cores = _cores()
    o = oracle.Oracle(cfg, grids)
    envs = o.init_envs(*[a[:n] for a in specs])
    bounds = np.linspace(0, n, cores + 1).astype(int)
    parts = [(envs[bounds[i]:bounds[i + 1]].copy(), env_id_base + int(bounds[i])) for i in range(cores)]
    bufs = [o.bench_buffers(len(p[0]), ring, teacher) for p in parts]
    steps = [0] * cores
    ticks = [0] * cores
    t0 = time.perf_counter()
    deadline = t0 + seconds

    def work(i):
        e, base = parts[i]
        while time.perf_counter() < deadline:
            steps[i] += o.bench(e, base, ticks[i], 4, seed, bufs[i])
            ticks[i] += 4

    threads = [threading.Thread(target=work, args=(i,)) for i in range(cores)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    dt = time.perf_counter() - t0
    total = sum(steps)
    what = ("step + satisfies + full features() + the DemonstrationTeacher's BFS label of every "
            "env's new state" if teacher else "step + satisfies + full features()")
    return {"value": total / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n} envs x {total // n} ticks ({dt:.1f} s) of the same workload (12x12 "
                      f"craft_medium, global-id hashed actions, auto-reset): {what}, obs/reward/"
                      f"done/success written to each env's own row, observations cycled through a "
                      f"{ring}-slot ring per thread ({ring * 256 * 1616 // 2**20} MB per thread of "
                      f"256 envs: stores reach DRAM); oracle/craft_oracle.c (gcc -O3), {cores} "
                      "threads on contiguous env slices"}


def cpu_baseline_numpy(cfg, grids, specs, env_id_base, seed, seconds):
    """The pure-Python/numpy restatement (oracle/craft_numpy.py: the reference's
    per-env loop and data layout) over all the job's cores as processes."""
    from oracle import craft_numpy
    n = 1024
    rate, procs, total, dt = craft_numpy.bench(cfg, grids, np.stack(specs, 1)[:n], env_id_base,
                                               seed, seconds)
    return {"value": rate, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "sample": f"{n} envs, {total} env-steps in {dt:.1f} s: oracle/craft_numpy.py "
                      "(float64 one-hot grids, per-env step/features/satisfies as in "
                      f"worlds/craft.py), {procs} processes on contiguous env slices"}


# ---- the GPU run -----------------------------------------------------------------------------
def fill_ceiling(bufs, reps=8):
    """In-situ write ceiling: GB/s of torch's zero_ fill over the same buffers the
    timed kernels write, one fill launch per buffer, cycled like the kernels cycle them, timed
    with HIP events after one warm pass.  Returns (GB/s, µs per buffer)."""
    import torch
    for b in bufs:
        b.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for b in bufs:
            b.zero_()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    nbytes = sum(b.numel() * b.element_size() for b in bufs) * reps
    return nbytes / (ms * 1e-3) / 1e9, ms * 1e3 / (reps * len(bufs))



def pmc_traffic(args, workload, k):
    """HBM bytes per launch of this workload's dominant kernel from the PMC passes
    (tools/profile.sh + tools/pmc_summary.py -> profiles/pmc_traffic.json), or None."""
    tpath = args.traffic or os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(tpath) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None
    for e in (tj if isinstance(tj, list) else [tj]):
        if e.get("workload") == workload and e.get("ticks_per_launch", 1) == k:
            return e.get("hbm_bytes_per_launch")
    return None


def hbm_rate(traffic, kernel_us):
    """The real HBM rate beside the algorithmic one: the PMC bytes per launch (FETCH_SIZE +
    WRITE_SIZE, corrected) over the kernel's launch time, and its fraction of the 8 TB/s peak.
    Differs from `achieved` where algorithmic bytes never reach HBM (config 5's teacher reads of
    the navigation grid: the pool row, L2-resident) or where a kernel re-reads."""
    if not traffic or not kernel_us:
        return {"achieved_hbm_gbs": None, "hbm_frac": None}
    gbs = traffic / (kernel_us * 1e-6) / 1e9
    return {"achieved_hbm_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS}


def profiled_kernel_us(fn, m, name):
    """Mean device duration (µs) of the kernels whose name contains `name` over m calls of fn(),
    from the torch profiler's device activity (roctracer on ROCm: the same launch records as
    rocprofv3 --kernel-trace), or None when the profiler yields no such kernel.  Unlike a pair of
    HIP events around back-to-back launches it excludes the dispatch gaps between launches."""
    import torch
    from torch.profiler import ProfilerActivity, profile
    try:
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(m):
                fn()
            torch.cuda.synchronize()
        durs = [e.device_time if hasattr(e, "device_time") else e.cuda_time
                for e in prof.events() if name in e.name and getattr(e, "device_type", None) is not None
                and str(e.device_type).endswith("CUDA")]
        durs = [d for d in durs if d and d > 0]
        return float(np.mean(durs)) if durs else None
    except Exception:                               # no device tracer on this build
        return None



def _init_ranks(args):
    """torch.distributed.run's environment -> (rank, world_size, local_rank, device), with the
    process group (RCCL when WORLD_SIZE > 1) initialised; the world size reported is the process
    group's own (dist.get_world_size), which must agree with the launcher's."""
    import torch
    from psketch_amd import distributed as D
    rank, world_size, local_rank = D.world()
    if args.one_device:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    D.init(device=dev, backend=args.dist_backend)
    if D.group_size() != world_size:
        raise RuntimeError(f"process group has {D.group_size()} ranks, WORLD_SIZE={world_size}")
    return rank, D.group_size(), local_rank, dev


def run(args):
    import torch
    from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
    from psketch_amd import distributed as D

    rank, world_size, local_rank, dev = _init_ranks(args)

    teacher = args.workload == "teacher"
    K = args.ticks_per_launch
    timed_plan = plan_launches(args.steps, K)
    warm_plan = plan_launches(args.warmup, K)
    k_eff = timed_plan[0]                     # = min(K, steps): the launch the events time

    env_base, n = D.env_shard(rank, args.envs)
    sim = CraftSim(args.world, n_envs=n, device=local_rank, env_id_base=env_base,
                   pool_capacity=args.pool)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, args.pool)
    sim.load_pool(grids)
    if args.obs_store >= 0 or args.tile:
        obs_store = args.obs_store if args.obs_store >= 0 else 2
        sim.tune(args.tile, 0, obs_store)
    else:                                     # the library's defaults (include/craft.h craft_sim_tune)
        obs_store = 1 if args.workload == "teacher" and args.ticks_per_launch > 1 else 2
    sim.set_obs_format(args.obs_format)
    sim.tune_rollout(args.rollout_chunk, args.rollout_threads)
    sim.tune_teach(0, 0, ("auto", "always", "never").index(args.teach_table))
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, sim.width, sim.height, n, env_base, seed=args.seed,
                            task_ids=tasks)
    sim.reset(*specs)
    F = sim.n_features
    R = args.ring
    ring = torch.empty((R, n, F), dtype=sim.obs_dtype, device=dev)     # one tick's obs per slot
    reward = torch.empty((R, n), dtype=torch.float32, device=dev)
    done = torch.empty((R, n), dtype=torch.uint8, device=dev)
    success = torch.empty((R, n), dtype=torch.int8, device=dev)
    labels = torch.empty((R, n), dtype=torch.int32, device=dev)
    # --teacher-actions label / mix: the labels of the reset states, then each launch's last
    label_in = [sim.teacher()[0].clone()] if teacher and args.teacher_actions != "policy" else [None]
    bc_mask = (torch.as_tensor(np.random.RandomState(args.seed + env_base).binomial(1, 0.5, size=n)
                               .astype(np.uint8), device=dev) if teacher and args.teacher_actions == "mix" else None)

    tick = 0

    def launch(k):
        """k ticks: one craft_rollout launch, or k craft_step (+ teacher) launches."""
        nonlocal tick
        if K == 1:
            for _ in range(k):
                r = tick % R
                if teacher and args.teacher_mode == "fused":
                    # the tick, then the DAgger label of every env's new state, one launch
                    sim.step(seed=args.seed, tick=tick, obs=ring[r], reward=reward[r], done=done[r],
                             success=success[r], labels=labels[r])
                else:
                    if teacher:
                        sim.teacher(action_out=labels[r])  # DAgger label of the tick's state
                    sim.step(seed=args.seed, tick=tick, obs=ring[r], reward=reward[r],
                             done=done[r], success=success[r])
                tick += 1
        elif teacher:
            # k ticks and every env's label per tick, one craft_rollout_teach launch; with label
            # actions the previous launch's last labels are this one's label_in
            src = {}
            if args.teacher_actions != "policy":
                src = dict(label_in=label_in[0], label_actions=args.teacher_actions == "label",
                           behavior_clone=bc_mask if args.teacher_actions == "mix" else None)
            sim.rollout_teach(k, seed=args.seed, tick0=tick, obs=ring, reward=reward, done=done,
                              success=success, labels=labels, **src)
            tick += k
            label_in[0] = labels[(tick - 1) % R]
        else:
            if args.obs_only:
                sim.rollout(k, seed=args.seed, tick0=tick, obs=ring)
            else:
                sim.rollout(k, seed=args.seed, tick0=tick, obs=ring, reward=reward, done=done,
                            success=success)
            tick += k

    # the in-situ write ceiling of the same ring, slot by slot (before the warmup, so that the
    # timed region follows the kernel's own warm launches)
    ceiling_gbs, ceiling_slot_us = fill_ceiling([ring[r] for r in range(R)], reps=4)
    for k in warm_plan:
        launch(k)
    sim.check()

    def barrier():
        D.barrier()
        torch.cuda.synchronize()

    # ---- timed region: exactly args.steps ticks, barrier + synchronize on both sides.  Each
    # rank's clock stops when its own GPU is done (synchronize), before the closing barrier's
    # exchange; the line reports the slowest rank. -------------------------------------------
    barrier()
    t0 = time.perf_counter()
    for k in timed_plan:
        launch(k)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max_over_ranks(t1 - t0, dev)
    local_s = t1 - t0

    # ---- per-launch kernel duration, HIP events on the launch stream (outside the timed
    # region): m back-to-back launches of k_eff ticks (as many as the timed region had, at
    # least 8) between one pair of events, so no event sits between two launches -------------
    kstream = torch.cuda.current_stream(dev)
    m = min(max(len(timed_plan), 8), 200)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record(kstream)
    for _ in range(m):
        launch(k_eff)
    ev1.record(kstream)
    torch.cuda.synchronize()
    kernel_ms = ev0.elapsed_time(ev1) / m                                # per launch (k_eff ticks)
    # one launch per tick (craft_step / craft_step_teach): price the kernel's own duration (the
    # profiler's device records, as rocprof reports them), not launches plus dispatch gaps
    prof_us = None
    if K == 1 and not args.no_kernel_profiler:
        if teacher and args.teacher_mode == "fused":
            pname = sim.step_shape(teach=True)[0]
        else:
            pname = sim.step_shape()[0]
        prof_us = profiled_kernel_us(lambda: launch(1), min(m, 64), pname)

    # ---- scalar episode summary: one RCCL all-reduce of int64[3]; every rank's own summary,
    # shard and clock gathered over the process group for the line ---------------------------
    local = sim.stats()
    report = D.run_report(local_s, env_base, n, local.cpu().tolist(), dev)
    stats = D.reduce_episode_stats(local).cpu().tolist()
    sim.check()

    if rank == 0:
        win = sim.params["WINDOW_WIDTH"]
        total_steps = n * world_size * args.steps
        value = total_steps / elapsed
        obs_bytes = {"f32": 4, "bf16": 2, "u8": 1}[sim.obs_format]
        bps = bytes_per_env_step(sim.width, sim.height, win, F, teacher, obs_bytes)
        obs_dtype = {"f32": "fp32", "bf16": "bf16", "u8": "u8"}[sim.obs_format]
        if K > 1 and teacher:
            tile = 32 if win == 3 else 16
            nw = sim.teach_words()
            la = "true" if args.teacher_actions != "policy" else "false"   # (labels feed actions: the LA instantiation)
            kname = f"rollout_teach_kernel<{win}, {tile}, {nw}, {la}>"
            shape = {"tile": tile, "rollout_threads": 512, "teacher_wave": 1,
                     "rollout_unit_ticks": k_eff, "kernel": "rollout_teach_kernel (craft_rollout_teach)"}
        elif K > 1:
            tile, threads, split = sim.rollout_shape()          # what the library launched
            fmt = {"f32": "0", "bf16": "1", "u8": "2"}[sim.obs_format]
            kname = (f"rollout_split_kernel<{win}, {tile}, {threads}, {fmt}, *, false>" if split
                     else f"rollout_kernel<{win}, {tile}, {threads}, {fmt}, *, false>")
            shape = {"tile": tile, "rollout_threads": threads, "split_producer": split,
                     "rollout_unit_ticks": (k_eff if args.rollout_chunk <= 0 else args.rollout_chunk),
                     "rollout_pipeline": "continuous" if args.rollout_chunk == -1 else "per unit"}
        else:
            # what the library launches (craft_sim_step_shape), not a mirror of its defaults
            kn, kenvs, lanes = sim.step_shape(teach=teacher and args.teacher_mode == "fused")
            kname = f"{kn}<{win}> ({kenvs} envs per workgroup"
            kname += f", {lanes} teacher lanes per env) (craft_step_teach)" if lanes else ") (craft_step)"
            if teacher and args.teacher_mode != "fused":
                kname += " + teacher_kernel"
            shape = {"tile": kenvs, "kernel": kn, "teacher_lanes": lanes}
        kernel_us_priced = prof_us if prof_us is not None else kernel_ms * 1e3
        achieved = bps * n * k_eff / (kernel_us_priced * 1e-6) / 1e9
        workload = f"{args.world}_w{win}_B{n}_" + (
            "teacher_labels_full_features" if teacher else "random_rollout_full_features")
        if K > 1:
            workload += f"_K{K}"
        if sim.obs_format != "f32":
            workload += f"_obs_{sim.obs_format}"
        if teacher:
            workload += "_" + args.teacher_mode
            if args.teacher_actions != "policy":
                workload += "_" + ("label_actions" if args.teacher_actions == "label" else "bc_mix")
        traffic = pmc_traffic(args, workload, k_eff)
        if teacher and K > 1:
            bound = "hbm (the teacher's walk and BFS run in the interval's slack beside the stream)"
        elif teacher:
            bound = ("latency: the tick's prologue plus the BFS beside the observation stream "
                     "(store floor of the tick's bytes at the in-situ ceiling below)")
        elif K == 1:
            bound = "hbm (one launch per tick: plus the tick's latency-bound prologue)"
        else:
            bound = "hbm"
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
            "dtype": obs_dtype,
            "data": "synthetic: 1024 make_data.sample_scenario worlds (RandomState(123)), "
                    "per-env init keyed by global id, splitmix64 actions",
            "config": dict({"workload": workload, "world": args.world, "envs_per_gpu": n,
                            "global_batch": n * world_size, "window": win,
                            "n_features": F, "obs_dtype": obs_dtype,
                            "state_dtype": "u8 (exact small integers; the reference's float64 "
                                           "arrays hold the same values)",
                            "obs_ring": args.ring, "pool": args.pool,
                            "parallelism": f"env-shard x{world_size}",
                            "max_timesteps": sim.config.max_timesteps, "ticks_per_launch": K,
                            "launches": len(timed_plan), "teach_table": args.teach_table,
                            "obs_store": ["write-back", "nontemporal", "sc1"][obs_store]}, **shape),
            "roofline": {"bound": bound, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                         "kernel_us": kernel_us_priced,
                         "kernel_us_source": "torch profiler device records (as rocprof)" if prof_us
                         is not None else "HIP events over back-to-back launches",
                         "kernel_us_events": kernel_ms * 1e3, "ticks_per_launch": k_eff,
                         "bytes_per_launch": bps * n * k_eff, "bytes_per_env_step": bps,
                         "ceiling_gbs": ceiling_gbs, "frac_of_ceiling": achieved / ceiling_gbs,
                         **hbm_rate(traffic, kernel_us_priced),
                         "ceiling": f"torch zero_ of each {R}-slot ring buffer in turn "
                                    f"({ceiling_slot_us:.1f} us per {ring[0].numel() * ring.element_size() / 1e6:.0f} MB "
                                    "slot), measured in this run before the timed region"},
            "episodes": {"successes": stats[0], "episodes": stats[1], "env_steps": stats[2]},
            "dist": report,
        }
        if world_size == 1 and not args.no_cpu_baseline:
            c_leg = cpu_baseline_c(sim.config, grids, specs, env_base, args.seed, args.cpu_seconds,
                                   teacher=teacher)
            if teacher:                     # the numpy restatement has no teacher: no like-for-like leg
                np_leg = None
            else:
                try:
                    np_leg = cpu_baseline_numpy(sim.config, grids, specs, env_base, args.seed,
                                                args.cpu_seconds)
                except Exception as e:      # the C leg stands alone if process pools are refused
                    np_leg = {"error": f"{type(e).__name__}: {e}"}
            if teacher and args.teacher_actions != "policy":
                c_leg["note"] = ("the C leg acts on the hashed policy, not on the labels: the same "
                                 "step, features and teacher work per env-step")
            line["cpu_baseline"] = dict(c_leg, **({"python_numpy": np_leg} if np_leg is not None else {}))
        print(json.dumps(line), flush=True)
    D.shutdown()


# ---- the closed-loop trainer workload (--workload trainer) ------------------------------------
def trainer_policy(n_features, device, seed=7, L=4):
    """A fixed student with tests/golden/imitation_rollout.npz's shape: scores = obs @ W[t % L] * 8
    + bias, argmax over the 6 actions; small integer weights, so the fp32 GEMM is exact and the
    policy has no side effects (do_rollout's lookahead may queue a tick ahead)."""
    import torch
    rng = np.random.RandomState(seed)
    W = rng.randint(-3, 4, size=(L, n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, -8])
    Wd = torch.as_tensor(W, dtype=torch.float32, device=device)
    bd = torch.as_tensor(bias, dtype=torch.float32, device=device)

    def act(obs, t):
        return torch.addmm(bd, obs, Wd[t % L], alpha=8).argmax(dim=1).to(torch.int32)
    return act, W, bias


def cpu_baseline_trainer(cfg, grids, specs, W, bias, bc, seconds, n=256, max_rollouts=64):
    """oracle/rollout_oracle.py's do_rollout (trainers/imitation.py:18-101 one env at a time,
    with the C oracle's step / features / DemonstrationTeacher) and the same fixed policy in
    numpy, on rollouts of n envs of the same workload, one core.  value = live env-steps/s:
    num_interactions (imitation.py:54, one per env that has not finished, per tick: the env-ticks
    the reference steps or ends), as the GPU line counts; slot_env_steps_per_s counts every env
    slot every tick (n x the rollout's ticks = n x its student.receive calls)."""
    import oracle
    from oracle import rollout_oracle
    oracle.build()
    o = oracle.Oracle(cfg, grids)
    spec = np.stack(specs, axis=1)
    pol = rollout_oracle.fake_policy(W, bias)
    live = slots = ticks = rollouts = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and rollouts < max_rollouts:
        lo = (rollouts * n) % len(spec)
        sub = spec[lo:lo + n]
        info = rollout_oracle.do_rollout(o, sub, pol, False, bc_mask=bc[lo:lo + n])
        live += info["num_interactions"]
        ticks += len(info["received"])                  # one receive() per tick (imitation.py:77)
        slots += len(sub) * len(info["received"])
        rollouts += 1
    dt = time.perf_counter() - t0
    return {"value": live / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "slot_env_steps_per_s": slots / dt, "live_env_steps": live, "slot_env_ticks": slots,
            "ticks": ticks, "rollouts": rollouts,
            "sample": f"{rollouts} rollouts of {n} envs ({ticks} ticks, {live} live env-steps = "
                      f"num_interactions, {slots} env-slot ticks, {dt:.1f} s): "
                      "oracle/rollout_oracle.py do_rollout (train mode, the C oracle's "
                      "DemonstrationTeacher every live env every tick, behaviour cloning) with "
                      "the same fixed policy in numpy, one core"}


def run_trainer(args):
    """configs[2]/[4] as a trainer runs them: psketch_amd.rollout.do_rollout (the whole
    ImitationTrainer.do_rollout, trainers/imitation.py:18-101) per --steps rollout, train
    mode: every tick the student's act() on the device observations, then one
    craft_step_teach launch (behaviour cloning, the action record, the all(done) flag and the
    DemonstrationTeacher's labels for the next tick), the flag read one tick behind
    (lookahead).  Value = live env-steps / s over every rank: num_interactions
    (imitation.py:54), the env-ticks of envs that have not finished, which are what the reference
    steps (a done env is skipped, imitation.py:63-73); slot_env_steps_per_s also counts the frozen
    slots the batched loop carries until every episode has ended."""
    import torch
    from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
    from psketch_amd import distributed as D
    from psketch_amd.rollout import do_rollout

    rank, world_size, local_rank, dev = _init_ranks(args)
    env_base, n = D.env_shard(rank, args.envs)
    sim = CraftSim(args.world, n_envs=n, device=local_rank, env_id_base=env_base,
                   pool_capacity=args.pool)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, args.pool)
    sim.load_pool(grids)
    if args.obs_store >= 0:
        sim.tune(args.tile, 0, args.obs_store)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    specs = synthetic_specs(grids, sim.width, sim.height, n, env_base, seed=args.seed,
                            task_ids=tasks)
    spec_d = [torch.as_tensor(a, device=dev) for a in specs]
    act, W, bias = trainer_policy(sim.n_features, dev, seed=args.seed + 7)
    bc = np.random.RandomState(args.seed + env_base).binomial(1, 0.5, size=n)
    bc_d = torch.as_tensor(bc, device=dev)
    received = []

    def receive(r):                                  # student.receive keeps the labels
        received.append(r)

    fused = args.trainer_teacher == "fused"

    def rollout():
        received.clear()
        return do_rollout(sim, spec_d, act, False, behavior_clone=bc_d, receive=receive,
                          lookahead=fused, graph=args.rollout_graph, fused_teacher=fused)

    for _ in range(args.warmup):
        rollout()
    sim.check()
    ceil_buf = sim.empty_obs()          # do_rollout rewrites one observation buffer every tick
    ceiling_gbs, ceiling_us = fill_ceiling([ceil_buf], reps=16)
    del ceil_buf
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ticks = live = 0
    for _ in range(args.steps):
        info = rollout()
        ticks += info.ticks
        live += info.num_interactions
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max_over_ranks(t1 - t0, dev)
    local = [n * ticks, live, ticks]
    report = D.run_report(t1 - t0, env_base, n, local, dev,
                          names=("slot_env_ticks", "live_env_steps", "ticks"))
    tot = D.reduce_episode_stats(torch.as_tensor(local, dtype=torch.int64, device=dev)).cpu().tolist()

    # ---- per-tick split, outside the timed region: HIP events at the start and the end of the
    # student's kernels of every tick of one more rollout; the env launch (craft_step_teach)
    # runs between one tick's policy end and the next one's start ----
    marks = []

    def timed_act(obs, t):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = act(obs, t)
        b.record()
        marks.append((a, b))
        return out

    torch.cuda.synchronize()
    w0 = time.perf_counter()
    info = do_rollout(sim, spec_d, timed_act, False, behavior_clone=bc_d, receive=receive,
                      lookahead=fused, fused_teacher=fused)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - w0) / max(1, info.ticks)
    pol_us = float(np.mean([a.elapsed_time(b) for a, b in marks[:info.ticks]])) * 1e3
    env_us = float(np.mean([marks[k][1].elapsed_time(marks[k + 1][0])
                            for k in range(min(info.ticks, len(marks) - 1))])) * 1e3
    sim.check()
    # the tick kernel's own device duration over one more rollout (as rocprof prices it: without
    # the dispatch gaps env_kernel above includes)
    kname, kenvs, lanes = sim.step_shape(teach=fused)
    prof_us = None if args.no_kernel_profiler else profiled_kernel_us(
        lambda: do_rollout(sim, spec_d, act, False, behavior_clone=bc_d, receive=receive,
                           lookahead=fused, fused_teacher=fused), 1, kname)
    kernel_us = prof_us if prof_us else env_us

    if rank == 0:
        win = sim.params["WINDOW_WIDTH"]
        F = sim.n_features
        bps = bytes_per_env_step(sim.width, sim.height, win, F, True, 4)
        achieved = bps * n / (kernel_us * 1e-6) / 1e9
        workload = f"{args.world}_w{win}_B{n}_trainer_closed_loop_train_{args.trainer_teacher}_teacher"
        value = tot[1] / elapsed                     # live env-steps (num_interactions)
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
            "dtype": "fp32",
            "data": "synthetic: 1024 make_data.sample_scenario worlds (RandomState(123)), per-env "
                    "init keyed by global id, a fixed integer-weight linear student, behaviour "
                    "cloning mix 0.5",
            "config": {"workload": workload,
                       "world": args.world, "envs_per_gpu": n, "global_batch": n * world_size,
                       "window": win, "n_features": F, "max_timesteps": sim.config.max_timesteps,
                       "rollouts": args.steps, "ticks": tot[2], "step": "one do_rollout "
                       "(ticks until every episode has ended, <= max_timesteps); value counts live "
                       "env-steps (num_interactions, imitation.py:54: envs not yet done), "
                       "slot_env_steps_per_s every env slot every tick", "lookahead": True,
                       "rollout_graph_ticks": args.rollout_graph, "teacher": args.trainer_teacher,
                       "parallelism": f"env-shard x{world_size}"},
            "slot_env_steps_per_s": tot[0] / elapsed,
            "dist": report,
            "per_tick_us": {"timed_wall": elapsed * 1e6 / max(1, tot[2] // world_size),
                            "eager_wall": wall * 1e6, "policy": pol_us, "env": env_us,
                            "env_kernel_device": kernel_us,
                            "host_gap": wall * 1e6 - pol_us - env_us,
                            "note": "timed_wall: the timed region per tick; the rest from one "
                                    "instrumented eager (lookahead, no graph) rollout after it: "
                                    "HIP events at the start and end of the student's kernels; "
                                    "env = policy end to the next tick's policy start (the "
                                    "craft_step_teach launch, its any-live flag stored into mapped "
                                    "host memory, and the dispatch gaps around it); "
                                    "env_kernel_device = the kernel's own duration"},
            "roofline": {"bound": "latency (tick prologue + BFS beside the observation stream)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(args, workload, 1),
                         **hbm_rate(pmc_traffic(args, workload, 1), kernel_us),
                         "kernel": (f"{kname} (craft_step_teach, {kenvs} envs, {lanes} teacher lanes)" if fused
                                    else f"{kname} (craft_step_ex, {kenvs} envs; craft_teacher beside act())"),
                         "kernel_us": kernel_us,
                         "kernel_us_source": ("torch profiler device records (as rocprof)" if prof_us
                                              else "HIP events: policy end to next policy start"),
                         "bytes_per_env_step": bps,
                         "bytes_per_launch": bps * n, "ceiling_gbs": ceiling_gbs,
                         "frac_of_ceiling": achieved / ceiling_gbs,
                         "ceiling": f"torch zero_ of one [n, F] fp32 buffer rewritten in place, as "
                                    f"do_rollout's observation buffer is ({ceiling_us:.1f} us per fill)"},
        }
        if world_size == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_trainer(sim.config, grids, specs, W, bias, bc,
                                                        args.cpu_seconds)
        print(json.dumps(line), flush=True)
    D.shutdown()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    what = world_check(args)
    if what == "spawn":
        return spawn_ranks(args, argv)
    if what != "run":
        print(f"bench.py: {what}", file=sys.stderr)
        return 2
    if args.workload == "trainer":
        run_trainer(args)
    else:
        run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
