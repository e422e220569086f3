"""Diagnostic: one tick at 65536 envs through craft_step (the one-tile kernel) against
craft_rollout with K = 1 (per-unit and continuous pipelines), HIP events over 200
back-to-back launches each."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs

n = int(os.environ.get("N_ENVS", "65536"))
sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
sim.load_pool(g)
sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
R = 16
ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
rew = torch.empty((R, n), dtype=torch.float32, device="cuda")
done = torch.empty((R, n), dtype=torch.uint8, device="cuda")
succ = torch.empty((R, n), dtype=torch.int8, device="cuda")
st = {"t": 0}

def step():
    r = st["t"] % R
    sim.step(seed=0, tick=st["t"], obs=ring[r], reward=rew[r], done=done[r], success=succ[r]); st["t"] += 1

def roll():
    sim.rollout(1, seed=0, tick0=st["t"], obs=ring, reward=rew, done=done, success=succ); st["t"] += 1

def timeit(fn, iters=200):
    for _ in range(20): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3

for obs_store in (1, 2):
    sim.tune(0, 0, obs_store)
    print(f"store {obs_store}: craft_step {timeit(step):.2f} us", flush=True)
    for chunk in (0, -1):
        sim.tune_rollout(chunk, 0)
        print(f"store {obs_store}: craft_rollout K=1 chunk {chunk}: {timeit(roll):.2f} us", flush=True)
sim.check()
