"""Ablation timing of the tick kernel's phases (diagnostic, not a benchmark)."""
import sys, os, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs

def timeit(fn, iters=200, warm=20):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us

res = {}
for world in sys.argv[1:] or ["craft_medium_12x12"]:
    n = 65536
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=1024)
    grids, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(grids)
    specs = synthetic_specs(grids, sim.width, sim.height, n, 0, 0, [t.id for t in sim.task_manager.dataset_tasks()])
    sim.reset(*specs)
    ring = [sim.empty_obs() for _ in range(4)]
    done = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = {"t": 0}
    def step_obs():
        sim.step(seed=0, tick=st["t"], obs=ring[st["t"] % 4], done=done); st["t"] += 1
    def step_noobs():
        sim.step(seed=0, tick=st["t"], done=done); st["t"] += 1
    def observe():
        sim.observe(obs=ring[st["t"] % 4], n=n); st["t"] += 1
    def fill():
        ring[st["t"] % 4].zero_(); st["t"] += 1
    src = torch.empty_like(ring[0])
    def copy():
        ring[st["t"] % 4].copy_(src); st["t"] += 1
    r = {k: timeit(f) for k, f in [("step_obs", step_obs), ("step_noobs", step_noobs),
                                   ("observe", observe), ("torch_zero", fill), ("torch_copy", copy)]}
    r["obs_MB"] = ring[0].numel() * 4 / 1e6
    res[world] = r
    sim.check()
print(json.dumps(res, indent=1))
