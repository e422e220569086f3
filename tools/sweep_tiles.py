"""Diagnostic sweep of craft_sim_tune(tile_envs, max_resident_per_cu) on the tick kernel."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs

def timeit(fn, iters=300, warm=30):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3

out = {}
for world in sys.argv[1:] or ["craft_medium_12x12"]:
    n = 65536
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, 0, [t.id for t in sim.task_manager.dataset_tasks()]))
    ring = [sim.empty_obs() for _ in range(4)]
    st = {"t": 0}
    def step():
        sim.step(seed=0, tick=st["t"], obs=ring[st["t"] % 4]); st["t"] += 1
    res = {}
    for pol in (0, 1, 2):
        for tile in (32, 64):
            for cap in (0, 4, 6):
                sim.tune(tile, cap, pol)
                res[f"p{pol}_t{tile}_c{cap}"] = round(timeit(step), 2)
    sim.tune(0, 0, 1)
    sim.check()
    out[world] = dict(sorted(res.items(), key=lambda kv: kv[1]))
print(json.dumps(out, indent=1))
