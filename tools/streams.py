"""Diagnostic: one tick of 65536 envs as S sims of 65536/S envs on S streams
(kernels of different streams overlap: one's prologue hides under another's
observation stores)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs

def run(world, S, n=65536, iters=300, warm=30):
    sims, rings, streams = [], [], []
    g = None
    for i in range(S):
        m = n // S
        sim = CraftSim(world, n_envs=m, device=0, env_id_base=i * m, pool_capacity=1024)
        if g is None:
            g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
        sim.load_pool(g)
        sim.reset(*synthetic_specs(g, sim.width, sim.height, m, i * m, 0, [t.id for t in sim.task_manager.dataset_tasks()]))
        sims.append(sim); rings.append([sim.empty_obs() for _ in range(4)])
        streams.append(torch.cuda.Stream() if S > 1 else torch.cuda.current_stream())
    torch.cuda.synchronize()
    st = {"t": 0}
    def tick():
        t = st["t"]
        for i in range(S):
            with torch.cuda.stream(streams[i]):
                sims[i].step(seed=0, tick=t, obs=rings[i][t % 4])
        st["t"] += 1
    for _ in range(warm): tick()
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(iters): tick()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    for s in sims: s.check()
    return round(dt * 1e6, 2)

out = {}
for w in sys.argv[1:] or ["craft_medium_12x12"]:
    out[w] = {f"S{S}": run(w, S) for S in (1, 2, 4)}
print(json.dumps(out, indent=1))
