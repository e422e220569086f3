"""Config 5 timing: 65536 12x12 envs, one rollout tick + DemonstrationTeacher
labels (and find_closest_resources distances) per step, all on the GPU."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs

def timeit(fn, iters=100, warm=10):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3

out = {}
sizes = [int(x) for x in os.environ.get("TEACHER_ENVS", "65536").split(",")]
for world, n in [(w, n) for w in (sys.argv[1:] or ["craft_medium_12x12"]) for n in sizes]:
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.tune_teach(int(os.environ.get("TEACH_KERNEL", "0")))   # craft_step_teach's kernel (0 = auto)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, 0, [t.id for t in sim.task_manager.dataset_tasks()]))
    obs = sim.empty_obs()
    act = torch.empty(n, dtype=torch.int32, device="cuda")
    plen = torch.empty(n, dtype=torch.int32, device="cuda")
    st = {"t": 0}
    def tick():
        sim.step(seed=0, tick=st["t"], obs=obs); st["t"] += 1
    def teach():
        sim.teacher(action_out=act)
    def teach_len():
        sim.teacher(action_out=act, path_len_out=plen)
    def both():
        tick(); teach()
    def fused():
        sim.step(seed=0, tick=st["t"], obs=obs, labels=act); st["t"] += 1
    r = {"tick_us": timeit(tick), "teacher_us": timeit(teach), "teacher_with_len_us": timeit(teach_len),
         "tick_plus_teacher_us": timeit(both), "step_teach_us": timeit(fused)}
    r["config5_env_steps_per_s"] = n / (min(r["tick_plus_teacher_us"], r["step_teach_us"]) * 1e-6)
    sim.check()
    out[f"{world}/{n}"] = {k: round(v, 2) for k, v in r.items()}
print(json.dumps(out, indent=1))
