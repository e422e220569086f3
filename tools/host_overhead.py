"""Host-side cost per call of the rollout loop's pieces (launch only, no sync):
plain craft_step, craft_step_ex with rollout fields, craft_teacher, a torch
policy, and the per-tick scalar read-back.  Used to size the host overhead of
psketch_amd.rollout.do_rollout against its kernel time."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, synthetic_specs  # noqa: E402


def per_call(fn, reps=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return 1e6 * (t1 - t0) / reps, 1e6 * (t2 - t0) / reps


def main():
    n = 65536
    dev = torch.device("cuda", 0)
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    grids, _ = sim.sample_pool(1024, seed=123)
    spec = synthetic_specs(grids, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()])
    sim.reset(*spec)
    obs = sim.empty_obs()
    acts = torch.zeros(n, dtype=torch.int32, device=dev)
    ref = torch.empty(n, dtype=torch.int32, device=dev)
    bc = torch.ones(n, dtype=torch.uint8, device=dev)
    rec = torch.empty(n, dtype=torch.int32, device=dev)
    live = torch.zeros(1000, dtype=torch.int32, device=dev)
    W = torch.randn(sim.n_features, 6, device=dev).to(torch.bfloat16)
    R = 16
    ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device=dev)
    rr = torch.empty((R, n), dtype=torch.float32, device=dev)
    rd = torch.empty((R, n), dtype=torch.uint8, device=dev)
    rs = torch.empty((R, n), dtype=torch.int8, device=dev)
    rows = {
        "step plain": lambda i: sim.step(seed=0, tick=i, obs=obs),
        "step fused": lambda i: sim.step(acts, tick=i, obs=obs, ref_actions=ref, behavior_clone=bc,
                                         action_record=rec, any_live=live[i:i + 1]),
        "step acts": lambda i: sim.step(acts, tick=i, obs=obs),
        "step +rec": lambda i: sim.step(acts, tick=i, obs=obs, action_record=rec),
        "step +bc": lambda i: sim.step(acts, tick=i, obs=obs, ref_actions=ref, behavior_clone=bc,
                                       action_record=rec),
        "teacher": lambda i: sim.teacher(action_out=ref),
        "rollout K=1": lambda i: sim.rollout(1, tick0=i, obs=ring, reward=rr, done=rd, success=rs),
        "policy": lambda i: (obs.to(torch.bfloat16) @ W).argmax(dim=1).to(torch.int32),
        "scalar read": lambda i: int(live[i]),
    }
    for name, fn in rows.items():
        fn(0)
        host, wall = per_call(fn)
        print(f"{name:12s} host {host:7.1f} us/call   wall {wall:7.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
