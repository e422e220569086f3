"""Where the bench's timed region goes beyond the kernel: one 20-tick craft_rollout
launch at the bench's configuration, repeated as bench.py times it (synchronize,
clock, launch, synchronize, clock), with HIP events around the same launch, the
host-side cost of the launch call alone, and a one-element torch kernel for the
launch + completion latency floor.  Medians over REPS repetitions, microseconds."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psketch_amd import CraftSim, synthetic_specs  # noqa: E402


def main():
    n = int(os.environ.get("ENVS", 65536))
    K = int(os.environ.get("TICKS", 20))
    reps = int(os.environ.get("REPS", 25))
    dev = torch.device("cuda", 0)
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    grids, _ = sim.sample_pool(1024, seed=123)
    spec = synthetic_specs(grids, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()])
    sim.reset(*spec)
    sim.tune(0, 0, 2)
    R = 16
    ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device=dev)
    rr = torch.empty((R, n), dtype=torch.float32, device=dev)
    rd = torch.empty((R, n), dtype=torch.uint8, device=dev)
    rs = torch.empty((R, n), dtype=torch.int8, device=dev)
    tick = [0]

    def launch():
        sim.rollout(K, seed=0, tick0=tick[0], obs=ring, reward=rr, done=rd, success=rs)
        tick[0] += K

    stream = torch.cuda.current_stream(dev)

    # bench.py's sequence on output rings no launch has written yet: one 5-tick warmup launch,
    # then the timed 20-tick launch (which writes ring slots the warmup never touched); the
    # "zeroed" rings were cleared by a fill kernel first
    def first_touch(zero):
        g = torch.empty((R, n, sim.n_features), dtype=torch.float32, device=dev)
        if zero:
            g.zero_()
        torch.cuda.synchronize()
        sim.rollout(5, seed=0, tick0=tick[0], obs=g, reward=rr, done=rd, success=rs)
        tick[0] += 5
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.rollout(K, seed=0, tick0=tick[0], obs=g, reward=rr, done=rd, success=rs)
        tick[0] += K
        torch.cuda.synchronize()
        return 1e6 * (time.perf_counter() - t0), g

    keep = []
    for zero in (False, True, False, True):
        w, g = first_touch(zero)
        keep.append(g)                  # held, so the next ring is fresh memory
        print(f"first-touch ring ({'zeroed' if zero else 'fresh'}): timed launch wall {w:8.1f}", flush=True)
    del keep
    torch.cuda.synchronize()
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    rows = {"wall": [], "host_call": [], "event": [], "wall_with_events": []}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows["wall"].append(1e6 * (t2 - t0))
        rows["host_call"].append(1e6 * (t1 - t0))
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        launch()
        e1.record(stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows["event"].append(1e3 * e0.elapsed_time(e1))
        rows["wall_with_events"].append(1e6 * (t2 - t0))
    # back-to-back launches between one event pair (bench.py's kernel figure)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(8):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    b2b = 1e3 * e0.elapsed_time(e1) / 8
    x = torch.zeros(1, device=dev)
    tiny = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        tiny.append(1e6 * (time.perf_counter() - t0))
    sim.check()
    for k, v in rows.items():
        print(f"{k:18s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  max {max(v):8.1f}")
    print(f"{'back_to_back':18s} {b2b:8.1f} per launch")
    print(f"{'tiny_kernel_wall':18s} median {statistics.median(tiny):8.1f}  min {min(tiny):8.1f}")


if __name__ == "__main__":
    main()
