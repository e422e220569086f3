"""Diagnostic: where a per-unit rollout launch (the default craft_rollout path) spends its
fixed cost: workgroup start spread, time to the first stores, unit durations, and how the
last units end (CRAFT_STAMPS build from tools/rollout_stamps.py --build, never the product).

  python tools/rollout_stamps.py --build       # here (CPU): the diagnostic library
  python tools/unit_stamps.py [n_envs ...]     # on the GPU box (K = 20 and 32 each)"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from psketch_amd import _native  # noqa: E402
_native.LIB_PATH = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag.so")
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402

lib = _native.lib()
lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
R = 16
for n in [int(x) for x in sys.argv[1:]] or [65536, 16384]:
    sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.tune(0, 0, 2)
    sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
    st = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
    lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
    ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
    tick = 0
    for K in (20, 32):
        for rep in range(3):
            st.zero_()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            sim.rollout(K, tick0=tick, obs=ring)
            ev1.record()
            tick += K
            torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.float64)
        s = s[s[:, 15] > 0]
        t0 = s[:, 0].min()
        us = lambda c: (s[:, c] - t0) / 100.0  # noqa: E731
        start, first, end = us(0), us(13), us(15)
        units = s[:, 14].astype(int)
        claims = [(s[i, 1:1 + units[i]] - t0) / 100.0 for i in range(len(s))]
        udur = np.concatenate([np.diff(np.append(c, end[i])) for i, c in enumerate(claims) if len(c)])
        last_claim = np.array([c[-1] if len(c) else 0.0 for c in claims])
        pct = lambda x: "/".join(f"{np.percentile(x, q):.1f}" for q in (10, 50, 90, 100))  # noqa: E731
        print(f"n={n} K={K}: event {ev0.elapsed_time(ev1) * 1e3:.1f} us, span {end.max():.1f} us, "
              f"{len(s)} wg, units/wg {np.bincount(units).tolist()}; p10/50/90/max: start {pct(start)} | "
              f"first stores {pct(first)} | unit {pct(udur)} | last claim {pct(last_claim)} | end {pct(end)}",
              flush=True)
    sim.check()
