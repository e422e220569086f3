"""Diagnostic: where the split-producer rollout kernel's time goes, per role
(CRAFT_STAMPS build of tools/rollout_stamps.py, never the product).

Per launch: span and workgroup durations; per interval (one tick of one tile)
the mean time wave 0 spends producing (tile switch + transition), wave 1
scattering, wave 2 streaming, and waves 0 / 1 waiting at the barrier.

  python tools/rollout_stamps.py --build     # here (CPU): the diagnostic library
  python tools/split_stamps.py [K ...]        # on the GPU box"""
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
n, R = 65536, 16
sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
sim.load_pool(g)
sim.tune(0, 0, 0)
sim.tune_rollout(-1, 0)                 # the continuous pipeline (the stamped path)
sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
st = torch.zeros((n // 32, 16), dtype=torch.int64, device="cuda")   # 16 words per workgroup
lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
tick = 0
for K in [int(x) for x in sys.argv[1:]] or [20, 32]:
    for rep in range(3):
        st.zero_()
        sim.rollout(K, tick0=tick, obs=ring)
        tick += K
        torch.cuda.synchronize()
    s = st.cpu().numpy().astype(np.float64)
    s = s[s[:, 6] > 0]
    t0 = s[:, 0].min()
    start, end = (s[:, 0] - t0) / 100.0, (s[:, 6] - t0) / 100.0
    dur = end - start
    tiles = n // 32 / len(s)
    per = s[:, 1:6].mean(0) / 100.0 / (K * tiles)
    sw = s[:, 7].mean() / 100.0 / tiles
    vm, pub, ld = (s[:, c].mean() / 100.0 / tiles for c in (8, 9, 10))
    dma = s[:, 11].mean() / 100.0 / tiles
    print(f"K={K}: span {end.max():.1f} us ({end.max() / K:.2f}/tick), {len(s)} workgroups x "
          f"{tiles:.2f} tiles; dur p10/p50/max {np.percentile(dur, 10):.1f}/{np.median(dur):.1f}/"
          f"{dur.max():.1f}; per interval (us): w0 produce {per[0]:.2f} wait {per[1]:.2f} | "
          f"w1 D {per[2]:.2f} wait {per[3]:.2f} | w2 E {per[4]:.2f}; tile switch {sw:.2f} us each "
          f"(prefetch wait {vm:.2f}, publish {pub:.2f}, load {ld:.2f}); prefetch issue {dma:.2f} per tile",
          flush=True)
sim.check()
