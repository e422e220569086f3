"""Diagnostic: per-workgroup timing of the multi-tick rollout kernel on several
allocations of the observation ring (CRAFT_STAMPS build, never the product).

For each ring: the launch span, the distribution of workgroup durations, the
mean duration per XCD, and the per-tick phase split of the two roles: producer
(C transition, D scatter, barrier wait) and consumer wave 1 (E stream, barrier
wait); shows whether a slow launch is uniformly slow or held up by a subset of
workgroups, and which role sets the tick.

  python tools/rollout_stamps.py --build          # here (CPU): the diagnostic library
  python tools/rollout_stamps.py [tile] [store] [chunk] [rings] [K] [threads]   # on the GPU box"""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402

DIAG = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag.so")
if "--build" in sys.argv:
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(REPO, "psketch_amd", "lib", "obj_diag")
    os.makedirs(objdir, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DCRAFT_STAMPS"]
    if "--c-split" in sys.argv:    # slots 4 / 5 time C's parts instead of the consumer
        flags.append("-DCRAFT_STAMPS_C")
    objs = [os.path.join(objdir, os.path.splitext(x)[0] + ".o") for x in ge.SOURCES]

    def cc(pair):
        subprocess.check_call([ge.HIPCC] + flags + ["-c", os.path.join(ge.CSRC, pair[0]), "-o", pair[1]])
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(cc, zip(ge.SOURCES, objs)))
    subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", DIAG] + objs)
    sys.exit(0)
import torch  # noqa: E402
from psketch_amd import _native  # noqa: E402
_native.LIB_PATH = DIAG
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402

lib = _native.lib()
lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
n, R = 65536, 16
K = int(sys.argv[5]) if len(sys.argv) > 5 else 32
tile = int(sys.argv[1]) if len(sys.argv) > 1 else 64
store = int(sys.argv[2]) if len(sys.argv) > 2 else 0
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 0
sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
sim.load_pool(g)
sim.tune(tile, 0, store)
threads = int(sys.argv[6]) if len(sys.argv) > 6 else 0
sim.tune_rollout(chunk, threads)
sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
tiles = n // 16                     # one row per workgroup; grids never exceed n / 16
st = torch.zeros((tiles, 8), dtype=torch.int64, device="cuda")
lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
keep, tick = [], 0
for i in range(int(sys.argv[4]) if len(sys.argv) > 4 else 6):
    ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
    keep.append(ring)
    res = []
    for rep in range(4):
        st.zero_()
        sim.rollout(K, tick0=tick, obs=None if os.environ.get("NO_OBS") else ring)
        tick += K
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.float64)
        res.append(s)
    s = res[-1]
    s = s[s[:, 6] > 0]                  # the launch's workgroups
    t0 = s[:, 0].min()
    start, end = (s[:, 0] - t0) / 100.0, (s[:, 6] - t0) / 100.0     # 100 MHz -> us
    dur = end - start
    xcc = s[:, 7].astype(int)
    per_xcc = [round(float(dur[xcc == x].mean()), 1) for x in range(8)]
    print(f"ring {i}: span {end.max():.1f} us ({end.max() / K:.2f}/tick)  start p50/max "
          f"{np.median(start):.1f}/{start.max():.1f}  dur p10/p50/p90/max {np.percentile(dur, 10):.1f}/"
          f"{np.median(dur):.1f}/{np.percentile(dur, 90):.1f}/{dur.max():.1f}  per-XCD {per_xcc}",
          flush=True)
    units = tiles * 16 // tile / len(s)                  # tiles per workgroup
    ph = s[:, 1:6].mean(0) / 100.0 / (K * units)        # us per tick per workgroup
    print(f"   per tick (us): producer C {ph[0]:.2f} D {ph[1]:.2f} wait {ph[2]:.2f} | "
          f"slot4 {ph[3]:.2f} slot5 {ph[4]:.2f} (consumer E / wait; C-split builds: C before / in "
          f"the transition)  ({len(s)} workgroups, {units:.2f} tiles each)", flush=True)
sim.check()
