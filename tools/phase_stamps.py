"""Diagnostic: per-phase timing of the tick kernel from s_memrealtime stamps.

Builds psketch_amd/lib/libpsketch_craft_diag.so with -DCRAFT_STAMPS (never the
product library), runs N ticks, and reports per-workgroup phase durations and
the spread of phase start times across the grid (all in microseconds)."""
import ctypes, json, os, subprocess, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge
DIAG = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag.so")
if "--build" in sys.argv:          # the tile kernel and craft_sim stamped, every other object the product's
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import diag_build
    diag_build.build(stamped=("craft_sim", "craft_tile"))
    sys.exit(0)
import torch
from psketch_amd import _native
_native.LIB_PATH = DIAG
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
lib = _native.lib()
lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

def run(world, n=65536, ticks=20, obs=True, tile=0):
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=1024)
    sim.tune(tile, 0, 2)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, 0, [t.id for t in sim.task_manager.dataset_tasks()]))
    tiles = (n + 15) // 16
    st = torch.zeros((tiles, 8), dtype=torch.int64, device="cuda")
    lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
    ring = [sim.empty_obs() for _ in range(16)] if obs else None     # bench.py's 16-slot ring
    rows = (n + sim.tile_shape()[0] - 1) // sim.tile_shape()[0]
    res = []
    for t in range(ticks):
        sim.step(seed=0, tick=t, obs=ring[t % 16] if obs else None)
        torch.cuda.synchronize()
        s = st[:rows].cpu().numpy().astype(np.float64) / 100.0   # 100 MHz -> us
        t0 = s[:, 0].min()
        res.append(s[:, :7] - t0)
    r = np.stack(res[5:])                       # [ticks, tiles, 7]
    out = {"world": world, "obs": obs, "tile": sim.tile_shape()[0]}
    names = ["A", "C", "D_wait", "D", "E"]
    idx = [(0, 1), (1, 3), (3, 4), (4, 5), (5, 6)] if obs else [(0, 1), (1, 3)]
    for nm, (i, j) in zip(names, idx):
        d = r[:, :, j] - r[:, :, i]
        out[nm + "_med"] = round(float(np.median(d)), 2)
        out[nm + "_p90"] = round(float(np.percentile(d, 90)), 2)
    out["start_spread_p50_p100"] = [float(np.median(r[:, :, 0])), float(r[:, :, 0].max())]
    last = 6
    out["end_p50"] = float(np.median(r[:, :, last]))
    out["end_max"] = float(np.median(r[:, :, last].max(axis=1)))
    out["xcc_hist"] = np.bincount(st[:rows, 7].cpu().numpy().astype(np.int64), minlength=8).tolist()
    sim.check()
    return out

for w in sys.argv[1:] or ["craft_medium_12x12"]:
    if w.startswith("--"):
        continue
    w, _, tile = w.partition(":")               # world[:tile envs]
    print(json.dumps(run(w, obs=True, tile=int(tile or 0))))
