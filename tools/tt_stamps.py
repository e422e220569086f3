"""Diagnostic: where the one-tile teacher tick (craft_step_teach, tile_kernel<WIN, MODE_TICK, TILE,
TL, NW>) spends its time, per workgroup, from CRAFT_STAMPS_TT stamps (never the product library):
0 start, 1 the first teacher wave's walks done, 2 the last teacher wave's dense pass done, 3 wave
0's A + C done, 4 the last streaming wave done, 5 D done, 6 the end, 7 the XCC.

    python tools/diag_build.py craft_sim craft_tick_teach -DCRAFT_STAMPS_TT --out libpsketch_craft_diag_tt.so
    python tools/tt_stamps.py [world]            (on the GPU box)"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from psketch_amd import _native  # noqa: E402
_native.LIB_PATH = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag_tt.so")
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402

lib = _native.lib()
lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def run(world, n=65536, ticks=24):
    sim = CraftSim(world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    tasks = [t.id for t in sim.task_manager.dataset_tasks()]
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, seed=0, task_ids=tasks))
    rows = (n + 15) // 16
    st = torch.zeros((rows, 8), dtype=torch.int64, device="cuda")
    lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
    R = 16
    ring = torch.empty((R, n, sim.n_features), dtype=sim.obs_dtype, device="cuda")
    labels = torch.empty((R, n), dtype=torch.int32, device="cuda")
    res = []
    for t in range(ticks):
        st.zero_()
        sim.step(seed=0, tick=t, obs=ring[t % R], labels=labels[t % R])
        torch.cuda.synchronize()
        s = st.cpu().numpy()
        used = s[:, 0] > 0
        s = s[used]
        v = s[:, :7].astype(np.float64)
        t0 = v[:, 0].min()
        v = (v - t0) / 100.0                     # 100 MHz -> us
        res.append((v, s[:, 7]))
    vs = [r[0] for r in res[4:]]
    wg = vs[0].shape[0]
    out = {"world": world, "workgroups": wg}
    names = {"start": 0, "teach_walk": 1, "teach_dense": 2, "C": 3, "E": 4, "D": 5, "end": 6}
    for nm, k in names.items():
        out[nm] = [round(float(np.median([np.median(v[:, k]) for v in vs])), 2),
                   round(float(np.median([np.percentile(v[:, k], 90) for v in vs])), 2),
                   round(float(np.median([v[:, k].max() for v in vs])), 2)]
    out["fields"] = "p50 / p90 / max over workgroups, us from the first start (median over ticks)"
    conc = []
    for v in vs:                                   # workgroups alive at once (start .. end)
        ev = np.concatenate([np.stack([v[:, 0], np.ones(len(v))], 1), np.stack([v[:, 6], -np.ones(len(v))], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        conc.append(np.cumsum(ev[:, 1]).max())
    out["max_alive"] = float(np.median(conc))
    out["life_p50"] = round(float(np.median([np.median(v[:, 6] - v[:, 0]) for v in vs])), 2)
    out["teacher_after_E"] = round(float(np.median([np.mean(v[:, 2] > v[:, 4]) for v in vs])), 3)
    out["xcc_hist"] = np.bincount(res[-1][1].astype(np.int64), minlength=8).tolist()
    sim.check()
    return out


for w in sys.argv[1:] or ["craft_medium_12x12_w5"]:
    print(json.dumps(run(w)), flush=True)
