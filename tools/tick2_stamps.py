"""Diagnostic: where the fused tick + teacher's time goes (craft_step_teach's two-tile kernel,
csrc/craft_tick2.h), from its CRAFT_STAMPS stamps (never the product library): per workgroup,
in µs from the launch's first stamp, its start, wave 0's loads landed and C done, the barrier,
wave 0's first store issued, the last tick wave done issuing stores, and the last teacher wave
done; whether the BFS or the stores end each workgroup; and the XCC histogram.

    python tools/diag_build.py craft_sim craft_tick_teach      # here (CPU)
    python tools/diag_build.py craft_sim craft_tick_teach -DCRAFT_STAMPS_T --out libpsketch_craft_diag_t.so
    python tools/tick2_stamps.py [--ring 16|1] [--ticks 30]    # on the GPU box"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--world", default="craft_medium_12x12")
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--ring", type=int, nargs="+", default=[16, 1])
    p.add_argument("--ticks", type=int, default=30)
    p.add_argument("--lib", default="libpsketch_craft_diag.so",
                   help="diagnostic library; libpsketch_craft_diag_c.so (-DCRAFT_STAMPS_C): wave 0's A + C; "
                        "libpsketch_craft_diag_t.so (-DCRAFT_STAMPS_T): the teacher's walk and dense pass")
    args = p.parse_args()
    import torch
    from psketch_amd import _native
    _native.LIB_PATH = os.path.join(REPO, "psketch_amd", "lib", args.lib)
    from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
    lib = _native.lib()
    lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    n = args.envs
    sim = CraftSim(args.world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, 0,
                               [t.id for t in sim.task_manager.dataset_tasks()]))
    kname, per_wg, lanes = sim.step_shape(teach=True)
    wgs = (n + per_wg - 1) // per_wg
    st = torch.zeros((wgs, 8), dtype=torch.int64, device="cuda")
    lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
    names = ["start", "loads", "C", "barrier", "first_store", "stores_issued", "teacher_done"]
    if "diag_c" in args.lib:             # CRAFT_STAMPS_C: wave 0's A + C in detail
        names = ["start", "state_landed", "row_in_lds", "pre_step_done", "transition_done", "stores_issued",
                 "C_done"]
    tmode = "diag_t" in args.lib        # CRAFT_STAMPS_T: the teacher's walk, the dense pass, the count
    if tmode:
        names = ["start", "walk_done", "dense_start", "barrier", "deferred", "stores_issued", "teacher_done"]
    for R in args.ring:
        ring = [sim.empty_obs() for _ in range(R)]
        lab = torch.empty(n, dtype=torch.int32, device="cuda")
        rows = []
        for t in range(args.ticks):
            st.zero_()
            sim.step(seed=0, tick=t, obs=ring[t % R], labels=lab)
            torch.cuda.synchronize()
            s = st.cpu().numpy().astype(np.float64)
            tcols = [0, 1, 2, 3, 5, 6] if tmode else list(range(7))
            s[:, tcols] = (s[:, tcols] - s[:, 0].min()) / 100.0     # 100 MHz -> µs
            rows.append(s)
        r = np.stack(rows[5:])                                     # [ticks, wgs, 8]
        out = {"world": args.world, "envs": n, "ring": R, "kernel": kname, "envs_per_wg": per_wg,
               "teacher_lanes": lanes}
        for i, nm in enumerate(names):
            v = r[:, :, i]
            out[nm] = {"p10": round(float(np.percentile(v, 10)), 2), "p50": round(float(np.median(v)), 2),
                       "p90": round(float(np.percentile(v, 90)), 2), "max": round(float(v.max(axis=1).mean()), 2)}
        print(json.dumps(out) if "diag_c" in args.lib else "", end="\n" if "diag_c" in args.lib else "")
        if "diag_c" in args.lib:
            continue
        end = np.maximum(r[:, :, 5], r[:, :, 6])
        out["wg_end_max_mean"] = round(float(end.max(axis=1).mean()), 2)
        out["teacher_ends_wg_frac"] = round(float((r[:, :, 6] > r[:, :, 5]).mean()), 3)
        out["teacher_after_stores_us_p50"] = round(float(np.median(r[:, :, 6] - r[:, :, 5])), 2)
        out["last_store_wave_us_mean"] = round(float(r[:, :, 5].max(axis=1).mean()), 2)
        out["last_teacher_wave_us_mean"] = round(float(r[:, :, 6].max(axis=1).mean()), 2)
        out["xcc_hist"] = np.bincount(r[-1, :, 7].astype(np.int64), minlength=8).tolist()
        print(json.dumps(out), flush=True)
        del ring
    sim.check()


if __name__ == "__main__":
    main()
