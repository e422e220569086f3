"""Diagnostic: phase timing of the step kernel (csrc/craft_step.h) from s_memrealtime stamps,
and where its workgroups land (HW_ID / XCC_ID).

Links psketch_amd/lib/libpsketch_craft_diag.so from the product objects except craft_sim and
craft_step, which are compiled again with -DCRAFT_STAMPS (never the product library), then
runs 20 craft_step ticks at 65,536 envs (ring of 16 observation slots) per knob setting and
reports, in µs from the launch's first stamp (percentiles over tick waves): tick wave start,
A (loads landed), C, the first and last scatter published, the stream wave's first sub-chunk
issued and its stores drained, and the number of tick waves per CU.

    python tools/step_stamps.py [--build] [--cfg EPW:PER_CU ...]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
from collections import Counter

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402

DIAG = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_diag.so")


def build(stamped=("craft_sim", "craft_step")):
    ge.build()
    obj = os.path.join(REPO, "psketch_amd", "lib", "obj")
    dobj = os.path.join(REPO, "psketch_amd", "lib", "obj_diag")
    os.makedirs(dobj, exist_ok=True)
    objs = []
    for src in ge.SOURCES:
        base = os.path.splitext(src)[0]
        if base in stamped:
            o = os.path.join(dobj, base + ".o")
            subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                                   "-DCRAFT_STAMPS", "-c", os.path.join(ge.CSRC, src), "-o", o])
        else:
            o = os.path.join(obj, base + ".o")
        objs.append(o)
    subprocess.check_call([ge.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", DIAG] + objs)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true", help="(re)build the diagnostic library and exit")
    p.add_argument("--cfg", nargs="+", default=["64:0", "64:1", "32:0", "16:0"])
    p.add_argument("--world", default="craft_medium_12x12")
    p.add_argument("--envs", type=int, default=65536)
    args = p.parse_args()
    if args.build:
        build()
        return
    os.environ["PSKETCH_CRAFT_LIB"] = DIAG
    import torch
    from psketch_amd import _native
    from psketch_amd import CraftSim, sample_scenarios, synthetic_specs
    lib = _native.lib()
    lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.craft_debug_set_stamps.restype = ctypes.c_int
    n = args.envs
    sim = CraftSim(args.world, n_envs=n, device=0, pool_capacity=1024)
    g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
    sim.load_pool(g)
    sim.reset(*synthetic_specs(g, sim.width, sim.height, n, 0, 0,
                               [t.id for t in sim.task_manager.dataset_tasks()]))
    R = 16
    ring = torch.empty((R, n, sim.n_features), dtype=torch.float32, device="cuda")
    rows = 2 * ((n + 15) // 16)                            # + the extra stamps (STEP_STAMP2)
    st = torch.zeros((rows, 8), dtype=torch.int64, device="cuda")
    tick = 0
    for cfg in args.cfg:
        epw, per_cu = (int(x) for x in cfg.split(":"))
        sim.tune_step(2, epw, per_cu)
        res = []
        for t in range(20):
            lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr() if t >= 5 else 0))
            st.zero_()
            sim.step(seed=0, tick=tick, obs=ring[tick % R])
            tick += 1
            torch.cuda.synchronize()
            if t < 5:
                continue
            w = (n + epw - 1) // epw
            nw = ((n + 4 * epw - 1) // (4 * epw)) * 4           # tick waves of the launch
            s = st[:w].cpu().numpy()
            s2 = st[nw:nw + w].cpu().numpy()
            res.append(np.concatenate([s, s2[:, :5]], axis=1))
        lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(0))
        r = np.stack(res)                                   # [ticks, waves, 8]
        tm = np.concatenate([r[:, :, :7], r[:, :, 8:13]], axis=2).astype(np.float64) / 100.0   # µs
        t0 = tm[:, :, 0].min(axis=1, keepdims=True)
        rel = tm - t0[:, :, None]
        out = {"epw": epw, "per_cu": per_cu, "kernel_span_med": round(float(np.median(rel[:, :, 6].max(1))), 2)}
        names = [("start", 0), ("A1_landed", 7), ("pool_issued", 11), ("pool_landed", 8), ("A_done", 1),
                 ("C_done", 2), ("D0_first", 9),
                 ("D0_repeat", 10), ("D0_published", 3), ("D_all_published", 4), ("E0_issued", 5),
                 ("stream_drained", 6)]
        for nm, k in names:
            out[nm] = [round(float(np.percentile(rel[:, :, k], q)), 2) for q in (10, 50, 90, 100)]
        hw = r[0, :, 7]
        xcc = (hw >> 32) & 0xF
        h = hw & 0xFFFFFFFF
        key = (xcc << 16) | (((h >> 13) & 7) << 8) | (((h >> 12) & 1) << 4) | ((h >> 8) & 0xF)
        per = Counter(Counter(key.tolist()).values())
        out["tick_waves_per_cu_hist"] = {str(k): v for k, v in sorted(per.items())}
        out["cus_used"] = int(len(set(key.tolist())))
        print(json.dumps(out), flush=True)
    sim.check()


if __name__ == "__main__":
    main()
