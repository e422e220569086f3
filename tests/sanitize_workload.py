"""The host-code workload tests/test_sanitizers.py runs twice: in this process against the
regular -O3 builds, and in a child process against AddressSanitizer + UBSan builds of the
same sources ("ASan/UBSan on the C++ CPU restatement").  Kept free of torch
and psketch_amd imports so the sanitized child loads nothing but numpy, ctypes and the
libraries under test.

    run_oracle(oracle_mod, cfg, pool, specs)  oracle/craft_oracle.c: init, 60 hashed-action
        ticks with auto-reset (step, satisfies, features), the DemonstrationTeacher and
        find_closest_resources on every env every 6th tick, 4 ticks of oracle_bench with
        labels, and both scenario generators;
    run_scenarios(lib, args)  psketch_amd/csrc/scenario_gen.cpp's craft_sample_scenarios
        (the product's host-side make_data.sample_scenario).
"""
import ctypes

import numpy as np


def run_oracle(O, cfg, pool, specs, gen_args):
    o = O.Oracle(cfg, pool)
    envs = o.init_envs(*specs)
    n = len(envs)
    out = {"obs": [], "reward": [], "done": [], "success": [], "teacher": [], "closest": []}
    for t in range(60):
        rc, obs, rew, done, succ = o.batch_tick(envs, 0, None, 5, t, True)
        assert rc == 0, rc
        out["obs"].append(obs.sum(axis=1))
        out["reward"].append(rew)
        out["done"].append(done)
        out["success"].append(succ)
        if t % 6 == 0:
            lab, clo = np.zeros(n, np.int32), np.zeros((n, 3), np.int32)
            for i in range(n):
                e = envs[i:i + 1]
                rc, a = o.teacher(e, int(e["task"][0]))
                lab[i] = a if rc == 0 else -100 - rc
                clo[i] = o.closest_resource(e, 1 + (i % (o.K - 1)))
            out["teacher"].append(lab)
            out["closest"].append(clo)
    out = {k: np.stack(v) for k, v in out.items()}
    bufs = o.bench_buffers(n, ring=2, teach=True)
    o.bench(envs, 0, 60, 4, 5, bufs)
    out["bench_obs"] = bufs[0].sum(axis=2)
    out["bench_labels"] = bufs[4].copy()
    out["bench_stats"] = bufs[5].copy()
    for rng in ("splitmix", "mt19937"):
        g, init, _ = O.generate_scenarios(*gen_args, rng=rng, dedup=rng == "mt19937")
        out["gen_" + rng] = g
        out["gen_init_" + rng] = init
    return out


def run_scenarios(lib, W, H, boundary, prims, n_per, ws, seed, count, dedup):
    prims = np.ascontiguousarray(prims, dtype=np.int32)
    ws = np.ascontiguousarray(ws, dtype=np.int32)
    grids = np.zeros((count, W * H), dtype=np.uint8)
    init = np.zeros((count, 2), dtype=np.int32)
    mt = np.zeros(625, dtype=np.uint32)
    vp = ctypes.c_void_p
    st = lib.craft_sample_scenarios(W, H, boundary, prims.ctypes.data_as(vp), len(prims), n_per,
                                    ws.ctypes.data_as(vp), len(ws), ctypes.c_uint32(seed), count,
                                    int(dedup), grids.ctypes.data_as(vp), init.ctypes.data_as(vp),
                                    mt.ctypes.data_as(vp))
    assert st == 0, st
    return {"grids": grids, "init": init, "mt": mt}
