"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (race
detection / sanitizers: "ASan/UBSan on the C++ CPU restatement").

The C oracle (oracle/craft_oracle.c: step, features, satisfies, the BFS teacher, both
scenario generators, the multi-threadless bench loop) and the product's host-side scenario
generator (psketch_amd/csrc/scenario_gen.cpp) are compiled here with
-fsanitize=address,undefined and no recovery, loaded into a child Python with the ASan
runtime preloaded, and driven through tests/sanitize_workload.py on 8x8, 12x12 (w = 3 and 5)
and 16x16 w = 7 worlds.  The child must exit cleanly (any report aborts it) and its results
must equal the regular -O3 builds' in this process.  GPU code is not sanitized (not
available on the pool); the HIP kernels' own parity tests cover them."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from psketch_amd.cookbook import generator_primitives
from psketch_amd.sim import sample_scenarios, synthetic_specs
from tests.conftest import REPO
from tests.helpers import make_tables
from tests import sanitize_workload as WL

WORLDS = ["craft_medium", "craft_medium_12x12", "craft_medium_12x12_w5", "craft_16x16_w7"]
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=all", "-fPIC", "-shared"]

_CHILD = r"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import oracle as O
from tests import sanitize_workload as WL
d = os.environ["SAN_DIR"]
scen = ctypes.CDLL(os.path.join(d, "libscen_san.so"))
for w in os.environ["WORLDS"].split(","):
    z = np.load(os.path.join(d, w + ".in.npz"))
    raw = bytes(z["cfg"])
    class Cfg(ctypes.c_ubyte * len(raw)):
        pass
    cfg = Cfg.from_buffer_copy(raw)
    cfg.width, cfg.height, cfg.n_kinds, cfg.n_features = (int(x) for x in z["meta"])
    g = z["gen"]
    gen_args = (int(g[0]), int(g[1]), int(g[2]), z["prims"], int(g[3]), z["ws"], int(g[4]), int(g[5]))
    out = WL.run_oracle(O, cfg, z["pool"], [z["spec%d" % i] for i in range(5)], gen_args)
    sc = WL.run_scenarios(scen, int(g[0]), int(g[1]), int(g[2]), z["prims"], int(g[3]), z["ws"],
                          123, 24, True)
    out.update({"scen_" + k: v for k, v in sc.items()})
    np.savez(os.path.join(d, w + ".out.npz"), **out)
maps = open("/proc/self/maps").read()
assert "liboracle_san.so" in maps and "libasan" in maps and "libubsan" in maps
print("sanitized-ok")
"""


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def san_dir(tmp_path_factory):
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("gcc's AddressSanitizer runtime is not installed")
    d = str(tmp_path_factory.mktemp("san"))
    subprocess.check_call(["gcc", "-std=c11", *SAN, "-o", os.path.join(d, "liboracle_san.so"),
                           os.path.join(REPO, "oracle", "craft_oracle.c")])
    subprocess.check_call(["g++", "-std=c++17", *SAN, "-o", os.path.join(d, "libscen_san.so"),
                           os.path.join(REPO, "psketch_amd", "csrc", "scenario_gen.cpp")])
    return d, asan


def _inputs(world):
    params, cb, tm, cfg = make_tables(world)
    W, H = params["WIDTH"], params["HEIGHT"]
    pool, _, _ = sample_scenarios(params, cb, 123, 32)
    specs = synthetic_specs(pool, W, H, 96, 0, seed=1, task_ids=[t.id for t in tm.dataset_tasks()])
    prims = np.asarray(generator_primitives(cb), dtype=np.int32)
    ws = np.asarray([cb.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])], dtype=np.int32)
    gen = np.array([W, H, cb.index["boundary"], params["N_PRIMITIVES"], 16, 77], dtype=np.int64)
    return params, cb, cfg, pool, specs, prims, ws, gen


def test_host_code_clean_under_asan_ubsan(san_dir, oracle_mod):
    d, asan = san_dir
    expect = {}
    for w in WORLDS:
        params, cb, cfg, pool, specs, prims, ws, gen = _inputs(w)
        raw = np.frombuffer(ctypes.string_at(ctypes.addressof(cfg), ctypes.sizeof(cfg)), dtype=np.uint8)
        np.savez(os.path.join(d, w + ".in.npz"), cfg=raw, pool=pool, prims=prims, ws=ws, gen=gen,
                 meta=np.array([cfg.width, cfg.height, cfg.n_kinds, cfg.n_features]),
                 **{"spec%d" % i: np.asarray(s) for i, s in enumerate(specs)})
        gen_args = (int(gen[0]), int(gen[1]), int(gen[2]), prims, int(gen[3]), ws, int(gen[4]), int(gen[5]))
        e = WL.run_oracle(oracle_mod, cfg, pool, list(specs), gen_args)
        grids, init, mt = sample_scenarios(params, cb, 123, 24, dedup=True)
        e.update({"scen_grids": grids, "scen_init": init, "scen_mt": mt})
        expect[w] = e
    pre = os.environ.get("LD_PRELOAD", "")                 # the ASan runtime first, the rest kept
    env = dict(os.environ, REPO=REPO, SAN_DIR=d, WORLDS=",".join(WORLDS),
               LD_PRELOAD=asan + (":" + pre if pre else ""),
               PSKETCH_ORACLE_LIB=os.path.join(d, "liboracle_san.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:detect_odr_violation=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "sanitized-ok" in r.stdout, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    for w in WORLDS:
        got = dict(np.load(os.path.join(d, w + ".out.npz")))
        assert set(got) == set(expect[w]), w
        for k, v in expect[w].items():
            np.testing.assert_array_equal(got[k], v, err_msg=f"{w}: {k}")
        assert (expect[w]["teacher"] >= -1).mean() > 0.9, w      # the teacher ran, mostly labelled
