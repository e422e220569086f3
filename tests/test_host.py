"""CPU tests of the host side: the C ABI library loads and exports what
include/craft.h declares, the native scenario generator reproduces the
reference's random stream, and the host input layout is shard-invariant."""
import ctypes
import os
import re

import numpy as np
import pytest

from psketch_amd import _native as N
from psketch_amd.sim import sample_scenarios, synthetic_specs, hash_actions
from tests.helpers import make_tables

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "craft.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(craft_[a-z_]+)\s*\(", src)))


@pytest.mark.parametrize("cpu", [False, True])
def test_library_exports_every_header_symbol(cpu):
    """The HIP library and its CPU variant export every entry point
    include/craft.h declares, and the ctypes table binds exactly those."""
    lib = N.lib(cpu=cpu)
    names = header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    assert sorted(N.SIGNATURES) == names


def test_create_rejects_bad_config_on_both_libraries():
    for cpu in (False, True):
        _, _, _, cfg = make_tables()
        cfg.n_features += 1
        h = ctypes.c_void_p()
        assert N.lib(cpu=cpu).craft_sim_create(ctypes.byref(cfg), 0, 16, 0, 4, ctypes.byref(h)) == N.EINVAL
        assert not h.value


def test_config_layout_matches_c(oracle_mod):
    _, _, _, cfg = make_tables()
    assert oracle_mod.lib().oracle_sizeof_config() == ctypes.sizeof(cfg)


def test_strerror():
    assert N.strerror(N.EBADACTION) == "Unexpected action"
    assert N.strerror(N.OK) == "ok"


def test_create_rejects_bad_config_without_gpu():
    _, _, _, cfg = make_tables()
    cfg.n_features += 1           # craft.py:327 feature-length assertion
    h = ctypes.c_void_p()
    st = N.lib().craft_sim_create(ctypes.byref(cfg), 0, 16, 0, 4, ctypes.byref(h))
    assert st == N.EINVAL and not h.value


# ---- scenario generator -------------------------------------------------------------------
@pytest.mark.parametrize("name,world,count", [("w8", "craft_medium", 100),
                                              ("w12", "craft_medium_12x12", 64)])
def test_native_generator_matches_reference_stream(golden, name, world, count):
    """make_data.sample_scenario run by the reference on RandomState(123)."""
    g = golden("scenarios_seed123.npz")
    params, cb, _, _ = make_tables(world)
    grids, init, mt = sample_scenarios(params, cb, 123, count, dedup=True)
    np.testing.assert_array_equal(grids, g[f"{name}_grids"])
    np.testing.assert_array_equal(init, g[f"{name}_init"])
    np.testing.assert_array_equal(mt[:624], g[f"{name}_mt_key"])
    assert mt[624] == g[f"{name}_mt_pos"][0]


def test_native_mt19937_matches_numpy():
    params, cb, _, _ = make_tables("craft_medium_12x12")
    for seed in (0, 1, 2**32 - 1):
        _, _, mt = sample_scenarios(params, cb, seed, 3, dedup=False)
        rs = np.random.RandomState(seed)
        # replay: the native stream must equal numpy's after the same draws
        from oracle.make_data_oracle import sample_worlds
        from psketch_amd.cookbook import generator_primitives
        rs2 = np.random.RandomState(seed)
        for _ in range(3):
            from oracle.make_data_oracle import sample_scenario
            ws = [cb.index["workshop%d" % i] for i in range(3)]
            sample_scenario(12, 12, cb.index["boundary"], generator_primitives(cb), 2, ws, rs2)
        st = rs2.get_state()
        np.testing.assert_array_equal(mt[:624], st[1])
        assert mt[624] == st[2]
        del rs


def test_make_data_oracle_regenerates_reference_dataset(golden, oracle_mod):
    """make_data.py with seed 123 reproduces the reference's committed dev/test
    splits: worlds, task order, init positions, instance ids and teacher
    demonstrations.  Also the native generator equals the oracle's worlds."""
    from oracle.make_data_oracle import make_dataset, sample_worlds
    from psketch_amd.cookbook import generator_primitives
    params, cb, tm, cfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(cfg)
    data = make_dataset(params, cb, tm, o, generator_primitives(cb), seed=123)
    g = golden("devtest.npz")
    for split in ("dev", "test"):
        items = data[split]
        np.testing.assert_array_equal(np.stack([it["grid"].reshape(-1) for it in items]),
                                      g[f"{split}_grids"])
        rows = []
        for wi, it in enumerate(items):
            for ti in it["task_instances"]:
                for pos, iid, acts in zip(ti["init_pos"], ti["ids"], ti["ref_actions"]):
                    rows.append((wi, ti["task"], tuple(int(v) for v in pos), iid, tuple(acts)))
        assert [r[0] for r in rows] == g[f"{split}_world"].tolist()
        assert [r[1] for r in rows] == g[f"{split}_task"].tolist()
        assert [list(r[2]) for r in rows] == g[f"{split}_pos"].tolist()
        assert [r[3] for r in rows] == g[f"{split}_ids"].tolist()
        ref_acts = [tuple(int(a) for a in row if a >= 0) for row in g[f"{split}_actions"]]
        assert [r[4] for r in rows] == ref_acts
    assert sum(len(ti["init_pos"]) for it in data["train"] for ti in it["task_instances"]) == 17600
    worlds, _, _ = sample_worlds(params, cb, generator_primitives(cb), 123, 100)
    native, _, _ = sample_scenarios(params, cb, 123, 100, dedup=True)
    np.testing.assert_array_equal(native, np.stack([w.reshape(-1) for w in worlds]))


# ---- synthetic inputs --------------------------------------------------------------------
def test_synthetic_specs_properties_and_shard_invariance():
    params, cb, tm, _ = make_tables("craft_medium_12x12")
    grids, _, _ = sample_scenarios(params, cb, 123, 32)
    tasks = [t.id for t in tm.dataset_tasks()]
    full = synthetic_specs(grids, 12, 12, 1000, 0, seed=3, task_ids=tasks)
    scen, x, y, d, task = full
    assert (grids[scen, x * 12 + y] == 0).all()
    assert ((x > 0) & (x < 11) & (y > 0) & (y < 11)).all()
    assert (d == 0).all() and set(task.tolist()) == set(tasks)
    a = synthetic_specs(grids, 12, 12, 400, 0, seed=3, task_ids=tasks)
    b = synthetic_specs(grids, 12, 12, 600, 400, seed=3, task_ids=tasks)
    for fa, fb, ff in zip(a, b, full):
        np.testing.assert_array_equal(np.concatenate([fa, fb]), ff)
    again = synthetic_specs(grids, 12, 12, 1000, 0, seed=3, task_ids=tasks)
    for u, v in zip(full, again):
        np.testing.assert_array_equal(u, v)


def test_hash_actions_uniform():
    a = hash_actions(0, np.arange(60000), 5)
    counts = np.bincount(a, minlength=6)
    assert counts.min() > 9500 and counts.max() < 10500


def devtest_as_json(fx, split, tm, K):
    """Rebuilds the reference's split-file structure (data/craft_medium_{split}.json)
    from the compact devtest.npz fixture: same worlds, tasks, positions, ids."""
    names = [f"{t.goal_name}[{t.goal_arg}]" for t in tm.tasks]
    grids = fx[f"{split}_grids"]
    world, task, pos = fx[f"{split}_world"], fx[f"{split}_task"], fx[f"{split}_pos"]
    acts, ids = fx[f"{split}_actions"], fx[f"{split}_ids"]
    out = []
    W = int(round(np.sqrt(grids.shape[1])))
    for wi in range(len(grids)):
        g = grids[wi].reshape(W, W)
        onehot = (g[..., None] == np.arange(K)[None, None, :]) & (g[..., None] > 0)
        item = {"grid": onehot.astype(float).tolist(), "task_instances": []}
        sel = np.nonzero(world == wi)[0]
        for tk in dict.fromkeys(task[sel].tolist()):
            rows = sel[task[sel] == tk]
            item["task_instances"].append({
                "task": names[tk], "init_pos": pos[rows].tolist(),
                "ids": [f"{split}_{i}" for i in ids[rows]],
                "ref_actions": [[int(a) for a in acts[r] if a >= 0] for r in rows]})
        out.append(item)
    return out


def test_dataset_flatten_and_batches(golden):
    """psketch_amd.dataset.Dataset == data/dataset.py:47-86: flattening order,
    one-hot grid -> scenario pool, next_batch's shuffling through config.random."""
    from psketch_amd.dataset import Dataset
    fx = golden("devtest.npz")
    _, cb, tm, _ = make_tables("craft_medium")
    data = devtest_as_json(fx, "dev", tm, cb.n_kinds)
    ds = Dataset(data, "dev", tm, random=np.random.RandomState(3), batch_size=32)
    n = len(fx["dev_task"])
    assert len(ds) == n
    spec = np.stack(Dataset.specs(list(ds)), axis=1)
    # the fixture's own order is the flattening order of the reference
    first_seen = {w: i for i, w in enumerate(dict.fromkeys(fx["dev_world"].tolist()))}
    assert np.array_equal(spec[:, 0], [first_seen[w] for w in fx["dev_world"]])
    assert np.array_equal(spec[:, 1:3], fx["dev_pos"])
    assert np.array_equal(spec[:, 4], fx["dev_task"])
    assert [it["id"] for it in ds] == [f"dev_{i}" for i in fx["dev_ids"]]
    assert np.array_equal(ds.pool_array()[spec[:, 0]], fx["dev_grids"][fx["dev_world"]])
    # next_batch: the reference shuffles list(range(n)) with config.random on every pass
    rs = np.random.RandomState(3)
    for _ in range(2):
        order = list(range(n))
        rs.shuffle(order)
        got = [it["id"] for b in ds.iterate_batches() for it in b]
        assert got == [ds[i]["id"] for i in order]
    with pytest.raises(AssertionError):
        bad = devtest_as_json(fx, "dev", tm, cb.n_kinds)[:1]
        bad[0]["grid"][1][1][3] = 1.0
        bad[0]["grid"][1][1][4] = 1.0
        Dataset(bad, "dev", tm)


@pytest.mark.skipif(not os.path.isdir("/root/reference/data"), reason="reference split files absent")
def test_dataset_reads_reference_split_files(golden):
    """The committed split JSON files themselves (build container only)."""
    from psketch_amd.dataset import Dataset
    fx = golden("devtest.npz")
    _, _, tm, _ = make_tables("craft_medium")
    for split in ["dev", "test"]:
        ds = Dataset(f"/root/reference/data/craft_medium_{split}.json", split, tm)
        spec = np.stack(Dataset.specs(list(ds)), axis=1)
        assert np.array_equal(spec[:, 1:3], fx[f"{split}_pos"])
        assert np.array_equal(spec[:, 4], fx[f"{split}_task"])
        assert np.array_equal(ds.pool_array()[spec[:, 0]], fx[f"{split}_grids"][fx[f"{split}_world"]])
        L = fx[f"{split}_actions"]
        assert all(tuple(int(a) for a in L[i] if a >= 0) == it["ref_actions"] for i, it in enumerate(ds))


def test_step_args_layout_matches_c(tmp_path):
    """ctypes craft_step_args_t == the C struct of include/craft.h (offsets, size)."""
    import subprocess
    fields = [f for f, _ in N.craft_step_args_t._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "craft.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(craft_step_args_t, {f}));\n' for f in fields)
                   + 'printf("%zu\\n", sizeof(craft_step_args_t));\nreturn 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(N._HERE, "..", "include"),
                           "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [getattr(N.craft_step_args_t, f).offset for f in fields] + [ctypes.sizeof(N.craft_step_args_t)]
    assert got == want


def test_config1_train_instance_regenerated(golden, oracle_mod):
    """BASELINE configs[0]: the oracle's make_data restatement regenerates the
    reference's craft_medium_train.json worlds and the first world's instance
    positions and ids (tests/golden/config1_train0.npz, produced by the
    reference's make_data.py functions, make_data.py:154-238)."""
    from oracle.make_data_oracle import make_dataset
    from psketch_amd.cookbook import generator_primitives
    g = golden("config1_train0.npz")
    params, cb, tm, cfg = make_tables("craft_medium")
    data = make_dataset(params, cb, tm, oracle_mod.Oracle(cfg), generator_primitives(cb), seed=123)
    train = data["train"]
    np.testing.assert_array_equal(np.stack([it["grid"].reshape(-1) for it in train]), g["train_grids"])
    tis = train[0]["task_instances"]
    np.testing.assert_array_equal(np.asarray([ti["init_pos"] for ti in tis]), g["train0_pos"])
    np.testing.assert_array_equal(np.asarray([[int(str(i).split("_")[-1]) for i in ti["ids"]] for ti in tis]),
                                  g["train0_ids"])
    assert tis[0]["task"] == int(g["task"][0])
    assert list(tis[0]["ref_actions"][0]) == g["demo"].tolist()
