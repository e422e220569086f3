"""Pins the CPU oracle (and the host-side table compiler) against the
reference: its own committed demonstrations and the fixtures that
tests/golden/make_golden.py produced by running the reference's code."""
import numpy as np
import pytest

from psketch_amd import _native as N
from tests.helpers import make_tables, world_for


# ---- static tables ----------------------------------------------------------------------
def test_cookbook_matches_reference(golden):
    ref = golden("cookbook.json")
    params, cb, tm, cfg = make_tables()
    assert list(cb.index) == ref["index"]
    assert cb.n_kinds == ref["n_kinds"] == cfg.n_kinds
    assert list(cb.primitives) == ref["primitives_iter"]
    assert [[k, {str(a): b for a, b in d.items()}] for k, d in cb.recipes.items()] == ref["recipes"]
    for k in range(cb.n_kinds):
        cls = cfg.kind_class[k]
        if k == 0:
            continue
        if k in ref["grabbable_indices"]:
            assert cls == N.KIND_GRABBABLE
        elif k in ref["workshop_indices"]:
            assert cls == N.KIND_WORKSHOP
        elif k == ref["water_index"]:
            assert cls == N.KIND_WATER
        elif k == ref["stone_index"]:
            assert cls == N.KIND_STONE
        else:
            assert cls == N.KIND_INERT
    for name, F in ref["n_features"].items():
        assert make_tables(name)[3].n_features == F
    assert [[t.goal_name, t.goal_arg, [f"{s.goal_name}[{s.goal_arg}]" for s in (t.subtasks or [])]]
            for t in tm.tasks] == ref["tasks"]
    goals = {"get": N.GOAL_GET, "make": N.GOAL_MAKE, "go": N.GOAL_GO, "use": N.GOAL_USE}
    for i, t in enumerate(tm.tasks):
        assert cfg.task[i].goal == goals.get(t.goal_name, N.GOAL_OTHER)
        assert cfg.task[i].arg_kind == (cb.index[t.goal_arg] or 0)
        assert [cfg.task[i].subtask[j] for j in range(cfg.task[i].n_subtasks)] == \
            [s.id for s in (t.subtasks or [])]
    for name, (idx, (dx, dy)) in ref["actions"].items():
        assert idx == getattr(N, name)


def test_cookbook_from_reference_yaml_matches_builtin():
    import os
    path = "/root/reference/resources/craft/recipes.yaml"
    hints = "/root/reference/resources/craft/hints.hierarchy.yaml"
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    from psketch_amd.cookbook import Cookbook, TaskManager
    a, b = Cookbook(path), Cookbook()
    assert a.index.contents == b.index.contents and a.recipes == b.recipes
    assert [repr(t) for t in TaskManager(hints).tasks] == [repr(t) for t in TaskManager().tasks]


# ---- step / features / satisfies ---------------------------------------------------------
def test_oracle_edge_kats(golden, oracle_mod):
    _, _, _, cfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(cfg)
    for c in golden("kat_edges.json"):
        env = o.env(c["grid"], c["pos"][0], c["pos"][1], c["dir"], c["inv"])
        assert o.step(env, c["action"]) == 0, c["name"]
        assert [int(env["x"][0]), int(env["y"][0])] == c["post_pos"], c["name"]
        assert int(env["dir"][0]) == c["post_dir"], c["name"]
        assert env["inv"][0, :cfg.n_kinds].tolist() == c["post_inv"], c["name"]
        assert env["grid"][0, :64].tolist() == c["post_grid"], c["name"]


@pytest.mark.parametrize("W", [8, 12])
def test_oracle_random_step_kats(golden, oracle_mod, W):
    g = golden("kat_step.npz")
    p = f"w{W}_"
    _, _, tm, cfg = make_tables(world_for(W, 3))
    o = oracle_mod.Oracle(cfg)
    n = len(g[p + "action"])
    for i in range(n):
        x, y, d = g[p + "pre_agent"][i]
        env = o.env(g[p + "pre_grid"][i], x, y, d, g[p + "pre_inv"][i])
        np.testing.assert_array_equal(o.features(env), g[p + "features"][i], err_msg=str(i))
        sats = [o.satisfies(env, t) for t in range(len(tm))]
        assert sats == g[p + "satisfies"][i].tolist(), i
        assert o.step(env, int(g[p + "action"][i])) == 0
        assert [int(env["x"][0]), int(env["y"][0]), int(env["dir"][0])] == g[p + "post_agent"][i].tolist(), i
        assert env["inv"][0, :cfg.n_kinds].tolist() == g[p + "post_inv"][i].tolist(), i
        assert env["grid"][0, :W * W].tolist() == g[p + "post_grid"][i].tolist(), i


def test_oracle_bad_action(oracle_mod):
    _, _, _, cfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(cfg)
    grid = np.zeros((8, 8), dtype=np.uint8)
    grid[0, :] = grid[-1, :] = grid[:, 0] = grid[:, -1] = 1
    env = o.env(grid, 3, 3)
    assert o.step(env, 6) == N.EBADACTION
    assert o.step(env, -1) == N.EBADACTION


# ---- teacher ----------------------------------------------------------------------------------
@pytest.mark.parametrize("split", ["dev", "test"])
def test_oracle_replays_reference_demonstrations(golden, oracle_mod, split):
    """The reference's own data/craft_medium_{split}.json: every teacher action
    along every demonstration, and satisfies() at its end (make_data.py:146-152)."""
    g = golden("devtest.npz")
    _, _, tm, cfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(cfg)
    grids = g[f"{split}_grids"]
    n_steps = 0
    for i in range(len(g[f"{split}_task"])):
        w, t = int(g[f"{split}_world"][i]), int(g[f"{split}_task"][i])
        x, y = g[f"{split}_pos"][i]
        env = o.env(grids[w], x, y, 0)
        for a in g[f"{split}_actions"][i]:
            if a < 0:
                break
            rc, ta = o.teacher(env, t)
            assert rc == 0 and ta == a, (split, i)
            if a != N.STOP:
                assert o.step(env, int(a)) == 0
                n_steps += 1
        assert o.satisfies(env, t) == 1
    assert n_steps > 15000


def test_oracle_teacher_12x12(golden, oracle_mod):
    g = golden("teacher_12x12.npz")
    _, cb, tm, cfg = make_tables("craft_medium_12x12")
    o = oracle_mod.Oracle(cfg)
    for i in range(len(g["grid"])):
        x, y, d = g["agent"][i]
        env = o.env(g["grid"][i], x, y, d, g["inv"][i])
        for t in range(len(tm)):
            rc, a = o.teacher(env, t)
            ref = int(g["action"][i, t])
            if ref == -2:
                assert rc == N.ETEACHER, (i, t)
            else:
                assert rc == 0 and a == ref, (i, t, a, ref)
            ref_len = int(g["path_len"][i, t])
            if ref_len != -3:
                rc, fa, ln = o.closest_resource(env, cfg.task[t].arg_kind)
                if ref_len == -2:
                    assert rc == N.ETEACHER
                else:
                    assert rc == 0 and ln == ref_len, (i, t, ln, ref_len)


# ---- rollout protocol ----------------------------------------------------------------------
@pytest.mark.parametrize("window", [3, 5])
def test_oracle_rollout_fixture(golden, oracle_mod, window):
    g = golden(f"rollout_12x12_w{window}.npz")
    _, _, tm, cfg = make_tables(world_for(12, window))
    o = oracle_mod.Oracle(cfg, g["pool"])
    sp = g["spec"]
    envs = o.init_envs(sp[:, 0], sp[:, 1], sp[:, 2], sp[:, 3], sp[:, 4])
    seed = int(g["seed"][0])
    T = g["done"].shape[0]
    obs_ticks = list(g["obs_ticks"])
    for t in range(T):
        rc, obs, reward, done, success = o.batch_tick(envs, 0, None, seed, t, True)
        assert rc == 0
        np.testing.assert_array_equal(done, g["done"][t])
        np.testing.assert_array_equal(success, g["success"][t])
        np.testing.assert_array_equal(reward, g["reward"][t])
        np.testing.assert_array_equal(np.stack([envs["x"], envs["y"], envs["dir"], envs["timer"]], 1),
                                      g["agent"][t])
        np.testing.assert_array_equal(envs["inv"][:, :cfg.n_kinds], g["inv"][t])
        np.testing.assert_array_equal(envs["grid"][:, :144], g["grid"][t])
        if t in obs_ticks:
            np.testing.assert_array_equal(obs, g["obs"][obs_ticks.index(t)])


def test_hash_action_matches(oracle_mod):
    from psketch_amd.sim import hash_actions
    gids = np.arange(0, 5000, 7)
    for tick in (0, 1, 99, 12345):
        ref = [oracle_mod.hash_action(42, int(g), tick) for g in gids]
        assert hash_actions(42, gids, tick).tolist() == ref


def _imitation_case(golden, case):
    fx = golden("imitation_rollout.npz")
    world = {"dev8": "craft_medium", "w12": "craft_medium_12x12"}[case]
    return fx, world


@pytest.mark.parametrize("case", ["dev8", "w12"])
@pytest.mark.parametrize("mode", ["train", "eval"])
def test_oracle_do_rollout_matches_reference(golden, oracle_mod, case, mode):
    """oracle/rollout_oracle.do_rollout == the reference's ImitationTrainer.do_rollout
    (trainers/imitation.py:18-101) with its DemonstrationTeacher and a fixed student."""
    from oracle import rollout_oracle
    fx, world = _imitation_case(golden, case)
    _, _, _, cfg = make_tables(world)
    orc = oracle_mod.Oracle(cfg, fx[f"{case}_pool"])
    key = f"{case}_{mode}"
    act = rollout_oracle.fake_policy(fx[f"{case}_W"], fx[f"{case}_bias"])
    info = rollout_oracle.do_rollout(orc, fx[f"{case}_spec"], act, mode == "eval",
                                     bc_mask=fx[key + "_bc"])
    A = fx[key + "_action_seqs"]
    for i, seq in enumerate(info["action_seqs"]):
        assert seq == [int(a) for a in A[i] if a >= 0], i
    assert np.array_equal(np.asarray(info["success"], dtype=np.int8), fx[key + "_success"])
    assert info["distances"] == fx[key + "_distances"].tolist()
    assert [info["num_interactions"], info["num_steps"]] == fx[key + "_counts"].tolist()
    R = fx[key + "_received"]
    assert np.array_equal(np.asarray(info["received"], dtype=np.int8).reshape(R.shape), R)


@pytest.mark.parametrize("name,world,count", [("w8", "craft_medium", 100), ("w12", "craft_medium_12x12", 64)])
def test_oracle_generator_reproduces_reference_scenarios(golden, oracle_mod, name, world, count):
    """oracle_generate_scenarios with numpy's RandomState stream == the reference's
    make_data.sample_scenario (with its duplicate check): every grid, every initial
    position, and the MT19937 state after the last draw."""
    from psketch_amd.cookbook import generator_primitives
    fx = golden("scenarios_seed123.npz")
    params, cb, _, _ = make_tables(world)
    ws = [cb.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])]
    grids, init, mt = oracle_mod.generate_scenarios(
        params["WIDTH"], params["HEIGHT"], cb.index["boundary"], generator_primitives(cb),
        params["N_PRIMITIVES"], ws, count, 123, rng="mt19937", dedup=True)
    assert np.array_equal(grids, fx[f"{name}_grids"])
    assert np.array_equal(init, fx[f"{name}_init"])
    assert np.array_equal(mt[:624], fx[f"{name}_mt_key"]) and mt[624] == fx[f"{name}_mt_pos"][0]


def check_scenario_invariants(grids, init, W, H, boundary, prims, n_per, ws):
    """What every make_data world satisfies: the boundary ring, the object counts,
    one connected free region, every interior object next to a free cell, and a
    free interior initial position that keeps both properties when occupied."""
    from scipy import ndimage
    g = grids.reshape(-1, W, H)
    ring = np.zeros((W, H), bool)
    ring[0, :] = ring[-1, :] = ring[:, 0] = ring[:, -1] = True
    assert (g[:, ring] == boundary).all()
    for k in prims:
        assert ((g == k).sum(axis=(1, 2)) == n_per).all()
    for k in ws:
        assert ((g == k).sum(axis=(1, 2)) == 1).all()
    n_obj = len(prims) * n_per + len(ws)
    assert ((g[:, ~ring] != 0).sum(axis=1) == n_obj).all()
    cross = ndimage.generate_binary_structure(2, 1)
    for i in range(len(g)):
        x, y = init[i]
        assert 0 < x < W - 1 and 0 < y < H - 1 and g[i, x, y] == 0
        occ = g[i] != 0
        occ2 = occ.copy()
        occ2[x, y] = True
        for o in (occ, occ2):
            _, ncomp = ndimage.label(~o, structure=cross)
            assert ncomp == 1, i
            free_nb = ndimage.binary_dilation(~o, structure=cross)
            assert free_nb[o & ~ring].all(), i


def test_oracle_splitmix_generator_invariants(oracle_mod):
    from psketch_amd.cookbook import generator_primitives
    params, cb, _, _ = make_tables("craft_large")
    W, H = params["WIDTH"], params["HEIGHT"]
    prims = generator_primitives(cb)
    ws = [cb.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])]
    grids, init, _ = oracle_mod.generate_scenarios(W, H, cb.index["boundary"], prims,
                                                   params["N_PRIMITIVES"], ws, 300, 9)
    check_scenario_invariants(grids, init, W, H, cb.index["boundary"], prims, params["N_PRIMITIVES"], ws)
    # keyed by global id: any split of the ids gives the same worlds
    g2, i2, _ = oracle_mod.generate_scenarios(W, H, cb.index["boundary"], prims, params["N_PRIMITIVES"],
                                              ws, 100, 9, scenario_id0=200)
    assert np.array_equal(g2, grids[200:]) and np.array_equal(i2, init[200:])


def _language_codes_from_oracle(oracle_mod, fx):
    """Transition codes of the fixture's rollout, from the oracle's states."""
    from psketch_amd.language import codes_from_states
    _, _, _, cfg = make_tables("craft_medium_12x12")
    orc = oracle_mod.Oracle(cfg)
    pool, spec, actions = fx["pool"], fx["spec"], fx["actions"]
    envs = [orc.env(pool[sc], x, y, d) for sc, x, y, d in spec]
    T, B = actions.shape
    codes = np.zeros((T, B), dtype=np.int8)
    for t in range(T):
        for i in range(B):
            e = envs[i]
            p0, inv0 = (int(e["x"][0]), int(e["y"][0])), e["inv"][0].copy()
            assert orc.step(e, int(actions[t, i])) == 0
            codes[t, i] = codes_from_states(p0, (int(e["x"][0]), int(e["y"][0])), inv0, e["inv"][0])
    return codes


def test_language_teacher_matches_reference(golden, oracle_mod):
    """psketch_amd.language.PrimitiveLanguageTeacher == the reference's
    describe / instruct (teachers/primitive_language.py:17-90): one-action calls
    env by env with one shared teacher, whole-sequence calls with fresh teachers,
    the learned action map, and the same RandomState draws."""
    from psketch_amd.language import WORDS, PrimitiveLanguageTeacher
    fx = golden("language.npz")
    codes = _language_codes_from_oracle(oracle_mod, fx)
    actions = fx["actions"]
    T, B = actions.shape
    teacher = PrimitiveLanguageTeacher(np.random.RandomState(5))
    got = [teacher.describe_batch(actions[t], codes[t]) for t in range(T)]
    assert [[WORDS.index(w) for w in row] for row in got] == fx["desc_tick"].tolist()
    assert sorted((k, WORDS.index(v)) for k, v in teacher.student_action_map.items()) == \
        [tuple(r) for r in fx["map_tick"].tolist()]
    for i in range(B):
        t2 = PrimitiveLanguageTeacher(np.random.RandomState(100 + i))
        d = t2.describe_codes(actions[:, i], codes[:, i])
        assert [WORDS.index(w) for w in d] == fx["desc_seq"][i].tolist(), i
    for i in range(len(fx["instruct"])):
        assert [WORDS.index(w) for w in teacher.instruct(None, actions[:, i])] == fx["instruct"][i].tolist()


# ---- the numpy CPU leg of bench.py's cpu_baseline --------------------------------------------
@pytest.mark.parametrize("window", [3, 5])
def test_numpy_restatement_matches_reference_rollout(golden, window):
    """oracle/craft_numpy.py (the Python CPU comparator) replays the reference's own
    100-tick random rollout (tests/golden/rollout_12x12_w3.npz) observation for
    observation: step craft.py:332-424, features craft.py:296-330."""
    from oracle.craft_numpy import NumpyWorld
    g = golden(f"rollout_12x12_w{window}.npz")
    _, _, tm, cfg = make_tables(world_for(12, window))
    w = NumpyWorld(cfg)
    batch = w.start([w.onehot(p) for p in g["pool"]], g["spec"])
    seed = int(g["seed"][0])
    obs_ticks = list(g["obs_ticks"])
    for t in range(g["done"].shape[0]):
        rec = []
        w.tick(batch, 0, seed, t, rec)
        obs, reward, done, success = rec[0]
        np.testing.assert_array_equal(done, g["done"][t])
        np.testing.assert_array_equal(success, g["success"][t])
        np.testing.assert_array_equal(reward, g["reward"][t])
        pos = np.asarray([s["pos"] for s in batch["states"]])
        np.testing.assert_array_equal(pos, g["agent"][t][:, :2])
        if t in obs_ticks:
            np.testing.assert_array_equal(obs, g["obs"][obs_ticks.index(t)])


def test_oracle_config1_random_rollout(golden, oracle_mod):
    """BASELINE configs[0]: the reference's 100-step random rollout of the first
    craft_medium_train.json instance (tests/golden/config1_train0.npz), replayed
    step by step through the oracle: pos, dir, inventory, grid, features and
    satisfies after every step (craft.py:285-424)."""
    g = golden("config1_train0.npz")
    _, _, tm, cfg = make_tables("craft_medium")
    o = oracle_mod.Oracle(cfg)
    x, y = (int(v) for v in g["init_pos"])
    env = o.env(g["grid"][0], x, y, 0)
    task = int(g["task"][0])
    for t in range(len(g["actions"]) + 1):
        if t:
            assert o.step(env, int(g["actions"][t - 1])) == 0
        assert (int(env["x"][0]), int(env["y"][0])) == tuple(g["pos"][t])
        assert int(env["dir"][0]) == g["dir"][t]
        np.testing.assert_array_equal(env["inv"][0, :cfg.n_kinds], g["inv"][t])
        np.testing.assert_array_equal(env["grid"][0, :64], g["grid"][t])
        np.testing.assert_array_equal(o.features(env), g["features"][t].astype(np.float32))
        assert o.satisfies(env, task) == g["satisfies"][t]
    assert o.teacher(o.env(g["grid"][0], x, y, 0), task) == (0, int(g["demo"][0]))
