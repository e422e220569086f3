"""Generates tests/golden/* by running the REFERENCE's own Python code.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py

What it imports from the reference: worlds (CraftWorld/CraftState/Cookbook),
data.task (TaskManager), teachers (DemonstrationTeacher), misc.util, and the
function definitions of make_data.py (the script body is not executed: its
FunctionDefs are compiled with `world` injected, make_data.py:50 reads it as a
global).  Two libraries the reference imports are absent from this image:
  * skimage (scikit-image, version unpinned by the reference) — craft.py:12
    imports skimage.measure.block_reduce for the pooled features (craft.py:308-310).
    It is replaced by a restatement of its published algorithm: pad the array
    to a block multiple with `cval`, view it as blocks, reduce each block with
    `func`.  The windows used here (9/3, 25/5) divide evenly, so no padding
    occurs; ONLY the pooled section of features() depends on this stand-in.
  * jsonargparse — flags.py is not used; configs are built as misc.util.Struct.
The reference source never enters the repository: only the data it produced.
"""
import ast
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))


def _block_reduce(image, block_size, func=np.sum, cval=0):
    image = np.asarray(image)
    pad = []
    for n, b in zip(image.shape, block_size):
        r = n % b
        pad.append((0, (b - r) if r else 0))
    image = np.pad(image, pad, mode="constant", constant_values=cval)
    shape = []
    for n, b in zip(image.shape, block_size):
        shape += [n // b, b]
    blocks = image.reshape(shape)
    axes = tuple(range(1, 2 * image.ndim, 2))
    return func(blocks, axis=axes)


def import_reference():
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.measure")
    skm.block_reduce = _block_reduce
    sk.measure = skm
    sys.modules["skimage"] = sk
    sys.modules["skimage.measure"] = skm
    sys.dont_write_bytecode = True
    os.chdir(REF)                       # craft.py:62-63 opens configs relative to CWD
    sys.path.insert(0, REF)
    import worlds  # noqa
    import teachers  # noqa
    from misc import util  # noqa
    from data.task import TaskManager  # noqa
    return worlds, teachers, util, TaskManager


worlds, teachers, util, TaskManager = import_reference()


def make_config(world_yaml="craft_medium", seed=123):
    cfg = util.Struct(recipes="resources/craft/recipes.yaml",
                      world={"name": "CraftWorld", "config": world_yaml},
                      student={"model": {}}, teacher={"name": "DemonstrationTeacher"},
                      trainer={"hints": "resources/craft/hints.hierarchy.yaml", "batch_size": 32,
                               "max_timesteps": 40})
    cfg.random = np.random.RandomState(seed)
    return cfg


def make_world(W=None, window=None, seed=123):
    cfg = make_config(seed=seed)
    world = worlds.load(cfg)
    if W is not None:
        world.WIDTH = world.HEIGHT = W
    if window is not None:
        world.WINDOW_WIDTH = world.WINDOW_HEIGHT = window
        world.n_features = 2 * window * window * world.cookbook.n_kinds + world.cookbook.n_kinds + 5
    return cfg, world


def make_data_functions(world):
    """The FunctionDefs of make_data.py, bound to `world` (make_data.py:50)."""
    src = open(os.path.join(REF, "make_data.py")).read()
    tree = ast.parse(src)
    mod = ast.Module(body=[n for n in tree.body if isinstance(n, ast.FunctionDef)], type_ignores=[])
    ns = {"np": np, "world": world}
    exec(compile(mod, "make_data.py", "exec"), ns)
    return ns


def onehot_to_ids(grid):
    g = np.asarray(grid)
    assert (g.sum(axis=2) <= 1).all()
    return (g.argmax(axis=2) * (g.max(axis=2) > 0)).astype(np.uint8)


def ids_to_onehot(ids, K):
    ids = np.asarray(ids)
    g = np.zeros(ids.shape + (K,))
    for k in range(1, K):
        g[..., k] = ids == k
    return g


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash_action(seed, gid, tick):
    key = np.uint64(seed) ^ (np.uint64(gid) << np.uint64(20)) ^ np.uint64(tick)
    return int((splitmix64(key) >> np.uint64(32)) % np.uint64(6))


# --------------------------------------------------------------------------------------
def gen_cookbook():
    cfg, world = make_world()
    cb = world.cookbook
    tm = TaskManager(cfg)
    out = {
        "index": list(cb.index.ordered_contents),
        "n_kinds": cb.n_kinds,
        "environment_iter": list(cb.environment),
        "primitives_iter": list(cb.primitives),
        "recipes": [[out_k, {str(k): v for k, v in d.items()}] for out_k, d in cb.recipes.items()],
        "grabbable_indices": list(world.grabbable_indices),
        "workshop_indices": list(world.workshop_indices),
        "water_index": world.water_index,
        "stone_index": world.stone_index,
        "n_features": {"craft_medium": world.n_features},
        "tasks": [[t.goal_name, t.goal_arg, [f"{s.goal_name}[{s.goal_arg}]" for s in (t.subtasks or [])]]
                  for t in tm.tasks],
        "actions": {name: [getattr(world.actions, name).index,
                           list(getattr(world.actions, name).coord_change)]
                    for name in ["DOWN", "UP", "LEFT", "RIGHT", "USE", "STOP"]},
    }
    for name, W, w in [("craft_medium_12x12", 12, 3), ("craft_medium_12x12_w5", 12, 5),
                       ("craft_large", 10, 5)]:
        _, wd = make_world(W, w)
        out["n_features"][name] = wd.n_features
    with open(os.path.join(OUT, "cookbook.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("cookbook.json", out["n_kinds"], out["primitives_iter"])
    return cfg, world, tm


def gen_devtest(tm):
    """The reference's committed demonstrations, compacted (kind ids)."""
    task_ids = {f"{t.goal_name}[{t.goal_arg}]": i for i, t in enumerate(tm.tasks)}
    arrays = {}
    for split in ["dev", "test"]:
        data = json.load(open(os.path.join(REF, "data", f"craft_medium_{split}.json")))
        grids, world_idx, task_idx, pos, acts, ids = [], [], [], [], [], []
        for wi, item in enumerate(data):
            grids.append(onehot_to_ids(item["grid"]).reshape(-1))
            for ti in item["task_instances"]:
                for p, iid, ra in zip(ti["init_pos"], ti["ids"], ti["ref_actions"]):
                    world_idx.append(wi)
                    task_idx.append(task_ids[ti["task"]])
                    pos.append(p)
                    acts.append(ra)
                    ids.append(int(iid.split("_")[1]))
        L = max(len(a) for a in acts)
        A = np.full((len(acts), L), -1, dtype=np.int8)
        for i, a in enumerate(acts):
            A[i, :len(a)] = a
        arrays[f"{split}_grids"] = np.stack(grids)
        arrays[f"{split}_world"] = np.asarray(world_idx, dtype=np.int16)
        arrays[f"{split}_task"] = np.asarray(task_idx, dtype=np.int16)
        arrays[f"{split}_pos"] = np.asarray(pos, dtype=np.int8)
        arrays[f"{split}_actions"] = A
        arrays[f"{split}_ids"] = np.asarray(ids, dtype=np.int32)
        print(split, len(acts), "instances, max len", L)
    np.savez_compressed(os.path.join(OUT, "devtest.npz"), **arrays)


def gen_scenarios():
    """sample_scenario streams from RandomState(123): all 100 worlds of the
    8x8 dataset run (make_data.py:166-178 with its duplicate check) and the
    first 64 worlds at 12x12."""
    arrays = {}
    for name, W, count in [("w8", 8, 100), ("w12", 12, 64)]:
        cfg, world = make_world(W)
        fns = make_data_functions(world)
        ingredients = [world.cookbook.index[i] for i in ["wood", "grass", "iron"]]
        grids, inits = [], []
        while len(grids) < count:
            grid, init_pos = fns["sample_scenario"](world, ingredients, cfg)
            if any((grid == g).all() for g in grids):
                continue
            grids.append(grid)
            inits.append(init_pos)
        arrays[f"{name}_grids"] = np.stack([onehot_to_ids(g).reshape(-1) for g in grids])
        arrays[f"{name}_init"] = np.asarray(inits, dtype=np.int32)
        st = cfg.random.get_state()
        arrays[f"{name}_mt_key"] = np.asarray(st[1], dtype=np.uint32)
        arrays[f"{name}_mt_pos"] = np.asarray([st[2]], dtype=np.int32)
        print("scenarios", name, arrays[f"{name}_grids"].shape)
    np.savez_compressed(os.path.join(OUT, "scenarios_seed123.npz"), **arrays)
    return arrays


def gen_rollout(w12_grids, window, T, E, P, all_obs_ticks):
    """Synthetic random-action rollouts through the reference's CraftState,
    with ImitationTrainer.do_rollout's per-env protocol (imitation.py:59-73)
    and auto-reset to the env's initial state."""
    cfg, world = make_world(12, window)
    tm = TaskManager(cfg)
    K = world.cookbook.n_kinds
    W = H = 12
    task_objs = list(tm.tasks)
    task_list = [i for i, t in enumerate(task_objs) if t.goal_name in ("get", "make")]
    pool = w12_grids[:P]
    seed = 7
    gid = np.arange(E)
    scen = gid % P
    rng = np.random.RandomState(99)
    xs, ys, dirs = [], [], []
    for e in range(E):
        g = pool[scen[e]].reshape(W, H)
        free = [(x, y) for x in range(1, W - 1) for y in range(1, H - 1) if g[x, y] == 0]
        x, y = free[rng.randint(len(free))]
        xs.append(x); ys.append(y); dirs.append(rng.randint(4))
    tasks = np.asarray([task_list[e % len(task_list)] for e in range(E)])
    onehots = [ids_to_onehot(pool[p].reshape(W, H), K) for p in range(P)]

    def init(e):
        return world.init_state(onehots[scen[e]], (xs[e], ys[e]), dirs[e])

    states = [init(e) for e in range(E)]
    timer = [40] * E
    F = world.n_features
    rec = {k: [] for k in ["agent", "inv", "grid", "done", "success", "reward", "actions"]}
    obs_all = np.zeros((T, E, F), dtype=np.uint8)
    for t in range(T):
        row = {k: [] for k in rec}
        for e in range(E):
            a = hash_action(seed, e, t)
            timer[e] -= 1
            d = a == 5 or timer[e] <= 0
            if d:
                s = states[e].satisfies(task_objs[tasks[e]])
                succ = int(bool(s))
                states[e] = init(e)
                timer[e] = 40
            else:
                _, states[e] = states[e].step(a)
                succ = -1
            st = states[e]
            row["actions"].append(a)
            row["done"].append(int(d))
            row["success"].append(succ)
            row["reward"].append(1 if (d and succ == 1) else 0)
            row["agent"].append([st.pos[0], st.pos[1], st.dir, timer[e]])
            row["inv"].append(np.asarray(st.inventory, dtype=np.int64))
            row["grid"].append(onehot_to_ids(st.grid).reshape(-1))
            f = st.features()
            assert len(f) == F
            obs_all[t, e] = f.astype(np.uint8)
            assert (obs_all[t, e] == f).all()
        for k in rec:
            rec[k].append(row[k])
    arrays = {k: np.asarray(v) for k, v in rec.items()}
    arrays["agent"] = arrays["agent"].astype(np.int16)
    arrays["inv"] = arrays["inv"].astype(np.uint8)
    arrays["grid"] = arrays["grid"].astype(np.uint8)
    arrays["done"] = arrays["done"].astype(np.uint8)
    arrays["success"] = arrays["success"].astype(np.int8)
    arrays["reward"] = arrays["reward"].astype(np.uint8)
    arrays["actions"] = arrays["actions"].astype(np.int8)
    ticks = np.arange(T) if all_obs_ticks is None else np.asarray(all_obs_ticks)
    arrays["obs_ticks"] = ticks
    arrays["obs"] = obs_all[ticks]
    arrays["pool"] = pool
    arrays["spec"] = np.stack([scen, xs, ys, dirs, tasks], axis=1).astype(np.int32)
    arrays["seed"] = np.asarray([seed])
    name = f"rollout_12x12_w{window}.npz"
    np.savez_compressed(os.path.join(OUT, name), **arrays)
    print(name, os.path.getsize(os.path.join(OUT, name)))


def random_state_cases(n, W, seed):
    """Random grids with the boundary ring and arbitrary interior kinds."""
    cfg, world = make_world(W)
    tm = TaskManager(cfg)
    K = world.cookbook.n_kinds
    rng = np.random.RandomState(seed)
    cases = []
    for i in range(n):
        g = np.zeros((W, W), dtype=np.int64)
        g[0, :] = g[-1, :] = g[:, 0] = g[:, -1] = 1
        dens = rng.uniform(0.1, 0.6)
        inner = rng.randint(1, K, size=(W - 2, W - 2))
        inner[rng.uniform(size=inner.shape) > dens] = 0
        g[1:-1, 1:-1] = inner
        x, y = rng.randint(1, W - 1, size=2)
        if rng.uniform() < 0.9:
            g[x, y] = 0
        d = rng.randint(4)
        inv = np.zeros(K, dtype=np.int64)
        nz = rng.randint(0, 6)
        for k in rng.randint(1, K, size=nz):
            inv[k] += rng.randint(1, 3)
        a = rng.randint(6)
        cases.append((g, x, y, d, inv, a))
    return cfg, world, tm, cases


def gen_kat_step():
    arrays = {}
    for W in (8, 12):
        cfg, world, tm, cases = random_state_cases(1500, W, 1000 + W)
        K = world.cookbook.n_kinds
        pre_grid, pre_agent, pre_inv, act = [], [], [], []
        post_grid, post_agent, post_inv, feats, sats = [], [], [], [], []
        for g, x, y, d, inv, a in cases:
            st = world.init_state(ids_to_onehot(g, K), (int(x), int(y)), int(d))
            st.inventory = inv.astype(np.float64)
            f = st.features().astype(np.uint8)
            s_all = []
            for t in tm.tasks:
                try:
                    s = st.satisfies(t)
                    s_all.append(-1 if s is None else int(bool(s)))
                except Exception:
                    s_all.append(-9)
            _, st2 = st.step(int(a))
            pre_grid.append(g.reshape(-1)); pre_agent.append([x, y, d]); pre_inv.append(inv)
            act.append(a)
            post_grid.append(onehot_to_ids(st2.grid).reshape(-1))
            post_agent.append([st2.pos[0], st2.pos[1], st2.dir])
            post_inv.append(np.asarray(st2.inventory, dtype=np.int64))
            feats.append(f)
            sats.append(s_all)
        p = f"w{W}_"
        arrays[p + "pre_grid"] = np.asarray(pre_grid, dtype=np.uint8)
        arrays[p + "pre_agent"] = np.asarray(pre_agent, dtype=np.int8)
        arrays[p + "pre_inv"] = np.asarray(pre_inv, dtype=np.uint8)
        arrays[p + "action"] = np.asarray(act, dtype=np.int8)
        arrays[p + "post_grid"] = np.asarray(post_grid, dtype=np.uint8)
        arrays[p + "post_agent"] = np.asarray(post_agent, dtype=np.int8)
        arrays[p + "post_inv"] = np.asarray(post_inv, dtype=np.uint8)
        arrays[p + "features"] = np.asarray(feats, dtype=np.uint8)
        arrays[p + "satisfies"] = np.asarray(sats, dtype=np.int8)
    np.savez_compressed(os.path.join(OUT, "kat_step.npz"), **arrays)
    print("kat_step.npz", os.path.getsize(os.path.join(OUT, "kat_step.npz")))


def gen_kat_edges():
    """Hand-built edge cases of step() (SURVEY.md §7 hard parts), 8x8."""
    cfg, world = make_world()
    cb = world.cookbook
    K = cb.n_kinds
    I = cb.index
    cases = []

    def case(name, cells, pos, d, inv, action):
        g = np.zeros((8, 8), dtype=np.int64)
        g[0, :] = g[-1, :] = g[:, 0] = g[:, -1] = I["boundary"]
        for (x, y), k in cells.items():
            g[x, y] = I[k]
        iv = np.zeros(K)
        for k, c in inv.items():
            iv[I[k]] = c
        st = world.init_state(ids_to_onehot(g, K), pos, d)
        st.inventory = iv
        _, s2 = st.step(action)
        cases.append({
            "name": name, "grid": g.reshape(-1).tolist(), "pos": list(pos), "dir": d,
            "inv": iv.astype(int).tolist(), "action": action,
            "post_grid": onehot_to_ids(s2.grid).reshape(-1).tolist(),
            "post_pos": [int(s2.pos[0]), int(s2.pos[1])], "post_dir": int(s2.dir),
            "post_inv": np.asarray(s2.inventory).astype(int).tolist(),
        })

    R, L, U, D_, USE, STOP = 3, 2, 1, 0, 4, 5
    case("chain_ws1_wood_iron_to_shears", {(4, 3): "workshop1"}, (3, 3), R, {"wood": 1, "iron": 1}, USE)
    case("ws0_plank_axe_rope_order", {(4, 3): "workshop0"}, (3, 3), R, {"wood": 2, "stick": 1, "iron": 1, "grass": 1}, USE)
    case("ws2_bridge_then_ladder", {(4, 3): "workshop2"}, (3, 3), R, {"wood": 1, "iron": 1, "plank": 1, "stick": 1, "grass": 2}, USE)
    case("ws1_nothing_held", {(4, 3): "workshop1"}, (3, 3), R, {}, USE)
    case("ws_one_application_per_recipe", {(4, 3): "workshop1"}, (3, 3), R, {"wood": 3}, USE)
    case("water_with_bridge", {(3, 4): "water"}, (3, 3), U, {"bridge": 2}, USE)
    case("water_without_bridge", {(3, 4): "water"}, (3, 3), U, {}, USE)
    case("stone_with_axe_keeps_axe", {(2, 3): "stone"}, (3, 3), L, {"axe": 1}, USE)
    case("stone_without_axe", {(2, 3): "stone"}, (3, 3), L, {}, USE)
    case("use_boundary_noop", {}, (1, 3), L, {"wood": 1}, USE)
    case("use_empty_noop", {}, (3, 3), D_, {}, USE)
    case("grab_wood", {(3, 2): "wood"}, (3, 3), D_, {"wood": 1}, USE)
    case("grab_gold", {(3, 2): "gold"}, (3, 3), D_, {}, USE)
    case("grab_crafted_item_on_grid", {(3, 2): "ladder"}, (3, 3), D_, {}, USE)
    case("blocked_move_turns", {(4, 3): "iron"}, (3, 3), D_, {}, R)
    case("blocked_by_boundary_turns", {}, (1, 1), R, {}, L)
    case("free_move", {}, (3, 3), R, {}, U)
    case("stop_keeps_dir", {}, (3, 3), L, {}, STOP)
    case("use_keeps_dir_and_pos", {(4, 3): "grass"}, (3, 3), R, {}, USE)
    case("move_into_water_blocked", {(3, 4): "water"}, (3, 3), D_, {}, U)
    with open(os.path.join(OUT, "kat_edges.json"), "w") as f:
        json.dump(cases, f)
    print("kat_edges.json", len(cases))


def gen_teacher(w12_grids, n_states=400):
    """DemonstrationTeacher actions and find_closest_resources lengths on 12x12
    worlds, random positions/directions/inventories, every task."""
    cfg, world = make_world(12)
    tm = TaskManager(cfg)
    teacher = teachers.load(cfg)
    K = world.cookbook.n_kinds
    I = world.cookbook.index
    rng = np.random.RandomState(5)
    items = ["wood", "grass", "iron", "plank", "stick", "axe", "rope", "bridge"]
    grids, agents, invs, acts, lens = [], [], [], [], []
    for i in range(n_states):
        g = w12_grids[rng.randint(len(w12_grids))].reshape(12, 12).astype(np.int64).copy()
        # sometimes remove a resource (as grabbing does) to vary the targets
        for _ in range(rng.randint(0, 3)):
            cells = [(x, y) for x in range(12) for y in range(12) if g[x, y] in (7, 8, 9)]
            if cells:
                x, y = cells[rng.randint(len(cells))]
                g[x, y] = 0
        free = [(x, y) for x in range(1, 11) for y in range(1, 11) if g[x, y] == 0]
        x, y = free[rng.randint(len(free))]
        d = rng.randint(4)
        inv = np.zeros(K)
        for k in rng.choice(items, size=rng.randint(0, 4)):
            inv[I[k]] += 1
        st = world.init_state(ids_to_onehot(g, K), (x, y), d)
        st.inventory = inv
        row_a, row_l = [], []
        for t in tm.tasks:
            try:
                a = teacher(t, st)
            except (AssertionError, TypeError, IndexError):
                a = -2
            row_a.append(a)
            if I[t.goal_arg] is not None:
                try:
                    _, seq = teacher.find_closest_resources(t, st)
                    row_l.append(-1 if seq is None else len(seq))
                except TypeError:
                    row_l.append(-2)
            else:
                row_l.append(-3)
        grids.append(g.reshape(-1)); agents.append([x, y, d]); invs.append(inv)
        acts.append(row_a); lens.append(row_l)
    np.savez_compressed(os.path.join(OUT, "teacher_12x12.npz"),
                        grid=np.asarray(grids, dtype=np.uint8), agent=np.asarray(agents, dtype=np.int8),
                        inv=np.asarray(invs, dtype=np.uint8), action=np.asarray(acts, dtype=np.int8),
                        path_len=np.asarray(lens, dtype=np.int16))
    print("teacher_12x12.npz", np.unique(np.asarray(acts), return_counts=True))


def fake_policy_weights(F, seed=11):
    """A deterministic integer 'student' for the rollout fixtures: action =
    argmax(features @ Wt[t % 3] * 8 + bias), exact in fp32 and float64 alike."""
    rng = np.random.RandomState(seed)
    Wt = rng.randint(-3, 4, size=(3, F, 6)).astype(np.int8)
    bias = np.asarray([0, 1, 2, 3, 4, -64], dtype=np.int32)
    return Wt, bias


def load_imitation_trainer():
    """trainers/imitation.py alone (trainers/__init__ pulls in the language
    trainers, which this fixture does not need)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_trainers_imitation",
                                                  os.path.join(REF, "trainers", "imitation.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.ImitationTrainer


class FakeStudent:
    """students/imitation.py's protocol (init/act/receive) around fake_policy_weights."""

    def __init__(self, Wt, bias):
        self.Wt, self.bias = Wt.astype(np.int64), bias.astype(np.int64)

    def init(self, tasks, states, is_eval):
        self.t = 0
        self.received = []

    def act(self, states):
        f = np.stack([s.features() for s in states]).astype(np.int64)
        scores = f @ self.Wt[self.t % 3] * 8 + self.bias
        self.t += 1
        return [int(a) for a in scores.argmax(axis=1)]

    def receive(self, ref_actions):
        self.received.append(list(ref_actions))


def gen_imitation(w12_grids):
    """ImitationTrainer.do_rollout (trainers/imitation.py:18-101) run by the
    reference with its DemonstrationTeacher and a deterministic fake student:
    (a) the first 256 craft_medium dev instances, policy mix 0.5 and eval;
    (b) 256 envs on 12x12 sampled worlds, policy mix 0.3."""
    Trainer = load_imitation_trainer()
    arrays = {}
    for case in ["dev8", "w12"]:
        if case == "dev8":
            cfg, world = make_world()
            data = json.load(open(os.path.join(REF, "data", "craft_medium_dev.json")))
        else:
            cfg, world = make_world(12, 3)
        tm = TaskManager(cfg)
        task_ids = {f"{t.goal_name}[{t.goal_arg}]": i for i, t in enumerate(tm.tasks)}
        K = world.cookbook.n_kinds
        W = world.WIDTH
        teacher = teachers.load(cfg)
        batch, spec = [], []
        if case == "dev8":
            pool = []
            for item in data:
                ids = onehot_to_ids(item["grid"]).reshape(-1)
                pool.append(ids)
                for ti in item["task_instances"]:
                    for p in ti["init_pos"]:
                        batch.append({"task": tm[ti["task"]], "grid": np.array(item["grid"]),
                                      "init_pos": tuple(p)})
                        spec.append([len(pool) - 1, p[0], p[1], 0, task_ids[ti["task"]]])
            batch, spec = batch[:256], spec[:256]
            mix = 0.5
        else:
            pool = list(w12_grids[:32])
            rng = np.random.RandomState(21)
            tasks = [i for i, t in enumerate(tm.tasks) if t.goal_name in ("get", "make")]
            for e in range(256):
                sc = e % len(pool)
                g = pool[sc].reshape(W, W)
                free = [(x, y) for x in range(1, W - 1) for y in range(1, W - 1) if g[x, y] == 0]
                x, y = free[rng.randint(len(free))]
                tk = tasks[rng.randint(len(tasks))]
                batch.append({"task": list(tm.tasks)[tk],
                              "grid": ids_to_onehot(g, K), "init_pos": (x, y)})
                spec.append([sc, x, y, 0, tk])
            mix = 0.3
        Wt, bias = fake_policy_weights(world.n_features)
        student = FakeStudent(Wt, bias)
        cfg.random = np.random.RandomState(77)
        trainer = Trainer(cfg)
        trainer.policy_mix_rate = mix
        for is_eval in [False, True]:
            st = cfg.random.get_state()
            bc = np.random.RandomState(0)
            bc.set_state(st)
            bc_mask = bc.binomial(1, mix, size=len(batch)) if not is_eval else np.zeros(len(batch), int)
            info = trainer.do_rollout(batch, world, student, teacher, is_eval)
            key = f"{case}_{'eval' if is_eval else 'train'}"
            L = max(len(a) for a in info["action_seqs"])
            A = np.full((len(batch), 40), -1, dtype=np.int8)
            for i, a in enumerate(info["action_seqs"]):
                A[i, :len(a)] = a
            arrays[key + "_action_seqs"] = A
            arrays[key + "_success"] = np.asarray(info["success"], dtype=np.int8)
            arrays[key + "_distances"] = np.asarray(info["distances"], dtype=np.int16)
            arrays[key + "_counts"] = np.asarray([info["num_interactions"], info["num_steps"]],
                                                 dtype=np.int64)
            arrays[key + "_bc"] = bc_mask.astype(np.uint8)
            R = np.asarray(student.received, dtype=np.int8) if student.received else \
                np.zeros((0, len(batch)), dtype=np.int8)
            arrays[key + "_received"] = R
            print("imitation", key, "ticks", len(student.received) or student.t, "max len", L,
                  "success", int(np.sum(info["success"])), "counts", arrays[key + "_counts"])
        arrays[case + "_pool"] = np.stack(pool).astype(np.uint8)
        arrays[case + "_spec"] = np.asarray(spec, dtype=np.int32)
        arrays[case + "_W"] = Wt
        arrays[case + "_bias"] = bias
    np.savez_compressed(os.path.join(OUT, "imitation_rollout.npz"), **arrays)
    print("imitation_rollout.npz", os.path.getsize(os.path.join(OUT, "imitation_rollout.npz")))


def gen_language(w12_grids):
    """PrimitiveLanguageTeacher.describe / instruct (teachers/primitive_language.py:17-90)
    run by the reference on random 12x12 rollouts: (1) one-action calls env by env
    each tick, sharing one teacher, as trainers/interactive_primitive_language.py:55-68
    calls it; (2) whole-sequence calls with a fresh teacher per env."""
    cfg, world = make_world(12, 3)
    cfg.teacher = util.Struct(name="PrimitiveLanguageTeacher")
    K = world.cookbook.n_kinds
    rng = np.random.RandomState(31)
    B, T = 64, 30
    pool = w12_grids[:16]
    spec, states = [], []
    for e in range(B):
        sc = e % len(pool)
        g = pool[sc].reshape(12, 12)
        free = [(x, y) for x in range(1, 11) for y in range(1, 11) if g[x, y] == 0]
        x, y = free[rng.randint(len(free))]
        d = rng.randint(4)
        spec.append([sc, x, y, d])
        states.append(world.init_state(ids_to_onehot(g, K), (x, y), d))
    actions = rng.randint(0, 6, size=(T, B))
    cfg.random = np.random.RandomState(5)
    teacher = teachers.load(cfg)
    desc1, seqs = [], [[s] for s in states]
    for t in range(T):
        row = []
        for i in range(B):
            prev = states[i]
            _, states[i] = prev.step(int(actions[t, i]))
            seqs[i].append(states[i])
            row.append(teacher.describe(world, [int(actions[t, i])], [prev, states[i]])[0])
        desc1.append(row)
    map1 = sorted((int(k), v) for k, v in teacher.student_action_map.items())
    desc2 = []
    for i in range(B):
        t2 = teachers.load(cfg)
        t2.random = np.random.RandomState(100 + i)
        desc2.append(t2.describe(world, [int(a) for a in actions[:, i]], seqs[i]))
    instr = [teacher.instruct(world, [int(a) for a in actions[:, i]]) for i in range(4)]
    words = ["down", "up", "left", "right", "use", "stop"]
    enc = lambda ws: np.asarray([words.index(w) for w in ws], dtype=np.int8)  # noqa: E731
    np.savez_compressed(os.path.join(OUT, "language.npz"),
                        pool=np.asarray(pool, dtype=np.uint8), spec=np.asarray(spec, dtype=np.int32),
                        actions=actions.astype(np.int8),
                        desc_tick=np.stack([enc(r) for r in desc1]),
                        map_tick=np.asarray([[k, words.index(v)] for k, v in map1], dtype=np.int8),
                        desc_seq=np.stack([enc(r) for r in desc2]),
                        instruct=np.stack([enc(r) for r in instr]))
    print("language.npz", len(map1), "map entries;", os.path.getsize(os.path.join(OUT, "language.npz")))


def gen_config1(T=100, seed=1):
    """BASELINE configs[0]: one CraftWorld env on the first instance of the
    regenerated craft_medium_train.json, a 100-step random rollout on the
    reference's CPU worlds/craft.py.

    The train split is regenerated with make_data.py's own functions and
    RandomState(123) stream (make_data.py:154-238): 100 de-duplicated worlds,
    then per world and per get/make task 20 distinct init positions
    (random_free, keep_connected=False), then `config.random.shuffle` of the
    worlds; train = the first 80.  The DemonstrationTeacher draws no random
    numbers, so the demonstrations need not be computed to reach the shuffle;
    the first instance's demonstration is computed by the reference's teacher.
    Actions: hash_action(seed, 0, t), uniform over the 6 actions.  Recorded per
    step t (the state after action t; row 0 of `pre_*` is the initial state):
    pos, dir, inventory, grid (kind ids), features (uint8, exact) and
    satisfies(task) for the instance's task."""
    cfg, world = make_world()
    tm = TaskManager(cfg)
    fns = make_data_functions(world)
    teacher = teachers.load(cfg)
    ingredients = [world.cookbook.index[i] for i in ["wood", "grass", "iron"]]
    grids = []
    while len(grids) < world.N_WORLDS:
        grid, _ = fns["sample_scenario"](world, ingredients, cfg)
        if any((grid == g).all() for g in grids):
            continue
        grids.append(grid)
    items, n_inst = [], 0
    for grid in grids:
        insts = []
        for task in tm.tasks:
            if task.goal_name not in ("get", "make"):
                continue
            poss, ids = [], []
            while len(poss) < 20:
                pos = fns["random_free"](world, grid, cfg.random, keep_connected=False)
                if pos not in poss:
                    n_inst += 1
                    poss.append(pos)
                    ids.append(n_inst)
            insts.append((task, poss, ids))
        items.append((grid, insts))
    cfg.random.shuffle(items)
    train = items[:world.N_WORLDS * 80 // 100]
    grid, insts = train[0]
    task, poss, ids = insts[0]
    pos = poss[0]
    task_id = [f"{t.goal_name}[{t.goal_arg}]" for t in tm.tasks].index(f"{task.goal_name}[{task.goal_arg}]")
    # the reference demonstration of this instance (make_data.py:146-152)
    state = world.init_state(grid, pos)
    demo = [teacher(task, state)]
    while demo[-1] != world.actions.STOP.index:
        _, state = state.step(demo[-1])
        demo.append(teacher(task, state))
    assert state.satisfies(task)
    # the 100-step random rollout
    state = world.init_state(grid, pos)
    rec = {k: [] for k in ("pos", "dir", "inv", "grid", "features", "satisfies")}

    def record(st):
        rec["pos"].append(st.pos)
        rec["dir"].append(st.dir)
        rec["inv"].append(np.asarray(st.inventory))
        rec["grid"].append(onehot_to_ids(st.grid).reshape(-1))
        f = st.features()
        assert (f.astype(np.uint8) == f).all()
        rec["features"].append(f.astype(np.uint8))
        rec["satisfies"].append(int(bool(st.satisfies(task))))

    record(state)
    actions = [hash_action(seed, 0, t) for t in range(T)]
    for a in actions:
        r, state = state.step(a)
        assert r == 0
        record(state)
    arrays = {
        "train_grids": np.stack([onehot_to_ids(g).reshape(-1) for g, _ in train]).astype(np.uint8),
        "train0_pos": np.asarray([p for _, ps, _ in insts for p in ps], dtype=np.int8).reshape(len(insts), 20, 2),
        "train0_ids": np.asarray([i for _, _, ii in insts for i in ii], dtype=np.int32).reshape(len(insts), 20),
        "task": np.asarray([task_id], dtype=np.int32),
        "init_pos": np.asarray(pos, dtype=np.int32),
        "demo": np.asarray(demo, dtype=np.int8),
        "actions": np.asarray(actions, dtype=np.int8),
        "pos": np.asarray(rec["pos"], dtype=np.int8),
        "dir": np.asarray(rec["dir"], dtype=np.int8),
        "inv": np.stack(rec["inv"]).astype(np.uint8),
        "grid": np.stack(rec["grid"]).astype(np.uint8),
        "features": np.stack(rec["features"]),
        "satisfies": np.asarray(rec["satisfies"], dtype=np.int8),
        "seed": np.asarray([seed]),
    }
    np.savez_compressed(os.path.join(OUT, "config1_train0.npz"), **arrays)
    print("config1_train0.npz", task_id, pos, len(demo), os.path.getsize(os.path.join(OUT, "config1_train0.npz")))


if __name__ == "__main__":
    if sys.argv[1:] == ["language"]:            # only the language-teacher fixture
        gen_language(np.load(os.path.join(OUT, "scenarios_seed123.npz"))["w12_grids"])
        sys.exit(0)
    if sys.argv[1:] == ["config1"]:             # only the configs[0] train-instance fixture
        gen_config1()
        sys.exit(0)
    if sys.argv[1:] == ["imitation"]:           # only the do_rollout fixture
        gen_imitation(np.load(os.path.join(OUT, "scenarios_seed123.npz"))["w12_grids"])
        sys.exit(0)
    cfg, world, tm = gen_cookbook()
    gen_devtest(tm)
    sc = gen_scenarios()
    gen_kat_edges()
    gen_kat_step()
    gen_teacher(sc["w12_grids"])
    gen_rollout(sc["w12_grids"], 3, T=100, E=64, P=16, all_obs_ticks=None)
    gen_rollout(sc["w12_grids"], 5, T=60, E=48, P=16, all_obs_ticks=None)
    gen_imitation(sc["w12_grids"])
    gen_language(sc["w12_grids"])
    gen_config1()
