"""TEST INFRASTRUCTURE ONLY — restatement of the reference's dataset generator
make_data.py:27-238 on numpy's own RandomState (so the random stream is the
reference's by construction), with reference actions from the C oracle teacher.

Pinned by tests/test_host.py: with seed 123 on craft_medium it regenerates the
reference's committed data/craft_medium_{dev,test}.json (as compacted in
tests/golden/devtest.npz) instance for instance.
"""
import numpy as np

DX = (0, 0, -1, 1)   # DOWN, UP, LEFT, RIGHT (craft.py:77-91)
DY = (-1, 1, 0, 0)


def all_free_cells_reachable(nav, start=None):
    """make_data.py:27-72 over a W x H occupancy array."""
    W, H = nav.shape
    if start is None:
        free = np.argwhere(nav == 0)
        start = (int(free[0][0]), int(free[0][1]))
    seen = {start}
    queue = [start]
    head = 0
    while head < len(queue):
        x, y = queue[head]
        head += 1
        for a in range(4):
            nx, ny = x + DX[a], y + DY[a]
            if nav[nx, ny]:
                nx, ny = x, y
            if (nx, ny) not in seen:
                seen.add((nx, ny))
                queue.append((nx, ny))
    for x, y in np.argwhere(nav == 0):
        if (int(x), int(y)) not in seen:
            return False
    return True


def random_free(grid, rs, keep_connected=True):
    """make_data.py:74-103; grid: W x H kind ids."""
    W, H = grid.shape
    nav = (grid != 0).astype(np.int64)
    while True:
        x, y = rs.randint(W), rs.randint(H)
        if nav[x, y]:
            continue
        good = True
        if keep_connected:
            nav[x, y] = 1
            if not all_free_cells_reachable(nav):
                good = False
            else:
                for i in range(W):
                    for j in range(H):
                        if nav[i, j] == 1 and 0 < i < W - 1 and 0 < j < H - 1 and \
                                not all_free_cells_reachable(nav, (i, j)):
                            good = False
                            break
                    if not good:
                        break
        if good:
            return (x, y)
        nav[x, y] = 0


def sample_scenario(W, H, boundary, primitives, n_per_primitive, workshops, rs):
    """make_data.py:105-144 (make_island / make_cave off, as the script calls it)."""
    grid = np.zeros((W, H), dtype=np.int64)
    grid[0, :] = grid[W - 1, :] = grid[:, 0] = grid[:, H - 1] = boundary
    for p in primitives:
        for _ in range(n_per_primitive):
            x, y = random_free(grid, rs)
            grid[x, y] = p
    for w in workshops:
        x, y = random_free(grid, rs)
        grid[x, y] = w
    init_pos = random_free(grid, rs)
    return grid, init_pos


def sample_worlds(params, cookbook, primitives, seed, count, rs=None):
    """make_data.py:164-178: `count` distinct worlds."""
    rs = np.random.RandomState(seed) if rs is None else rs
    W, H = params["WIDTH"], params["HEIGHT"]
    workshops = [cookbook.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])]
    worlds, inits = [], []
    while len(worlds) < count:
        grid, init = sample_scenario(W, H, cookbook.index["boundary"], primitives,
                                     params["N_PRIMITIVES"], workshops, rs)
        if any((grid == g).all() for g in worlds):
            continue
        worlds.append(grid)
        inits.append(init)
    return worlds, inits, rs


def reference_actions(oracle, grid, pos, task_id):
    """get_reference_actions, make_data.py:146-152, on the C oracle."""
    env = oracle.env(grid, pos[0], pos[1], 0)
    actions = []
    for _ in range(1000):
        rc, a = oracle.teacher(env, task_id)
        assert rc == 0, rc
        actions.append(a)
        if a == 5:
            break
        oracle.step(env, a)
    assert oracle.satisfies(env, task_id) == 1
    return actions


def make_dataset(params, cookbook, task_manager, oracle, primitives, seed=123, n_pos=20):
    """make_data.py:154-230: worlds, 20 init positions per (world, get/make task)
    with their teacher demonstrations, shuffled and split 80/10/10."""
    worlds, _, rs = sample_worlds(params, cookbook, primitives, seed, params["N_WORLDS"])
    data_by_env = []
    i_instance = 0
    for grid in worlds:
        item = {"grid": grid, "task_instances": []}
        for task in task_manager.tasks:
            if task.goal_name not in ("get", "make"):
                continue
            ti = {"task": task.id, "init_pos": [], "ids": [], "ref_actions": []}
            while len(ti["init_pos"]) < n_pos:
                pos = random_free(grid, rs, keep_connected=False)
                if pos not in ti["init_pos"]:
                    i_instance += 1
                    ti["ids"].append(i_instance)
                    ti["init_pos"].append(pos)
                    ti["ref_actions"].append(reference_actions(oracle, grid, pos, task.id))
            item["task_instances"].append(ti)
        data_by_env.append(item)
    rs.shuffle(data_by_env)
    n_train = params["N_WORLDS"] * 80 // 100
    n_dev = params["N_WORLDS"] * 10 // 100
    return {"train": data_by_env[:n_train], "dev": data_by_env[n_train:n_train + n_dev],
            "test": data_by_env[n_train + n_dev:]}
