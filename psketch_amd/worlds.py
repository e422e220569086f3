"""Drop-in CraftWorld for psketch's world registry (worlds/__init__.py:5-11).

`CraftWorld(config)` and its `CraftState`s expose exactly the surface the
reference's trainers, students and teachers use:

  CraftWorld.__init__(config)    craft.py:59-109  (writes config.student.model.input_size / n_actions)
  .actions / .action_space       craft.py:77-99
  .n_features / .n_actions / .cookbook / .WIDTH / .HEIGHT / .WINDOW_* / ...
  .init_state(grid, pos, dir=0)  craft.py:258-259
  .make_scenario(grid, pos, dir) craft.py:255-256 (CraftScenario.init, craft.py:268-273)
  CraftState.step(a) -> (0, s')  craft.py:332-424   (old states stay valid)
  CraftState.features()          craft.py:296-330   (memoised, float64 like the reference)
  CraftState.satisfies(task)     craft.py:285-294
  CraftState.pos / .dir / .inventory / .grid, make_navigation_grid(),
  find_resource_positions(arg), neighbors(), render()

Each state is a slot of a CraftSim on the GPU; every transition, observation and
goal test runs in the HIP kernels (one launch per call — this surface exists so
the reference's per-env Python loops run unchanged; large batches use
CraftSim directly).  States are immutable: step() writes the successor into a
fresh slot (craft_transition with src != dst) and a slot is recycled when its
CraftState is garbage-collected.
"""
import os

import numpy as np
import torch
import yaml

from . import gamedef
from .cookbook import Cookbook
from .sim import CraftSim

DOWN, UP, LEFT, RIGHT, USE, STOP = range(6)
N_ACTIONS = 6


class _Struct:
    """misc.util.Struct (misc/util.py:10-43) for the actions table."""

    def __init__(self, **entries):
        for k, v in entries.items():
            setattr(self, k, _Struct(**v) if isinstance(v, dict) else v)


def _world_yaml(config):
    name = config.world.config
    path = os.path.join("configs/worlds", name + ".yaml")      # craft.py:62-63, relative to CWD
    if os.path.exists(path):
        with open(path) as f:
            return yaml.safe_load(f)
    if name in gamedef.WORLDS:
        return dict(gamedef.WORLDS[name])
    raise FileNotFoundError(path)


def _hints_source(config):
    trainer = getattr(config, "trainer", None)
    path = getattr(trainer, "hints", None) if trainer is not None else None
    return path if path and os.path.exists(path) else None


class CraftWorld:
    """psketch CraftWorld on the MI355X.  `capacity` bounds the number of
    simultaneously alive CraftStates (slots on the GPU)."""

    def __init__(self, config, capacity=65536, device=None, pool_capacity=4096):
        recipes = getattr(config, "recipes", None)
        recipes = recipes if recipes and os.path.exists(recipes) else None
        self.cookbook = Cookbook(recipes)
        for k, v in _world_yaml(config).items():                 # craft.py:64-67
            setattr(self, k, v)
        self.params = {k: getattr(self, k) for k in
                       ("WIDTH", "HEIGHT", "WINDOW_WIDTH", "WINDOW_HEIGHT", "N_WORKSHOPS")}
        self.params.setdefault("N_PRIMITIVES", getattr(self, "N_PRIMITIVES", 2))
        self.n_features = (2 * self.WINDOW_WIDTH * self.WINDOW_HEIGHT * self.cookbook.n_kinds +
                           self.cookbook.n_kinds + 4 + 1)
        self.n_actions = N_ACTIONS
        student = getattr(config, "student", None)
        if student is not None and getattr(student, "model", None) is not None:
            config.student.model.input_size = self.n_features     # craft.py:69-76 side effects
            config.student.model.n_actions = N_ACTIONS
        self.actions = _Struct(**{
            "DOWN": {"index": DOWN, "coord_change": (0, -1)},
            "UP": {"index": UP, "coord_change": (0, 1)},
            "LEFT": {"index": LEFT, "coord_change": (-1, 0)},
            "RIGHT": {"index": RIGHT, "coord_change": (1, 0)},
            "USE": {"index": USE, "coord_change": (0, 0)},
            "STOP": {"index": STOP, "coord_change": (0, 0)},
        })
        self.action_space = [self.actions.DOWN, self.actions.UP, self.actions.LEFT,
                             self.actions.RIGHT, self.actions.USE, self.actions.STOP]
        self.non_grabbable_indices = self.cookbook.environment
        self.grabbable_indices = [i for i in range(self.cookbook.n_kinds)
                                  if i not in self.non_grabbable_indices]
        self.workshop_indices = [self.cookbook.index["workshop%d" % i]
                                 for i in range(self.N_WORKSHOPS)]
        self.water_index = self.cookbook.index["water"]
        self.stone_index = self.cookbook.index["stone"]
        self.random = getattr(config, "random", None)

        max_t = getattr(getattr(config, "trainer", None), "max_timesteps", gamedef.MAX_TIMESTEPS)
        # the episode timer (trainers/imitation.py:29, timer = max_timesteps) is a u8 field of the
        # packed state word (include/craft.h): refuse what it cannot hold instead of clamping
        if int(max_t) != max_t or not 1 <= int(max_t) <= 255:
            raise ValueError(f"CraftWorld: trainer.max_timesteps = {max_t!r}; the GPU episode timer "
                             "holds 1 .. 255 ticks")
        self.sim = CraftSim(dict(self.params), n_envs=capacity, device=device,
                            pool_capacity=pool_capacity, recipes=recipes,
                            hints=_hints_source(config), max_timesteps=int(max_t))
        self.task_manager = self.sim.task_manager
        self._free = list(range(capacity - 1, -1, -1))
        self._pool = {}                  # grid bytes -> pool entry
        self._dev = self.sim.device

    # ---- slots ----------------------------------------------------------------------
    def _alloc(self):
        if not self._free:
            # a slot comes back only when its CraftState is garbage-collected (CraftState.__del__)
            raise RuntimeError(
                f"CraftWorld: all {self.sim.n_envs} state slots are alive ({self.sim.n_envs} "
                "CraftStates are still referenced; every step() keeps its predecessor alive "
                "until the caller drops it). Drop old states or build the world with a larger "
                f"capacity= (now {self.sim.n_envs})")
        return self._free.pop()

    def _release(self, slot):
        self._free.append(slot)

    def _pool_entry(self, ids):
        key = ids.tobytes()
        p = self._pool.get(key)
        if p is None:
            p = len(self._pool)
            if p >= self.sim.pool_capacity:
                raise RuntimeError("CraftWorld: scenario pool full")
            self.sim.load_pool(ids.reshape(1, -1), first=p)
            self._pool[key] = p
        return p

    def _task_id(self, task):
        goal = f"{task.goal_name}[{task.goal_arg}]"
        t = self.task_manager.tasks_by_goal.get(goal)
        if t is None:
            raise KeyError(f"task {goal} is not in the hint table the world was built with")
        return t.id

    # ---- reference surface ---------------------------------------------------------------
    def grid_to_ids(self, grid):
        g = np.asarray(grid)
        if g.ndim == 3:
            if (g.sum(axis=2) > 1).any():                         # craft.py:365-371
                raise AssertionError("impossible world configuration: a cell holds several kinds")
            ids = np.where(g.max(axis=2) > 0, g.argmax(axis=2), 0)
        else:
            ids = g
        return np.ascontiguousarray(ids, dtype=np.uint8).reshape(self.WIDTH, self.HEIGHT)

    def init_state(self, grid, pos, dir=0):
        ids = self.grid_to_ids(grid)
        p = self._pool_entry(ids)
        slot = self._alloc()
        x, y = int(pos[0]), int(pos[1])
        spec = torch.tensor([[p, x, y, dir, 0]], dtype=torch.int32, device=self._dev)
        agent = torch.tensor([[x, y, dir, self.sim.config.max_timesteps]], dtype=torch.int32,
                             device=self._dev)
        self.sim.set_state(spec, agent, None, slots=torch.tensor([slot], dtype=torch.int32,
                                                                 device=self._dev))
        self.sim.check()
        return CraftState(self, slot, grid_ids=ids)

    def make_scenario(self, grid, pos, dir=0):
        return CraftScenario(grid, pos, self, init_dir=dir)

    def render(self, state):
        rows = []
        for y in reversed(range(self.HEIGHT)):
            row = ""
            for x in range(self.WIDTH):
                if (x, y) == tuple(state.pos):
                    row += "<^>v"[[LEFT, UP, RIGHT, DOWN].index(state.dir)] + " "
                else:
                    k = int(state.grid_ids[x, y])
                    row += (self.cookbook.index.get(k)[:2] if k else ". ").ljust(2)
            rows.append(row)
        print("\n".join(rows))
        return rows


class CraftScenario:
    """craft.py:262-273."""

    def __init__(self, grid, init_pos, world, init_dir=0):
        self.init_grid = grid
        self.init_pos = init_pos
        self.init_dir = init_dir
        self.world = world

    def init(self):
        return self.world.init_state(self.init_grid, self.init_pos, self.init_dir)


class CraftState:
    """One immutable CraftWorld state living in a GPU slot."""

    def __init__(self, world, slot, grid_ids=None):
        self.world = world
        self.scenario = None
        self._slot = slot
        self._grid_ids = grid_ids
        self._agent = None
        self._inv = None
        self._features = None

    def __del__(self):
        try:
            self.world._release(self._slot)
        except Exception:
            pass

    def _fetch(self):
        if self._agent is None:
            st = self.world.sim.get_state(slots=torch.tensor([self._slot], dtype=torch.int32,
                                                             device=self.world._dev))
            self._agent = st["agent"][0].cpu().numpy()
            self._inv = st["inventory"][0].cpu().numpy().astype(np.float64)
            self._grid_ids = st["grid"][0].cpu().numpy().reshape(self.world.WIDTH, self.world.HEIGHT)

    @property
    def pos(self):
        self._fetch()
        return (int(self._agent[0]), int(self._agent[1]))

    @property
    def dir(self):
        self._fetch()
        return int(self._agent[2])

    @property
    def inventory(self):
        self._fetch()
        return self._inv

    @property
    def grid_ids(self):
        self._fetch()
        return self._grid_ids

    @property
    def grid(self):
        """W x H x K one-hot float64, as the reference stores it."""
        ids = self.grid_ids
        K = self.world.cookbook.n_kinds
        g = np.zeros(ids.shape + (K,))
        for k in range(1, K):
            g[..., k] = ids == k
        return g

    def step(self, action):
        """craft.py:332-424; returns (reward 0, successor)."""
        if action not in range(N_ACTIONS):
            raise Exception("Unexpected action: %s" % action)       # craft.py:415-416
        w = self.world
        new = w._alloc()
        dev = w._dev
        w.sim.transition(torch.tensor([int(action)], dtype=torch.int32, device=dev),
                         src=torch.tensor([self._slot], dtype=torch.int32, device=dev),
                         dst=torch.tensor([new], dtype=torch.int32, device=dev))
        return 0, CraftState(w, new)

    def features(self):
        if self._features is None:
            w = self.world
            obs = w.sim.empty_obs(1)
            w.sim.observe(slots=torch.tensor([self._slot], dtype=torch.int32, device=w._dev),
                          obs=obs)
            self._features = obs[0].double().cpu().numpy()
        return self._features

    def satisfies(self, task):
        w = self.world
        tid = w._task_id(task)
        sat = torch.empty(1, dtype=torch.int8, device=w._dev)
        w.sim.observe(slots=torch.tensor([self._slot], dtype=torch.int32, device=w._dev),
                      tasks=torch.tensor([tid], dtype=torch.int32, device=w._dev), sat=sat)
        s = int(sat.item())
        return None if s < 0 else bool(s)

    def neighbors(self, pos, dir=None):
        """craft.py:426-437."""
        x, y = pos
        out = []
        if x > 0 and (dir is None or dir == LEFT):
            out.append((x - 1, y))
        if y > 0 and (dir is None or dir == DOWN):
            out.append((x, y - 1))
        if x < self.world.WIDTH - 1 and (dir is None or dir == RIGHT):
            out.append((x + 1, y))
        if y < self.world.HEIGHT - 1 and (dir is None or dir == UP):
            out.append((x, y + 1))
        return out

    def make_navigation_grid(self):
        """craft.py:450-451: grid.max(axis=2)."""
        return (self.grid_ids > 0).astype(np.float64)

    def find_resource_positions(self, goal_arg):
        """craft.py:453-455, np.nonzero (x-major) order."""
        kind = self.world.cookbook.index[goal_arg]
        return list(zip(*np.nonzero(self.grid_ids == kind)))

    def render(self):
        return self.world.render(self)


def load(config):
    """worlds.load (worlds/__init__.py:5-11) over this module's classes."""
    name = config.world.name
    cls = {"CraftWorld": CraftWorld, "CraftWorldHIP": CraftWorld}.get(name)
    if cls is None:
        raise Exception("No such world: {}".format(name))
    return cls(config)
