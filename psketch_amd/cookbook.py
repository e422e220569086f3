"""Host-side static tables: kind index, cookbook, task hierarchy, and their
compilation into the C ABI's craft_config_t.

Mirrors the reference interfaces so callers read the same:
  Index        misc/util.py:46-76        (1-based ids, 0 reserved)
  Cookbook     worlds/cookbook.py:7-26   (environment / primitives / recipes)
  Task         data/task.py:9-29         (goal_name, goal_arg, subtasks)
  TaskManager  data/task.py:32-75        (hint tree, tasks in file order)
"""
import re

import yaml

from . import _native as N
from . import gamedef


class Index:
    """misc/util.py:46-76: items get ids 1, 2, ... in first-seen order."""

    def __init__(self):
        self.contents = dict()
        self.ordered_contents = []
        self.reverse_contents = dict()

    def __getitem__(self, item):
        return self.contents.get(item)

    def index(self, item):
        if item not in self.contents:
            idx = len(self.contents) + 1
            self.ordered_contents.append(item)
            self.contents[item] = idx
            self.reverse_contents[idx] = item
        return self.contents[item]

    def get(self, idx):
        if idx == 0:
            return "*invalid*"
        return self.reverse_contents[idx]

    def __len__(self):
        return len(self.contents) + 1

    def __iter__(self):
        return iter(self.ordered_contents)


def _load_yaml(source, default):
    if source is None:
        return default
    if isinstance(source, dict):
        return source
    with open(source) as f:
        return yaml.safe_load(f)


class Cookbook:
    """worlds/cookbook.py:7-26.  `recipes` is a recipes.yaml path, a parsed dict,
    or None for the built-in table (gamedef.RECIPES)."""

    def __init__(self, recipes=None):
        spec = _load_yaml(recipes, gamedef.RECIPES)
        self.index = Index()
        self.environment = set(self.index.index(e) for e in spec["environment"])
        self.primitives = set(self.index.index(p) for p in spec["primitives"])
        self.recipes = {}
        for output, inputs in spec["recipes"].items():
            d = {}
            for inp, count in inputs.items():
                if "_" in inp:           # special keys (_at, _yield)
                    d[inp] = count
                else:
                    d[self.index.index(inp)] = count
            self.recipes[self.index.index(output)] = d
        self.n_kinds = len(self.index)

    def primitives_for(self, goal):
        """worlds/cookbook.py:28-52: the primitive kinds (and counts) that make `goal`, each
        intermediate ingredient made ceil(count / _yield) times."""
        out = {}
        for ing, count in self.recipes[goal].items():
            if not isinstance(ing, int):
                continue                                     # _at, _yield
            if ing in self.primitives:
                parts, times = {ing: 1}, count
            else:
                parts = self.primitives_for(ing)
                times = -(-count // self.recipes[ing].get("_yield", 1))
            for k, v in parts.items():
                if k not in self.primitives:
                    raise AssertionError(f"kind {k} is not a primitive")
                out[k] = out.get(k, 0) + v * times
        return out


_FEXP = re.compile(r"(.*)\[(.*)\]")


class Task:
    """data/task.py:9-29."""

    def __init__(self, goal, subtasks=None):
        m = _FEXP.match(goal)
        self.goal_name, self.goal_arg = m.group(1), m.group(2)
        self.subtasks = subtasks if subtasks else None
        self.id = None

    def __repr__(self):
        return f"Task({self.goal_name}[{self.goal_arg}])"

    def __hash__(self):
        return hash(self.__repr__())

    def __eq__(self, other):
        return self.goal_name == other.goal_name and self.goal_arg == other.goal_arg

    def __str__(self):
        return self.goal_name + " " + self.goal_arg


class TaskManager:
    """data/task.py:32-75 (without the vocabulary, which only the students use).
    `hints` is a hints.*.yaml path, a parsed dict, or None for the built-in tree."""

    def __init__(self, hints=None):
        self.hints = _load_yaml(hints, gamedef.HINTS)
        self.tasks_by_goal = {}
        self.tasks = []
        for goal, subgoals in self.hints.items():
            subtasks = [self.tasks_by_goal[s] for s in subgoals]
            task = Task(goal, subtasks)
            task.id = len(self.tasks)
            self.tasks_by_goal[goal] = task
            self.tasks.append(task)

    def __getitem__(self, goal):
        return self.tasks_by_goal[goal]

    def __len__(self):
        return len(self.tasks)

    def dataset_tasks(self):
        """The get/make tasks make_data.py:184-186 generates instances for."""
        return [t for t in self.tasks if t.goal_name in ("get", "make")]


_GOALS = {"get": N.GOAL_GET, "make": N.GOAL_MAKE, "go": N.GOAL_GO, "use": N.GOAL_USE}


def world_params(world):
    """A configs/worlds entry: a name in gamedef.WORLDS, a YAML path or a dict."""
    if isinstance(world, dict):
        return dict(world)
    if world in gamedef.WORLDS:
        return dict(gamedef.WORLDS[world])
    with open(world) as f:
        return yaml.safe_load(f)


def n_features(params, cookbook):
    """craft.py:69-75."""
    ww, wh = params["WINDOW_WIDTH"], params["WINDOW_HEIGHT"]
    return 2 * ww * wh * cookbook.n_kinds + cookbook.n_kinds + 4 + 1


def kind_classes(cookbook, n_workshops):
    """What USE does to each kind id, craft.py:101-107 and 373-410 (tested in
    that order: grabbable, workshop, water, stone)."""
    water = cookbook.index["water"]
    stone = cookbook.index["stone"]
    workshops = [cookbook.index["workshop%d" % i] for i in range(n_workshops)]
    classes = []
    for k in range(cookbook.n_kinds):
        if k == 0:
            classes.append(N.KIND_INERT)
        elif k not in cookbook.environment:
            classes.append(N.KIND_GRABBABLE)
        elif k in workshops:
            classes.append(N.KIND_WORKSHOP)
        elif k == water:
            classes.append(N.KIND_WATER)
        elif k == stone:
            classes.append(N.KIND_STONE)
        else:
            classes.append(N.KIND_INERT)
    return classes


def compile_config(params, cookbook, task_manager, max_timesteps=gamedef.MAX_TIMESTEPS):
    """Packs the static tables into craft_config_t (include/craft.h)."""
    c = N.craft_config_t()
    c.abi_version = N.ABI_VERSION
    c.width, c.height = params["WIDTH"], params["HEIGHT"]
    c.window_width, c.window_height = params["WINDOW_WIDTH"], params["WINDOW_HEIGHT"]
    c.n_kinds = cookbook.n_kinds
    c.n_features = n_features(params, cookbook)
    c.max_timesteps = max_timesteps
    c.bridge_kind = cookbook.index["bridge"] or 0
    c.axe_kind = cookbook.index["axe"] or 0
    if cookbook.n_kinds > N.MAX_KINDS:
        raise ValueError(f"{cookbook.n_kinds} kinds > {N.MAX_KINDS}")
    for k, cls in enumerate(kind_classes(cookbook, params["N_WORKSHOPS"])):
        c.kind_class[k] = cls
    if len(cookbook.recipes) > N.MAX_RECIPES:
        raise ValueError("too many recipes")
    c.n_recipes = len(cookbook.recipes)
    for r, (output, inputs) in enumerate(cookbook.recipes.items()):
        rc = c.recipe[r]
        rc.output = output
        rc.workshop = cookbook.index[inputs["_at"]]
        rc.yield_ = inputs.get("_yield", 1)
        ing = [(k, v) for k, v in inputs.items() if isinstance(k, int)]
        if len(ing) > N.MAX_INGREDIENTS:
            raise ValueError("too many ingredients")
        rc.n_inputs = len(ing)
        for i, (k, v) in enumerate(ing):
            rc.input_kind[i] = k
            rc.input_count[i] = v
    if len(task_manager) > N.MAX_TASKS:
        raise ValueError("too many tasks")
    c.n_tasks = len(task_manager)
    for t, task in enumerate(task_manager.tasks):
        ct = c.task[t]
        ct.goal = _GOALS.get(task.goal_name, N.GOAL_OTHER)
        ct.arg_kind = cookbook.index[task.goal_arg] or 0
        subs = task.subtasks or []
        if len(subs) > N.MAX_SUBTASKS:
            raise ValueError("too many subtasks")
        ct.n_subtasks = len(subs)
        for i, s in enumerate(subs):
            ct.subtask[i] = s.id
    return c


def generator_primitives(cookbook):
    """Primitive kinds sample_scenario places, in cookbook.primitives (set)
    iteration order with gold and gem skipped (make_data.py:128-134)."""
    gold, gem = cookbook.index["gold"], cookbook.index["gem"]
    return [p for p in cookbook.primitives if p != gold and p != gem]
