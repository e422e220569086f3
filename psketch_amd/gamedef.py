"""Built-in game definition: the craft recipe table, the task hierarchy and the
world configurations of the reference, as Python data.

These mirror resources/craft/recipes.yaml, resources/craft/hints.hierarchy.yaml
and configs/worlds/*.yaml of the reference so the simulator runs where the
reference tree is absent (the GPU box).  Callers that hold the reference's
YAML files pass their paths instead (cookbook.Cookbook(path),
tasks.TaskManager(path)), exactly like worlds/cookbook.py:8-10 and
data/task.py:35-37; tests/golden/cookbook.json pins that both agree.
"""

# recipes.yaml: environment, primitives, recipes (dict order matters:
# CraftState.step applies a workshop's recipes in this order, craft.py:391).
RECIPES = {
    "environment": ["boundary", "workshop0", "workshop1", "workshop2", "water", "stone"],
    "primitives": ["iron", "grass", "wood", "gold", "gem"],
    "recipes": {
        "plank": {"wood": 1, "_at": "workshop0"},
        "axe": {"stick": 1, "iron": 1, "_at": "workshop0"},
        "rope": {"grass": 1, "_at": "workshop0"},
        "stick": {"wood": 1, "_at": "workshop1"},
        "bed": {"plank": 1, "grass": 1, "_at": "workshop1"},
        "shears": {"stick": 1, "iron": 1, "_at": "workshop1"},
        "cloth": {"grass": 1, "_at": "workshop2"},
        "bridge": {"wood": 1, "iron": 1, "_at": "workshop2"},
        "ladder": {"plank": 1, "stick": 1, "_at": "workshop2"},
    },
}

# hints.hierarchy.yaml: goal -> subgoals, in file order (TaskManager order).
HINTS = {
    "left[none]": [],
    "right[none]": [],
    "up[none]": [],
    "down[none]": [],
    "use[none]": [],
    "stop[none]": [],
    "go[wood]": [],
    "go[iron]": [],
    "go[grass]": [],
    "go[workshop0]": [],
    "go[workshop1]": [],
    "go[workshop2]": [],
    "get[wood]": ["go[wood]", "use[none]"],
    "get[grass]": ["go[grass]", "use[none]"],
    "get[iron]": ["go[iron]", "use[none]"],
    "makeat[workshop0]": ["go[workshop0]", "use[none]"],
    "makeat[workshop1]": ["go[workshop1]", "use[none]"],
    "makeat[workshop2]": ["go[workshop2]", "use[none]"],
    "make[plank]": ["get[wood]", "makeat[workshop0]"],
    "make[stick]": ["get[wood]", "makeat[workshop1]"],
    "make[cloth]": ["get[grass]", "makeat[workshop2]"],
    "make[rope]": ["get[grass]", "makeat[workshop0]"],
    "make[bridge]": ["get[iron]", "get[wood]", "makeat[workshop2]"],
    "make[bed]": ["make[plank]", "get[grass]", "makeat[workshop1]"],
    "make[axe]": ["make[stick]", "get[iron]", "makeat[workshop0]"],
    "make[shears]": ["make[stick]", "get[iron]", "makeat[workshop1]"],
}

# configs/worlds/*.yaml.  "craft_medium_12x12" is the benchmark world named by
# BASELINE.json: craft_medium with WIDTH = HEIGHT = 12, other keys unchanged.
WORLDS = {
    "craft_medium": dict(WIDTH=8, HEIGHT=8, WINDOW_WIDTH=3, WINDOW_HEIGHT=3, N_WORKSHOPS=3,
                         N_PRIMITIVES=2, N_WORLDS=100),
    "craft_large": dict(WIDTH=10, HEIGHT=10, WINDOW_WIDTH=5, WINDOW_HEIGHT=5, N_WORKSHOPS=3,
                        N_PRIMITIVES=4, N_WORLDS=100),
    "craft_medium_12x12": dict(WIDTH=12, HEIGHT=12, WINDOW_WIDTH=3, WINDOW_HEIGHT=3,
                               N_WORKSHOPS=3, N_PRIMITIVES=2, N_WORLDS=100),
    "craft_medium_12x12_w5": dict(WIDTH=12, HEIGHT=12, WINDOW_WIDTH=5, WINDOW_HEIGHT=5,
                                  N_WORKSHOPS=3, N_PRIMITIVES=2, N_WORLDS=100),
    # largest geometry the kernels support (W*H = 256, window 7): coverage only
    "craft_16x16_w7": dict(WIDTH=16, HEIGHT=16, WINDOW_WIDTH=7, WINDOW_HEIGHT=7,
                           N_WORKSHOPS=3, N_PRIMITIVES=4, N_WORLDS=100),
}

# trainer.max_timesteps, configs/experiments/imitation.yaml:21
MAX_TIMESTEPS = 40
