"""Host-side preconditions of the drop-in CraftWorld (psketch_amd.worlds) that must fail
loudly before any GPU work: the episode timer's range (trainers/imitation.py:29,
timer = max_timesteps, a u8 field of the packed state word) and the slot-exhaustion
message.  No GPU: the checks run before the simulator is created."""
from types import SimpleNamespace as NS

import numpy as np
import pytest

from psketch_amd import worlds


def make_config(max_timesteps):
    return NS(recipes="resources/craft/recipes.yaml", world=NS(name="CraftWorld", config="craft_medium"),
              student=NS(model=NS()), teacher=NS(name="DemonstrationTeacher"),
              trainer=NS(hints="resources/craft/hints.hierarchy.yaml", max_timesteps=max_timesteps),
              random=np.random.RandomState(0))


@pytest.mark.parametrize("max_t", [256, 1000, 0, -3, 40.5])
def test_max_timesteps_out_of_range_raises(max_t):
    """The shim used to clamp to 255 silently; now it refuses (before touching the GPU)."""
    with pytest.raises(ValueError, match="max_timesteps"):
        worlds.CraftWorld(make_config(max_t))


def test_slot_exhaustion_names_live_states_and_capacity():
    w = worlds.CraftWorld.__new__(worlds.CraftWorld)        # no simulator: only the slot list
    w.sim = NS(n_envs=4)
    w._free = [3, 2, 1, 0]
    slots = [w._alloc() for _ in range(4)]
    assert sorted(slots) == [0, 1, 2, 3]
    with pytest.raises(RuntimeError) as e:
        w._alloc()
    msg = str(e.value)
    assert "all 4 state slots are alive" in msg and "capacity=" in msg
    w._release(slots[0])
    assert w._alloc() == slots[0]
