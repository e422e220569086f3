"""Shared test helpers: compiled configs for the worlds the fixtures use."""
import numpy as np

from psketch_amd import gamedef
from psketch_amd.cookbook import Cookbook, TaskManager, compile_config, world_params


def make_tables(world="craft_medium", max_timesteps=gamedef.MAX_TIMESTEPS):
    params = world_params(world)
    cb = Cookbook()
    tm = TaskManager()
    cfg = compile_config(params, cb, tm, max_timesteps)
    return params, cb, tm, cfg


def world_for(W, window):
    name = {(8, 3): "craft_medium", (12, 3): "craft_medium_12x12",
            (12, 5): "craft_medium_12x12_w5", (10, 5): "craft_large"}[(W, window)]
    return name


def pad_inv(inv, K=32):
    inv = np.asarray(inv)
    out = np.zeros(inv.shape[:-1] + (K,), dtype=np.int32)
    out[..., :inv.shape[-1]] = inv
    return out
