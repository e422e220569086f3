"""psketch_amd — MI355X-native batched CraftWorld simulator.

A from-scratch HIP/CDNA4 implementation of psketch's CraftWorld hot path
(worlds/craft.py step/features/satisfies, the cookbook recipe semantics and the
DemonstrationTeacher BFS), struct-of-arrays in HBM, behind a C ABI
(include/craft.h) bound here with ctypes.  See DESIGN.md.
"""
from . import gamedef
from .cookbook import Cookbook, Index, Task, TaskManager, compile_config, world_params
from .sim import CraftSim, hash_actions, sample_scenarios, splitmix64, synthetic_specs
from .dataset import Dataset
from .rollout import ImitationRollout, RolloutInfo, do_rollout
from .language import PrimitiveLanguageTeacher

__all__ = ["gamedef", "Cookbook", "Index", "Task", "TaskManager", "compile_config",
           "world_params", "CraftSim", "hash_actions", "sample_scenarios", "splitmix64",
           "synthetic_specs", "Dataset", "ImitationRollout", "RolloutInfo", "do_rollout",
           "PrimitiveLanguageTeacher"]
