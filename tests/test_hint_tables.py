"""The hint walk tabulated per task (csrc/craft_host.h hint_tables, read by craft_rollout_teach's
teacher wave): for every task and every truth assignment of its satisfies() predicates, the leaf
byte equals what the reference's DemonstrationTeacher decides (teachers/demonstration.py:9-24 over
teachers/base.py:10-25's recursive find_incomplete_subtask), restated here in Python from those
lines: STOP when nothing is incomplete, USE for a use leaf, the kind of a go leaf, and the
reference's AssertionError (base.py:24, demonstration.py:18) as the error byte.  Tasks with more
predicates than the table takes keep the walk (descriptor flag); a hint tree built to exceed it
checks that."""
import copy
import ctypes

import numpy as np
import pytest

from psketch_amd import _native as N
from psketch_amd import gamedef
from psketch_amd.cookbook import Cookbook, TaskManager, compile_config, world_params

ERR, STOP_B, USE_B, WALK = 0xFF, 0xFE, 0xFD, 1 << 31


def _tables(cfg):
    L = N.lib(cpu=True)
    L.craft_debug_hint_tables.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_int32)]
    desc = np.zeros(N.MAX_TASKS * 4, dtype=np.uint32)
    leaf = np.zeros(4096, dtype=np.uint8)
    n = ctypes.c_int32()
    assert L.craft_debug_hint_tables(ctypes.byref(cfg), desc.ctypes.data, leaf.ctypes.data, len(leaf),
                                     ctypes.byref(n)) == 0
    return desc.reshape(N.MAX_TASKS, 4), leaf[:n.value]


def _reference_leaf(cfg, task, sat):
    """DemonstrationTeacher.__call__'s decision before the BFS, from the compiled task table."""
    def subs(t):
        tk = cfg.task[t]
        return [tk.subtask[q] for q in range(tk.n_subtasks)] or None

    def find(t):                                       # teachers/base.py:10-25
        if sat(t):
            return None
        s = subs(t)
        if s is None:
            return t
        for c in s[:-1]:
            r = find(c)
            if r is not None:
                return r
        r = find(s[-1])
        if r is None:
            raise AssertionError                       # base.py:24
        return r

    try:
        leaf = find(task)
    except (AssertionError, RecursionError):
        return ERR
    if leaf is None:
        return STOP_B                                  # demonstration.py:12-13
    goal = cfg.task[leaf].goal
    if goal == N.GOAL_USE:
        return USE_B
    if goal == N.GOAL_GO:
        return cfg.task[leaf].arg_kind
    return ERR                                         # demonstration.py:18


def _check(cfg):
    desc, leaf = _tables(cfg)
    walked = tabulated = 0
    for t in range(cfg.n_tasks):
        if desc[t, 2] & WALK:
            walked += 1
            continue
        tabulated += 1
        preds = []
        for j in range(8):
            b = int((desc[t, j >> 2] >> (8 * (j & 3))) & 0xFF)
            if b & 0x80:
                preds.append((bool(b & 0x40), b & 0x3F))
        off = int(desc[t, 2])

        def key(node):
            tk = cfg.task[node]
            if tk.goal in (N.GOAL_GET, N.GOAL_MAKE):
                return (False, tk.arg_kind)
            if tk.goal == N.GOAL_GO:
                return (True, tk.arg_kind)
            return None

        for bits in range(1 << len(preds)):
            truth = {p: bool((bits >> j) & 1) for j, p in enumerate(preds)}

            def sat(node):
                k = key(node)
                return False if k is None else truth[k]
            assert leaf[off + bits] == _reference_leaf(cfg, t, sat), (t, bits)
    return walked, tabulated


def _config(hints=None):
    params = world_params("craft_medium_12x12")
    return compile_config(params, Cookbook(), TaskManager(hints), gamedef.MAX_TIMESTEPS)


def test_hint_tables_match_the_reference_walk():
    walked, tabulated = _check(_config())
    assert walked == 0 and tabulated == 26            # hints.hierarchy.yaml: every task fits


def test_hint_tables_keep_the_walk_past_eight_predicates():
    hints = copy.deepcopy(gamedef.HINTS)
    hints["make[ladder]"] = ["make[bed]", "make[axe]", "make[shears]", "makeat[workshop2]"]
    walked, tabulated = _check(_config(hints))
    assert walked == 1 and tabulated == 26
