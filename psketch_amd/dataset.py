"""Dataset ingestion: the reference's split files (data/craft_medium_{split}.json)
onto the GPU.

`Dataset` mirrors data/dataset.py:10-93 — same flattening order
(flatten_data, :47-67), same `next_batch` shuffling through `config.random`
(:69-86) — and additionally compacts every instance's grid into a scenario
pool entry (kind ids, deduplicated), so a batch becomes device arrays
(scenario, x, y, dir, task) for CraftSim.reset / set_state.
"""
import json
import os

import numpy as np


def onehot_to_ids(grid):
    """W x H x K one-hot (the JSON's nested lists) -> W x H kind ids; a cell
    with several kinds is the reference's AssertionError (craft.py:365-371)."""
    g = np.asarray(grid)
    if (g.sum(axis=2) > 1).any():
        raise AssertionError("impossible world configuration: a cell holds several kinds")
    return np.where(g.max(axis=2) > 0, g.argmax(axis=2), 0).astype(np.uint8)


class Dataset:
    """data/dataset.py:10-93 over a split file (or the parsed list)."""

    def __init__(self, source, split, task_manager, random=None, batch_size=32):
        self.split = split
        self.task_manager = task_manager
        self.random = random
        self.batch_size = batch_size
        if isinstance(source, (str, os.PathLike)):
            self.file_name = str(source)
            with open(source) as f:
                data = json.load(f)
        else:
            self.file_name = None
            data = source
        self.pool = []                   # distinct scenario grids (kind ids, W x H)
        self._pool_index = {}
        self.data = self.flatten_data(data)
        self.instance_by_id = {item["id"]: item for item in self.data}
        self.item_idx = 0

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx]

    def __iter__(self):
        return iter(self.data)

    def get_instance_by_id(self, instance_id):
        return self.instance_by_id[instance_id]

    def _scenario(self, ids):
        key = ids.tobytes()
        p = self._pool_index.get(key)
        if p is None:
            p = len(self.pool)
            self.pool.append(ids)
            self._pool_index[key] = p
        return p

    def flatten_data(self, data):
        """data/dataset.py:47-67: one instance per (world, task, init_pos)."""
        new_data = []
        for item in data:
            grid = np.array(item["grid"])        # the reference's one-hot, dataset.py:62
            scen = self._scenario(onehot_to_ids(grid))
            for ti in item["task_instances"]:
                task = self.task_manager[ti["task"]]
                for pos, iid, ref in zip(ti["init_pos"], ti["ids"], ti["ref_actions"]):
                    new_data.append({"id": iid, "task": task, "grid": grid, "scenario": scen,
                                     "init_pos": tuple(pos), "ref_actions": tuple(ref)})
        return new_data

    def next_batch(self):
        """data/dataset.py:69-86 (same use of the shared RandomState)."""
        if self.item_idx == 0:
            self.data_indices = list(range(len(self)))
            self.random.shuffle(self.data_indices)
        start_idx = self.item_idx
        end_idx = self.item_idx + self.batch_size
        batch_indices = self.data_indices[start_idx:end_idx]
        self.item_idx = end_idx
        end_pass = False
        if self.item_idx >= len(self):
            self.item_idx = 0
            end_pass = True
        return [self[idx] for idx in batch_indices], end_pass

    def iterate_batches(self):
        end_pass = False
        while not end_pass:
            batch, end_pass = self.next_batch()
            yield batch

    def pool_array(self):
        """uint8 [P, W*H] for CraftSim.load_pool."""
        return np.stack([g.reshape(-1) for g in self.pool])

    @staticmethod
    def specs(batch, pool_offset=0):
        """(scenario, x, y, dir, task) int32 arrays for CraftSim.reset."""
        scen = np.asarray([it["scenario"] + pool_offset for it in batch], dtype=np.int32)
        x = np.asarray([it["init_pos"][0] for it in batch], dtype=np.int32)
        y = np.asarray([it["init_pos"][1] for it in batch], dtype=np.int32)
        task = np.asarray([it["task"].id for it in batch], dtype=np.int32)
        return scen, x, y, np.zeros(len(batch), dtype=np.int32), task
