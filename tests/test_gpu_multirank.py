"""bench.py's multi-rank path through the HIP kernels on one card: `--gpus 2`
spawns two ranks (torch.distributed.run), each simulates its shard of global
env ids [r * N, (r + 1) * N) and the episode summary is all-reduced (gloo
here; RCCL on a node).  The reduced summary must equal one process simulating
all 2N envs — envs are independent (worlds/craft.py) and every draw is keyed by
global id."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5",
                          "--no-cpu-baseline", *args], cwd=REPO, env=env, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_on_one_card_equal_one_process():
    two = _bench("--gpus", "2", "--one-device", "--dist-backend", "gloo", "--envs", "4096")
    one = _bench("--gpus", "1", "--envs", "8192")
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 8192
    assert two["episodes"] == one["episodes"]
    assert two["episodes"]["env_steps"] > 8192 * 25      # warmup + timed + the event-timed launches
    # the process group's own account (bench line "dist"), gathered over the group
    d2, d1 = two["dist"], one["dist"]
    assert d2["backend"] == "gloo" and d2["world_size"] == 2 and len(d2["per_rank_s"]) == 2
    assert d1["backend"] is None and d1["world_size"] == 1
    assert [r["env_id_base"] for r in d2["ranks"]] == [0, 4096]
    assert sum(r["episodes"]["env_steps"] for r in d2["ranks"]) == one["episodes"]["env_steps"]
    assert (sum(r["episodes"]["successes"] for r in d2["ranks"]) ==
            d1["ranks"][0]["episodes"]["successes"])


def test_eight_ranks_on_one_card_equal_one_process():
    """The 8-GPU node's shape rehearsed on one card: 8 ranks (gloo) of 8,192 envs each, rank r
    simulating global ids [r * 8192, (r + 1) * 8192), reduce to the same episode summary as one
    process simulating all 65,536 (the N=8 scaling line's work split)."""
    eight = _bench("--gpus", "8", "--one-device", "--dist-backend", "gloo", "--envs", "8192", timeout=420)
    one = _bench("--gpus", "1", "--envs", "65536")
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == 65536
    assert eight["episodes"] == one["episodes"]
    d8 = eight["dist"]
    assert d8["backend"] == "gloo" and d8["world_size"] == 8 and len(d8["per_rank_s"]) == 8
    assert [r["env_id_base"] for r in d8["ranks"]] == [8192 * r for r in range(8)]
    assert all(r["envs"] == 8192 for r in d8["ranks"])
    assert sum(r["episodes"]["env_steps"] for r in d8["ranks"]) == one["episodes"]["env_steps"]


_RCCL_ONE_RANK = r"""
import torch, torch.distributed as dist
from psketch_amd import distributed as D
dev = torch.device("cuda:0")
D.init(device=dev, force=True)
assert dist.get_backend() == "nccl", dist.get_backend()
stats = torch.tensor([3, 7, 1 << 40], dtype=torch.int64, device=dev)
D._reduce(stats, dist.ReduceOp.SUM)
torch.cuda.synchronize()
assert stats.tolist() == [3, 7, 1 << 40], stats.tolist()
t = torch.tensor([2.5], dtype=torch.float64, device=dev)
D._reduce(t, dist.ReduceOp.MAX)
assert t.item() == 2.5
D.barrier()
dist.barrier()
dist.destroy_process_group()
print("rccl-ok")
"""


def test_rccl_process_group_on_the_card():
    """The nccl (= RCCL) branch of distributed.init with device_id, and the int64[3] summary
    and float64 max all-reduces bench.py issues, executed over RCCL on the GPU (one rank: a
    one-GPU box cannot hold two RCCL ranks on one device)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK], cwd=REPO, env=env, capture_output=True,
                         text=True, timeout=180)
    assert out.returncode == 0 and "rccl-ok" in out.stdout, (out.stdout[-1000:], out.stderr[-2000:])
