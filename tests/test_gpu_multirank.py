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


def _bench(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5",
                          "--no-cpu-baseline", *args], cwd=REPO, env=env, capture_output=True,
                         text=True, timeout=240)
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
