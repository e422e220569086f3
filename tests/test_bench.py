"""CPU tests of bench.py's host logic: the launch planner (any --steps/--warmup
works with any --ticks-per-launch) and the --gpus / WORLD_SIZE check, which
runs before any GPU call."""
import types

import pytest

import bench


@pytest.mark.parametrize("steps,k,expect", [
    (20, 32, [20]),
    (5, 32, [5]),
    (1024, 32, [32] * 32),
    (64, 32, [32, 32]),
    (7, 32, [7]),
    (0, 32, []),
    (70, 32, [32, 32, 6]),
    (3, 1, [1, 1, 1]),
])
def test_plan_launches(steps, k, expect):
    plan = bench.plan_launches(steps, k)
    assert plan == expect
    assert sum(plan) == steps
    assert all(1 <= x <= k for x in plan)


def test_plan_rejects_bad_arguments():
    with pytest.raises(ValueError):
        bench.plan_launches(-1, 32)
    with pytest.raises(ValueError):
        bench.plan_launches(10, 0)


def test_driver_command_line_parses():
    a = bench.parse(["--gpus", "1", "--steps", "20", "--warmup", "5"])
    assert (a.gpus, a.steps, a.warmup, a.ticks_per_launch) == (1, 20, 5, 32)
    assert bench.plan_launches(a.steps, a.ticks_per_launch) == [20]
    assert bench.plan_launches(a.warmup, a.ticks_per_launch) == [5]


@pytest.mark.parametrize("argv", [["--steps", "0"], ["--gpus", "0"], ["--warmup", "-1"],
                                  ["--ticks-per-launch", "0"], ["--tile", "48"]])
def test_parse_rejects_before_gpu_work(argv):
    with pytest.raises(SystemExit):
        bench.parse(argv)


def test_world_check():
    a = types.SimpleNamespace(gpus=1)
    assert bench.world_check(a, {}) == "run"
    assert bench.world_check(a, {"WORLD_SIZE": "1"}) == "run"
    a8 = types.SimpleNamespace(gpus=8)
    assert bench.world_check(a8, {}) == "spawn"
    assert bench.world_check(a8, {"WORLD_SIZE": "8"}) == "run"
    msg = bench.world_check(a8, {"WORLD_SIZE": "2"})
    assert msg not in ("run", "spawn") and "WORLD_SIZE=2" in msg


def test_mismatched_world_size_exits_nonzero(monkeypatch, capsys):
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "2", "--steps", "20"]) == 2
    assert "WORLD_SIZE=1" in capsys.readouterr().err


def test_spawn_refuses_more_gpus_than_visible(monkeypatch, capsys):
    """--gpus 2 on a box with fewer GPUs fails loudly instead of printing n_gpus 1."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.main(["--gpus", "2", "--steps", "20"]) == 2
    assert "only 1 GPU" in capsys.readouterr().err


def test_bytes_per_env_step():
    # 1754 B (w=3), 4505 B (w=5); the teacher adds 144 + 2 + 4 B
    assert bench.bytes_per_env_step(12, 12, 3, 404) == 1754
    assert bench.bytes_per_env_step(12, 12, 5, 1076) == 4505
    assert bench.bytes_per_env_step(12, 12, 3, 404, teacher=True) == 1754 + 150
    # bf16 / u8 observations (same values): the observation row shrinks to 2F / F bytes
    assert bench.bytes_per_env_step(12, 12, 3, 404, obs_bytes=2) == 1754 - 2 * 404
    assert bench.bytes_per_env_step(12, 12, 3, 404, obs_bytes=1) == 1754 - 3 * 404


def test_obs_format_argument():
    assert bench.parse([]).obs_format == "f32"
    assert bench.parse(["--obs-format", "u8"]).obs_format == "u8"
    with pytest.raises(SystemExit):
        bench.parse(["--obs-format", "f16"])


def test_pmc_traffic_lookup(tmp_path):
    """roofline.traffic comes from the PMC entry of the same workload and ticks per launch."""
    import json
    f = tmp_path / "t.json"
    f.write_text(json.dumps([
        {"workload": "w", "ticks_per_launch": 20, "hbm_bytes_per_launch": 1.0},
        {"workload": "w", "ticks_per_launch": 32, "hbm_bytes_per_launch": 2.0},
        {"workload": "x", "ticks_per_launch": 1, "hbm_bytes_per_launch": 3.0}]))
    a = types.SimpleNamespace(traffic=str(f))
    assert bench.pmc_traffic(a, "w", 20) == 1.0
    assert bench.pmc_traffic(a, "w", 32) == 2.0
    assert bench.pmc_traffic(a, "x", 1) == 3.0
    assert bench.pmc_traffic(a, "w", 1) is None
    assert bench.pmc_traffic(types.SimpleNamespace(traffic=str(tmp_path / "none.json")), "w", 20) is None


def test_pmc_summary_corrections(tmp_path, monkeypatch):
    """tools/pmc_summary.py: FETCH_SIZE doubled (gfx950 counts half of wide reads), KiB ->
    bytes, the dominant kernel by total duration, the first (warmup) launch left out of the
    per-launch trace mean."""
    import csv
    import json
    import sys
    sys.path.insert(0, str(bench.REPO) + "/tools")
    import pmc_summary
    src = tmp_path / "src"
    (src / "trace").mkdir(parents=True)
    line = {"config": {"workload": "w"}, "roofline": {"ticks_per_launch": 20, "kernel_us": 10.0,
                                                       "bytes_per_launch": 1000}}
    (src / "bench.json").write_text(json.dumps(line) + "\n")
    with open(src / "trace" / "run_kernel_stats.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Name", "Calls", "TotalDurationNs", "AverageNs"])
        w.writeheader()
        w.writerow({"Name": "k", "Calls": 3, "TotalDurationNs": 90, "AverageNs": 30})
        w.writerow({"Name": "small", "Calls": 1, "TotalDurationNs": 5, "AverageNs": 5})
    with open(src / "trace" / "run_kernel_trace.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for s, e in ((0, 10000), (20000, 60000), (70000, 110000)):
            w.writerow({"Kernel_Name": "k", "Start_Timestamp": s, "End_Timestamp": e})
    for c, v in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 8.0)):
        (src / f"pmc_{c}").mkdir()
        with open(src / f"pmc_{c}" / "run_counter_collection.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, ["Kernel_Name", "Counter_Value"])
            w.writeheader()
            w.writerow({"Kernel_Name": "k", "Counter_Value": v})
            w.writerow({"Kernel_Name": "small", "Counter_Value": 100.0})
    top = tmp_path / "profiles" / "pmc_traffic.json"
    top.parent.mkdir()
    top.write_text("[]")
    monkeypatch.setattr(pmc_summary.os.path, "abspath", lambda p: str(tmp_path / "tools" / "x.py"))
    pmc_summary.main(str(src), str(tmp_path / "dst"))
    e = json.loads((tmp_path / "dst" / "pmc_traffic.json").read_text())[0]
    assert e["kernel"] == "k" and e["ticks_per_launch"] == 20
    assert e["hbm_read_bytes_per_launch"] == 2 * 2.0 * 1024
    assert e["hbm_write_bytes_per_launch"] == 8.0 * 1024
    assert e["rocprof_avg_us_after_first"] == 40.0
    assert json.loads(top.read_text())[0]["workload"] == "w"


def test_trainer_cpu_leg_counts_live_env_steps():
    """cpu_baseline_trainer counts live env-steps (num_interactions: one per env not yet done,
    per tick, imitation.py:54) and env-slot ticks (envs x ticks), checked against
    oracle/rollout_oracle.do_rollout run on the same rollouts (round 3 counted envs x envs)."""
    import numpy as np
    import oracle
    from oracle import rollout_oracle
    from psketch_amd.sim import sample_scenarios, synthetic_specs
    from tests.helpers import make_tables
    params, cb, tm, cfg = make_tables("craft_medium_12x12")
    grids, _, _ = sample_scenarios(params, cb, 123, 16)
    n, rollouts = 12, 3
    specs = synthetic_specs(grids, 12, 12, n * rollouts, 0, seed=1,
                            task_ids=[t.id for t in tm.dataset_tasks()])
    rng = np.random.RandomState(2)
    W = rng.randint(-3, 4, size=(4, cfg.n_features, 6))
    bias = np.asarray([0, 1, 2, 3, 4, -8])
    bc = rng.binomial(1, 0.5, size=n * rollouts)
    leg = bench.cpu_baseline_trainer(cfg, grids, specs, W, bias, bc, seconds=600, n=n,
                                     max_rollouts=rollouts)
    oracle.build()
    o = oracle.Oracle(cfg, grids)
    spec = np.stack(specs, axis=1)
    pol = rollout_oracle.fake_policy(W, bias)
    live = ticks = 0
    for r in range(rollouts):
        info = rollout_oracle.do_rollout(o, spec[r * n:(r + 1) * n], pol, False,
                                         bc_mask=bc[r * n:(r + 1) * n])
        live += info["num_interactions"]
        ticks += len(info["received"])
        # a live env-step is an env acting before its episode ended: its action record
        assert info["num_interactions"] == sum(len(a) for a in info["action_seqs"])
    assert leg["rollouts"] == rollouts
    assert leg["live_env_steps"] == live and leg["ticks"] == ticks
    assert leg["slot_env_ticks"] == n * ticks
    assert 0 < live <= n * ticks
    assert leg["value"] == pytest.approx(leg["slot_env_steps_per_s"] * live / (n * ticks))
