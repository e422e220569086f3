"""Diagnostic: where the teacher-labelled rollout kernel's time goes, per wave (CRAFT_STAMPS
build of craft_rollout_teach, never the product).

Per launch: the workgroups' span; per interval (one tick of one tile) the mean shader-clock time
each wave spends working and waiting at the barrier; the teacher wave's walk, decode, job push,
BFS steps and idle time.

  python tools/rt_stamps.py --build            # here (CPU): psketch_amd/lib/libpsketch_craft_rtst.so
  python tools/rt_stamps.py [--label] [K ...]   # on the GPU box (config 5: 65,536 envs)

--label: every env acts on its label (demonstrations: label_actions, label_in the last tick's row)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "psketch_amd", "lib", "libpsketch_craft_rtst.so")
if "--lib" in sys.argv:                  # another stamped build (tools/diag_build.py --out NAME)
    i = sys.argv.index("--lib")
    LIB = os.path.join(REPO, "psketch_amd", "lib", sys.argv[i + 1])
    del sys.argv[i:i + 2]

if "--build" in sys.argv:
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import diag_build
    extra = [a for a in sys.argv[1:] if a.startswith("-D")]
    diag_build.build(("craft_sim", "craft_rollout_teach"), list(extra), LIB, True)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from psketch_amd import _native  # noqa: E402
_native.LIB_PATH = LIB
from psketch_amd import CraftSim, sample_scenarios, synthetic_specs  # noqa: E402

lib = _native.lib()
lib.craft_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
n, R = 65536, 16
sim = CraftSim("craft_medium_12x12", n_envs=n, device=0, pool_capacity=1024)
g, _, _ = sample_scenarios(sim.params, sim.cookbook, 123, 1024)
sim.load_pool(g)
sim.reset(*synthetic_specs(g, 12, 12, n, task_ids=[t.id for t in sim.task_manager.dataset_tasks()]))
st = torch.zeros((n // 32, 64), dtype=torch.int64, device="cuda")
lib.craft_debug_set_stamps(sim._h, ctypes.c_void_p(st.data_ptr()))
F = sim.n_features
out = dict(obs=torch.empty((R, n, F), dtype=torch.float32, device="cuda"),
           done=torch.empty((R, n), dtype=torch.uint8, device="cuda"),
           success=torch.empty((R, n), dtype=torch.int8, device="cuda"),
           reward=torch.empty((R, n), dtype=torch.float32, device="cuda"),
           labels=torch.empty((R, n), dtype=torch.int32, device="cuda"),
           action_record=torch.empty((R, n), dtype=torch.int32, device="cuda"))
names = ["C", "D", "E2", "E3", "E4", "E5", "E6", "T"]
tick = 0
label = "--label" in sys.argv
label_in = sim.teacher()[0].clone() if label else None
for K in [int(x) for x in sys.argv[1:] if not x.startswith("-")] or [20]:
    for rep in range(3):
        st.zero_()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        kw = dict(label_in=label_in, label_actions=True) if label else {}
        sim.rollout_teach(K, tick0=tick, **kw, **out)
        ev1.record()
        if label:
            label_in = out["labels"][(tick + K - 1) % R].clone()
        tick += K
        torch.cuda.synchronize()
    s = st.cpu().numpy().astype(np.float64).reshape(-1, 8, 8)
    s = s[s[:, 0, 7] > 0]
    wgs = len(s)
    tiles = n // 32 / wgs
    intervals = tiles * (K + 2)
    clk_per_us = s[:, 0, 7].mean() / (s[:, 0, 6].mean() / 100.0)
    per = s.mean(0) / clk_per_us / intervals                      # us per interval
    print(f"K={K}: launch {ev0.elapsed_time(ev1) * 1e3:.1f} us, {wgs} workgroups x {tiles:.2f} tiles, "
          f"WG span mean {s[:, 0, 6].mean() / 100:.1f} us max {s[:, 0, 6].max() / 100:.1f} us, "
          f"clock {clk_per_us:.0f} MHz; per interval ({intervals:.0f} per WG) us:")
    for w, nm in enumerate(names):
        if nm == "T":
            print(f"  T   barrier {per[w, 0]:.3f} walk {per[w, 2]:.3f} (decode {per[w, 3]:.3f} fetch issue {per[w, 1]:.3f}) jobs {per[w, 4]:.3f} "
                  f"bfs {per[w, 5]:.3f} ({s[:, w, 7].mean() / intervals:.1f} steps) idle {per[w, 6]:.3f}")
        elif nm == "C":
            print(f"  C   barrier {per[w, 0]:.3f} work {per[w, 2]:.3f} (sync {per[w, 4]:.3f} action {per[w, 5]:.3f} "
                  f"transition {per[w, 3]:.3f} label lookup + stores {per[w, 1]:.3f})")
        else:
            print(f"  {nm:3s} barrier {per[w, 0]:.3f} work {per[w, 2]:.3f}" +
                  (f" teacher-wait {per[w, 1]:.3f}" if w >= 2 else ""))
    sys.stdout.flush()
sim.check()
