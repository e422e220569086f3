"""The bench lines of one tools/bench_lines.sh run as a markdown table.

    python tools/lines_table.py gpurun_out/<tag>/lines [profiles/<round>/lines]

With a second argument the JSON lines are copied there too."""
import json
import os
import shutil
import sys

ORDER = ["driver", "steps512", "k1", "k1_ring1", "config5", "config5_k20", "config5_k1", "config5_label",
         "config5_mix", "trainer", "w5",
         "w5_k1", "config5_w5", "config5_w5_k1"]
WHAT = {
    "driver": "driver's command (`--steps 20 --warmup 5`)",
    "steps512": "`--steps 512` (32-tick launches)",
    "k1": "one tick per launch, 16-slot ring",
    "k1_ring1": "one tick per launch, one reused buffer",
    "config5": "config 5, K-tick teacher rollout, K = 32",
    "config5_k20": "config 5, K-tick teacher rollout, K = 20",
    "config5_k1": "config 5, one `craft_step_teach` per tick",
    "config5_label": "config 5, K = 20, every env acts on its label",
    "config5_mix": "config 5, K = 20, half the envs act on their label",
    "trainer": "trainer closed loop (live env-steps)",
    "w5": "w = 5 rollout, 20 ticks",
    "w5_k1": "w = 5, one tick per launch",
    "config5_w5": "config 5 at w = 5, K = 20",
    "config5_w5_k1": "config 5 at w = 5, one `craft_step_teach` per tick",
}


def main(src, dst=None):
    rows = ["| line | env-steps/s | kernel | µs per tick | frac of 8 TB/s | of the in-situ fill | CPU leg |",
            "|---|---|---|---|---|---|---|"]
    for name in ORDER:
        p = os.path.join(src, name + ".json")
        if not os.path.exists(p):
            continue
        d = json.loads(open(p).read().strip().splitlines()[-1])
        r = d["roofline"]
        k = r.get("ticks_per_launch", 1) or 1
        us = r["kernel_us"]
        per_tick = us / k
        kern = r["kernel"].split(" (")[0]
        cpu = d.get("cpu_baseline") or {}
        v = cpu.get("value", 0)
        amount = f"{v / 1e6:.1f} M" if v >= 1e6 else f"{v / 1e3:.0f} k"
        leg = f"{amount} ({cpu.get('cores', '?')} cores, {cpu.get('kind')})" if cpu else "—"
        rows.append(f"| {WHAT[name]} | {d['value'] / 1e9:.2f} G | `{kern}` {us:.1f} µs / {k} | {per_tick:.1f} | "
                    f"{r['frac']:.3f} | {r.get('frac_of_ceiling', float('nan')):.2f} | {leg} |")
        if dst:
            os.makedirs(dst, exist_ok=True)
            shutil.copy(p, os.path.join(dst, name + ".json"))
    print("\n".join(rows))


if __name__ == "__main__":
    main(*sys.argv[1:])
