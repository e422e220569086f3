"""Summarise one tools/profile.sh config into profiles/<round>/<name>/: the bench line, the
kernel-trace stats CSV, and the dominant kernel's per-launch HBM traffic from the FETCH_SIZE /
WRITE_SIZE passes, corrected as MI355X_MICROARCH.md §HBM prescribes (KiB units; FETCH_SIZE
reads half the bytes of wide coalesced loads on gfx950, so it is doubled; WRITE_SIZE is exact
for 16-byte-per-lane streaming stores).  The entry (keyed by the bench line's workload and
ticks per launch) goes into profiles/<round>/<name>/pmc_traffic.json and replaces the same
key in profiles/pmc_traffic.json, which bench.py reads for `roofline.traffic`.

    python tools/pmc_summary.py gpurun_out/<tag>/<name> profiles/<round>/<name>
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    line = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(stats_csv)))
    # the bench line's kernel (its name up to the first " (" note), else the longest in total; a
    # one-off setup kernel (the teacher table's build) can outlast a short timed region
    want = line.get("roofline", {}).get("kernel", "").split(" (")[0].split("<")[0]
    named = [r for r in stats if want and want in r["Name"]]
    name = max(named or stats, key=lambda r: float(r["TotalDurationNs"]))["Name"]
    top = next(r for r in stats if r["Name"] == name)
    # per-launch durations from the trace: the first launch is the warmup's when it ran fewer ticks
    trace_csv = os.path.join(src, "trace", "run_kernel_trace.csv")
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"] == name]
    roof = line["roofline"]
    k = roof.get("ticks_per_launch", 1)
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv"))):
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        per[c] = {kn: (sum(v) / len(v), len(v)) for kn, v in vals.items()}
    fetch_kib, n_f = per["FETCH_SIZE"][name]
    write_kib, n_w = per["WRITE_SIZE"][name]
    entry = {
        "workload": line["config"]["workload"], "ticks_per_launch": k, "kernel": name,
        "rocprof_calls": int(top["Calls"]), "rocprof_avg_us": float(top["AverageNs"]) / 1e3,
        "rocprof_avg_us_after_first": sum(durs[1:]) / max(1, len(durs) - 1),
        "bench_kernel_us": roof.get("kernel_us"), "launches_counted": min(n_f, n_w),
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
        "hbm_write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "algorithmic_bytes_per_launch": roof.get("bytes_per_launch"),
        "correction": "FETCH_SIZE x2 (gfx950 counts half of wide coalesced reads), KiB -> bytes",
    }
    json.dump([entry], open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    topf = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "pmc_traffic.json")
    kept = []
    if os.path.exists(topf):
        old = json.load(open(topf))
        kept = [e for e in (old if isinstance(old, list) else [old])
                if (e.get("workload"), e.get("ticks_per_launch")) != (entry["workload"], k)]
    json.dump(kept + [entry], open(topf, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
