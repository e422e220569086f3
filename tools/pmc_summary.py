"""Summarise a round's rocprofv3 output (tools/profile_round.sh) into
profiles/<round>/: the kernel-trace stats CSVs, and per-launch HBM traffic of the
rollout kernel from the FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md §HBM prescribes (KiB units; FETCH_SIZE reads half the bytes
of wide coalesced loads on gfx950, so it is doubled; WRITE_SIZE is exact for
16-byte-per-lane streaming stores).  One entry per ticks-per-launch (20: the
driver's --steps 20; 32: full launches) in profiles/pmc_traffic.json, which
bench.py reads for `roofline.traffic`.
usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<round> <workload>
       python tools/pmc_summary.py --teacher gpurun_out/<tag> profiles/<round>/config5 <workload>
(--teacher: tools/profile_teacher.sh output, the fused tick + teacher kernel, one tick per
launch).  Entries of other workloads already in profiles/pmc_traffic.json are kept."""
import csv, json, os, shutil, sys
from collections import defaultdict

teacher = sys.argv[1] == "--teacher"
args = sys.argv[2:] if teacher else sys.argv[1:]
src, dst, workload = args[0], args[1], args[2]
os.makedirs(dst, exist_ok=True)
if teacher:
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    runs = [("", 1)]
else:
    for S in (20, 512):
        shutil.copy(os.path.join(src, f"trace_{S}", "run_kernel_stats.csv"),
                    os.path.join(dst, f"kernel_stats_steps{S}.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace_512", "run_kernel_stats.csv"))))
    runs = [("20_", 20), ("128_", 32)]
name = max(stats, key=lambda r: float(r["TotalDurationNs"]))["Name"]
entries = []
for S, K in runs:
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, f"pmc_{S}{c}", "run_counter_collection.csv"))):
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        per[c] = {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}
    fetch_kib, n_f = per["FETCH_SIZE"][name]
    write_kib, n_w = per["WRITE_SIZE"][name]
    entries.append({
        "workload": workload, "ticks_per_launch": K, "kernel": name,
        "launches_counted": min(n_f, n_w),
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
        "hbm_write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "correction": "FETCH_SIZE x2 (gfx950 counts half of wide coalesced reads), KiB -> bytes",
    })
json.dump(entries, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
top = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
kept = []
if os.path.exists(top):
    old = json.load(open(top))
    kept = [e for e in (old if isinstance(old, list) else [old]) if e.get("workload") != workload]
json.dump(kept + entries, open(top, "w"), indent=1)
print(json.dumps(entries, indent=1))
