"""Summarise a round's rocprofv3 output (tools/profile_round.sh) into
profiles/<round>/: the kernel-trace stats CSV, and per-launch HBM traffic of the
tick kernel from the FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md §HBM prescribes (KiB units; FETCH_SIZE reads half the bytes
of wide coalesced loads on gfx950, so it is doubled; WRITE_SIZE is exact for
16-byte-per-lane streaming stores).  Writes profiles/pmc_traffic.json for bench.py.
usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<round> <workload>"""
import csv, json, os, shutil, sys
from collections import defaultdict

src, dst, workload = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv"))):
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    per[c] = {k: sum(v) / len(v) for k, v in vals.items()}
stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
tick = max(stats, key=lambda r: float(r["TotalDurationNs"]))
name = tick["Name"]
fetch_kib = per["FETCH_SIZE"][name]
write_kib = per["WRITE_SIZE"][name]
out = {
    "workload": workload,
    "kernel": name,
    "calls_traced": int(tick["Calls"]),
    "avg_duration_ns": float(tick["AverageNs"]),
    "fetch_size_kib_raw": fetch_kib,
    "write_size_kib_raw": write_kib,
    "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
    "hbm_write_bytes_per_launch": write_kib * 1024,
    "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
    "correction": "FETCH_SIZE x2 (gfx950 counts half of wide coalesced reads), KiB -> bytes",
}
out["hbm_gbs_at_avg_duration"] = out["hbm_bytes_per_launch"] / out["avg_duration_ns"]
json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
json.dump(out, open(os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
