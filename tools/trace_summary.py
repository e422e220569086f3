"""Per-launch durations of the bench kernel from rocprofv3 kernel traces
(tools/profile.sh), without the first launch of each run (bench.py's
--warmup 5: a 5-tick launch), so the average is over the launches of the timed
tick count only.  usage: python tools/trace_summary.py gpurun_out/<tag> profiles/<round>"""
import csv, json, os, sys

src, dst = sys.argv[1], sys.argv[2]
out = {}
for S, K in ((20, 20), (512, 32)):
    rows = list(csv.DictReader(open(os.path.join(src, f"trace_{S}", "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "rollout" in r["Kernel_Name"]][1:]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
    out[f"steps{S}"] = {"kernel": ks[0]["Kernel_Name"], "ticks_per_launch": K, "launches": len(d),
                        "mean_us": round(sum(d) / len(d), 1), "min_us": round(min(d), 1),
                        "max_us": round(max(d), 1), "us_per_tick": round(sum(d) / len(d) / K, 2)}
json.dump(out, open(os.path.join(dst, "kernel_trace_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
