"""Average duration of one kernel in a rocprofv3 kernel trace, over a window of its
launches (e.g. bench.py's timed steps: skip the warmup launches, take --steps), to compare
with bench.py's in-run roofline timing (profiles/<tag>_score_trace.json).

Usage: python tools/trace_split.py <run_kernel_trace.csv> <kernel substring> <skip> <take> [bytes_per_launch] [out.json]
"""
import csv
import json
import sys


def main():
    path, name, skip, take = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    nbytes = float(sys.argv[5]) if len(sys.argv) > 5 else None
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    win = rows[skip:skip + take]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in win]
    out = {"trace": path, "kernel": name, "launches_in_trace": len(rows), "skipped": skip, "window": len(durs),
           "avg_us": round(sum(durs) / max(len(durs), 1), 2), "durations_us": [round(d, 1) for d in durs]}
    if nbytes:
        out["achieved_GBps"] = round(nbytes / (out["avg_us"] * 1e-6) / 1e9, 1)
        out["frac"] = round(out["achieved_GBps"] / 8000.0, 4)
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 6:
        open(sys.argv[6], "w").write(s + "\n")


if __name__ == "__main__":
    main()
