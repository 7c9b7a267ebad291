#!/usr/bin/env python3
"""Per-step stream timeline of a C2 pipeline run from a rocprofv3 kernel trace.

Usage: trace_chain.py <run_kernel_trace.csv> [out.json]

A step = the interval between two consecutive k_score_packed (or k_score_assign_prev)
starts on the main stream. Per step and stream: busy time (sum of kernel durations),
idle time, kernel count, and the span from the first kernel start to the last kernel end
of the kernels that start in the step. The resolve chain of a batch is the span of the
resolve stream's kernels in the step (the chain starts after the batch's mark). Prints
the medians over the steps of the middle of the run (the first and last 10% dropped).
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name
    for p in ("rogtk::(anonymous namespace)::", "void ", "rogtk::"):
        n = n.replace(p, "")
    return n.split("(")[0].strip()


def main():
    path = sys.argv[1]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), short(r["Kernel_Name"])))
    rows.sort()
    score = [r for r in rows if r[3].startswith("k_score_packed") or r[3].startswith("k_score_assign_prev")]
    if len(score) < 4:
        raise SystemExit("fewer than 4 score launches in the trace")
    main_s = statistics.mode([r[2] for r in score])
    starts = [r[0] for r in score if r[2] == main_s]
    lo, hi = len(starts) // 10, len(starts) - 1 - len(starts) // 10
    per = defaultdict(lambda: defaultdict(list))
    kern = defaultdict(lambda: defaultdict(list))
    offs = defaultdict(lambda: defaultdict(list))  # (start, end) of each launch, us after the step start
    for i in range(lo, hi):
        t0, t1 = starts[i], starts[i + 1]
        by_stream = defaultdict(list)
        for r in rows:
            if t0 <= r[0] < t1:
                by_stream[r[2]].append(r)
        for s, ks in by_stream.items():
            busy = sum(e - b for b, e, _, _ in ks)
            span = max(e for _, e, _, _ in ks) - min(b for b, _, _, _ in ks)
            name = "main" if s == main_s else f"stream{s}"
            per[name]["busy_us"].append(busy / 1e3)
            per[name]["span_us"].append(span / 1e3)
            per[name]["kernels"].append(len(ks))
            seen = defaultdict(int)
            for b, e, _, n in ks:
                kern[name][n].append((e - b) / 1e3)
                offs[name][f"{n}#{seen[n]}"].append(((b - t0) / 1e3, (e - t0) / 1e3))
                seen[n] += 1
        per["step"]["us"].append((t1 - t0) / 1e3)
    med = lambda xs: round(statistics.median(xs), 2)
    out = {"steps": hi - lo, "main_stream": main_s,
           "per_step": {k: {kk: med(vv) for kk, vv in v.items()} for k, v in per.items()},
           "kernels_us": {s: {n: [med(v), len(v) // max(hi - lo, 1)] for n, v in sorted(d.items())}
                          for s, d in kern.items()},
           # median start / end of each launch (n-th of its name in the step) after the step's score start
           "offsets_us": {s: {n: [med([a for a, _ in v]), med([b for _, b in v])] for n, v in
                              sorted(d.items(), key=lambda kv: statistics.median(a for a, _ in kv[1]))}
                          for s, d in offs.items()}}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
