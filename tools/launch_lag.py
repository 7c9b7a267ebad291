"""Host launch vs GPU start for the last kernels of a rocprofv3 run made with
--kernel-trace --hip-runtime-trace: for each dispatch, when the host's launch call
returned, when the kernel started, and the idle gap on its queue before it. A gap with
`late` = yes means the GPU waited for the host (the launch returned after the previous
kernel on the queue had ended).

Usage: python tools/launch_lag.py <run_kernel_trace.csv> <run_hip_api_trace.csv> [last]
"""
import csv
import re
import sys


def main():
    kt = list(csv.DictReader(open(sys.argv[1])))
    api = {r["Correlation_Id"]: r for r in csv.DictReader(open(sys.argv[2]))}
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 80
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    kt = kt[-last:]
    t0 = int(kt[0]["Start_Timestamp"])
    qkey = "Stream_Id" if "Stream_Id" in kt[0] else "Queue_Id"
    prev_end = {}
    late_gap = free_gap = 0.0
    print(f"{'start':>9} {'dur':>7} {'gap':>6} {'launch->start':>13} late q  kernel")
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get(qkey, "?")
        a = api.get(r["Correlation_Id"])
        api_end = int(a["End_Timestamp"]) if a else None
        pe = prev_end.get(q)
        gap = (s - pe) / 1000 if pe is not None else 0.0
        late = api_end is not None and pe is not None and api_end > pe
        if gap > 0:
            if late:
                late_gap += gap
            else:
                free_gap += gap
        m = re.search(r"\b(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        lag = f"{(s - api_end) / 1000:13.1f}" if api_end is not None else f"{'?':>13}"
        print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} {gap:6.1f} {lag} {'yes ' if late else 'no  '}{q:>2} {name[:40]}")
        prev_end[q] = e
    print(f"queue idle before kernels: {late_gap:.1f} us waiting for the host, {free_gap:.1f} us with the launch already queued")


if __name__ == "__main__":
    main()
