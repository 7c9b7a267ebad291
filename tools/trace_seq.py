"""Per-dispatch kernel sequence (name, duration, gap) from a rocprofv3 kernel_trace.csv:
the last `--last` dispatches, to see round-by-round costs of one resolve."""
import csv
import re
import sys

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev_end = None
for r in rows[-last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"\b(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    gap = (s - prev_end) / 1000 if prev_end else 0.0
    print(f"{name[:40]:40s} dur_us={(e - s) / 1000:8.1f} gap_us={gap:7.1f} grid={r.get('Grid_Size', '')}")
    prev_end = e
