"""Timeline of the last dispatches of a rocprofv3 kernel_trace.csv: start/end (us, relative),
stream/queue, kernel — to see which pipeline stream bounds a step."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 80
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-last:]
t0 = int(rows[0]["Start_Timestamp"])
qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"\b(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    if "onesweep" in r["Kernel_Name"] or "rocprim" in r["Kernel_Name"]:
        name = "rocprim_sort"
    print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} q={r.get(qkey, '?'):>3} {name[:40]}")
