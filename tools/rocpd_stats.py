"""Per-kernel call count / average / total duration from a rocprofv3 rocpd database."""
import re
import sqlite3
import sys

for path in sys.argv[1:]:
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1000.0 from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    print("##", path)
    for name, n, avg, tot in rows[:24]:
        m = re.search(r"\b(k_\w+(<[^>]*>)?)", name)
        short = m.group(1) if m else name
        print(f"  {short[:44]:44s} calls={n:5d} avg_us={avg:9.1f} total_us={tot:10.1f}")
