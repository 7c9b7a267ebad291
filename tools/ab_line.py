"""One summary line of a bench.py JSON log (the last line of the file): ms/step, G reads/s,
frac, span, H3 distinct / clusters / rounds, per-phase kernel µs, sustained ms/step."""
import json
import sys

lines = open(sys.argv[1]).read().strip().splitlines()
j = json.loads(lines[-1])
r = j.get("roofline") or {}
k = j.get("kernels_us") or {}
c = j.get("config") or {}
print(j["ms_per_step"], round(j["value"] / 1e9, 2), r.get("frac"), r.get("avg_us"), c.get("n_distinct"),
      c.get("n_clusters"), c.get("h3_rounds"), k.get("cluster_mark"), k.get("cluster_union"), k.get("cluster_assign"),
      (j.get("sustained") or {}).get("ms_per_step"))
