#!/bin/bash
# GPU box: kernel trace/stats of the bench with 4 (then 2) ranks emulated on one GPU (per-rank resolve of the merged bitmap).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in 4 2; do
OUT=gpurun_out/prof_em$w
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --emulate-ranks $w --no-cpu-baseline --no-end-to-end --sustain-seconds 1 --steps 20 > $OUT/bench.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "EMU $w: $(python tools/ab_line.py $OUT/bench.log)"
python3 - $OUT/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:22]:
    n = r["Name"].replace("rogtk::(anonymous namespace)::", "").replace("void ", "")[:60]
    print(f"{n:62s} {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:8.2f} us {float(r['Percentage']):6.2f}%")
PY
done
