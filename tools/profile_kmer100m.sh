#!/bin/bash
# GPU box: kernel trace/stats of the C3 k-mer bench at BASELINE config C3's 100M reads.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_kmer100m
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 1 --warmup 1 > $OUT/bench.log 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -1 $OUT/bench.log
python3 - $OUT/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:25]:
    n = r["Name"].replace("rogtk::(anonymous namespace)::", "").replace("void ", "")[:70]
    print(f"{n:72s} {r['Calls']:>5} tot {float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Percentage']}")
PY
