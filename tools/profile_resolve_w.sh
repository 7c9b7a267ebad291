#!/bin/bash
# GPU box: kernel stats of tools/resolve_w.py per W (isolated resolve + assign).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_resolve_w
rm -rf $OUT && mkdir -p $OUT
for w in ${WS:-1 8}; do
  WS=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w$w -o run --output-format csv -- python3 tools/resolve_w.py > $OUT/w$w.log 2>&1 || { echo "rc=$?"; tail -5 $OUT/w$w.log; exit 1; }
  grep "^W=" $OUT/w$w.log
  f=$(find $OUT/w$w -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:14]: print('  %-44s %6s %9.1f' % (x['Name'][:44], x['Calls'], float(x['AverageNs'])/1e3))"
done
