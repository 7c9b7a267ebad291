# Kernel stats of bench.py --emulate-ranks 1 and 8 (tools only; trace pass, no PMC).
set -eu
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/scal_prof; rm -rf $OUT; mkdir -p $OUT
for w in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w$w -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --emulate-ranks $w > $OUT/w$w.log 2>&1
  f=$(find $OUT/w$w -name '*kernel_stats.csv' | head -1)
  echo "== W=$w $(tail -1 $OUT/w$w.log | cut -c1-200)"
  python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:22]: print('%-60s %6s %10.1f' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e3))"
done
