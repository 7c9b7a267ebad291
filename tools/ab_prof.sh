# Kernel stats of bench.py at W=1 for abtmp/old.so vs abtmp/new.so (tools only).
set -eu
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_prof; rm -rf $OUT; mkdir -p $OUT
for v in old new; do
  cp abtmp/$v.so rogtk_amd/librogtk_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --emulate-ranks ${W:-1} > $OUT/$v.log 2>&1
  f=$(find $OUT/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"
  python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
tot=0
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:16]:
  print('  %-44s %6s %9.1f %9.1f' % (x['Name'][:44], x['Calls'], float(x['AverageNs'])/1e3, float(x['TotalDurationNs'])/1e3/23)); tot+=float(x['TotalDurationNs'])
print('  total per step us', round(tot/1e3/23,1))"
done
