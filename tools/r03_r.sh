#!/bin/bash
# GPU box: C3 pack-kernel variants (ROGTK_PACK), interleaved, 100M reads; block staging
# parity tests under the chosen variants.
set -u
mkdir -p gpurun_out
for v in 1 2 3; do
  ROGTK_PACK=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q -m gpu -k "blocks or packed" --timeout 300 --timeout-method thread > gpurun_out/pytest_r$v.log 2>&1
  rc=$?; echo "pytest PACK=$v rc=$rc"; tail -1 gpurun_out/pytest_r$v.log; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in 0 1 2 3; do
    ROGTK_PACK=$v timeout -k 10 300 python tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 > gpurun_out/kb.log 2>&1 || { echo "PACK=$v failed"; tail -3 gpurun_out/kb.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/kb.log').read().strip().splitlines()[-1]); print('PACK=' + sys.argv[1], round(j['value']/1e6,1), 'M reads/s', j.get('phases_ms'), j.get('pack_ms'))" $v
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 3; do
rm -rf /tmp/pc3 && ROGTK_PACK=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pc3 -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1
echo "prof $v rc=$?"; cp /tmp/pc3/run_kernel_stats.csv gpurun_out/c3_pack${v}_kernel_stats.csv
done
