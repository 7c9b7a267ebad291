#!/bin/bash
# GPU box: k-mer tests under ROGTK_KMER_RUNS=1, then an interleaved C3 A/B at 100M reads.
set -u
mkdir -p gpurun_out
ROGTK_KMER_RUNS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_kmer.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    ROGTK_KMER_RUNS=$v timeout -k 10 300 python tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 > gpurun_out/kb.log 2>&1 || { echo "RUNS=$v failed"; tail -3 gpurun_out/kb.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/kb.log').read().strip().splitlines()[-1]); print('RUNS=' + sys.argv[1], round(j['value']/1e6,1), 'M reads/s', j.get('phases_ms'))" $v
  done
done
