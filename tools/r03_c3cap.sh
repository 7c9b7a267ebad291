#!/bin/bash
# GPU box: k-mer tests with the min_coverage capacity bound, then C3 (100M reads) with
# one spectrum call (default) vs 10M-row calls, interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_c3cap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c3cap.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for br in 100000000 10000000; do
    timeout -k 10 300 python tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 --group-batch-rows $br > gpurun_out/kb.log 2>&1 || { echo "bench_kmer $br failed"; tail -5 gpurun_out/kb.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('batch_rows', sys.argv[2], j['value']/1e6, 'M reads/s', j['phases_ms'], j['config'].get('spectrum_calls'))" gpurun_out/kb.log $br
  done
done
