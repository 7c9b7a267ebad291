#!/bin/bash
# GPU box: k-mer + pack-variant tests, then C3 at 100M reads with the word-parallel pack
# kernel (ROGTK_PACK=4, default) vs the lane-per-row one (3), interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "kmer or c3 or pack or spectr or packed or tight or capacity or group" > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pack.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in 4 3; do
    ROGTK_PACK=$v timeout -k 10 300 python tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 > gpurun_out/kb.log 2>&1 || { echo "bench_kmer $v failed"; tail -5 gpurun_out/kb.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('PACK', sys.argv[2], j['value']/1e6, 'M reads/s', j['phases_ms'])" gpurun_out/kb.log $v
  done
done
