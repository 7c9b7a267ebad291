#!/bin/bash
# GPU box: k-mer tests with the read-deduplicating LDS insert, then an interleaved A/B of
# the C3 front end against the previous build at 100M reads.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_kmer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
KARGS="--reads 100000000 --steps 3 --warmup 1" AB_ORDER="base new base new" bash tools/ab_kmer.sh
