#!/bin/bash
# GPU box: BAM read-ahead (tests + A/B), then the k-mer LDS insert change (tests + A/B at 100M reads).
set -u
mkdir -p gpurun_out
bash tools/r03_bam.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_kmer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "kmer pytest rc=$rc"; tail -3 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || exit $rc
AB_ORDER="base new base new" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?
cp tools/kt/new.so rogtk_amd/librogtk_hip.so
exit $rc
