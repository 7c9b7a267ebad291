#!/bin/bash
# GPU box: k-mer tests with class 3 / 1 workgroups of 256 threads, then the C3 A/B at 100M reads
# (tools/kt/base.so: 512 threads, tools/kt/tb256.so), interleaved.
set -u
mkdir -p gpurun_out
cp rogtk_amd/librogtk_hip.so tools/kt/cur.so
cp tools/kt/tb256.so rogtk_amd/librogtk_hip.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_tb.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_tb.log
if [ $rc -eq 0 ]; then AB_ORDER="base tb256 base tb256 base tb256" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?; fi
cp tools/kt/cur.so rogtk_amd/librogtk_hip.so
exit $rc
