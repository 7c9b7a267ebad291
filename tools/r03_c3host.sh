#!/bin/bash
# GPU box: k-mer tests, then C3 A/B at 100M reads: block-path capacities from staged rows (in classify, 16 lanes per group) +
# device-side path counts (new) vs HEAD (base), interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_c3host.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c3host.log; [ $rc -eq 0 ] || exit $rc
AB_ORDER="base new base new base new" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?
cp tools/kt/new.so rogtk_amd/librogtk_hip.so
exit $rc
