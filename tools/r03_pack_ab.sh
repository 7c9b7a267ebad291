#!/bin/bash
# GPU box: k-mer / C3 / pack tests on the new build (batched staging loads in k_pack_reads),
# then interleaved C3 A/B at 100M reads: base = previous build, new = this build.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "kmer or c3 or pack or spectr or packed or tight or capacity or group" > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pack.log; [ $rc -eq 0 ] || exit $rc
mkdir -p tools/kt && cp tools/ab/base.so tools/kt/base.so && cp tools/ab/new.so tools/kt/new.so
AB_ORDER="base new base new" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?
cp tools/ab/new.so rogtk_amd/librogtk_hip.so
exit $rc
