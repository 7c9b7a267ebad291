#!/bin/bash
# GPU box: k-mer tests (current build), then C3 A/B at 100M reads:
# base = HEAD, new = per-group flags double-buffered by parity (one barrier fewer per group); interleaved.
set -u
mkdir -p gpurun_out
cp rogtk_amd/librogtk_hip.so tools/kt/cur.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_kmer.py tests/test_gpu_c3.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "kmer or c3 or pack or spectr or packed or tight or capacity or group" > gpurun_out/pytest_units.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_units.log
if [ $rc -eq 0 ]; then AB_ORDER="base new base new base new" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?; fi
cp tools/kt/cur.so rogtk_amd/librogtk_hip.so
exit $rc
