#!/bin/bash
# GPU box: pack-variant identity tests + C3 tests at the new default; then the phase split
# of k_kmer_lds (timing build swapped in last: box copy only).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_c3.py -x -q -m gpu -k "pack or c3 or blocks" --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_s.log; [ $rc -eq 0 ] || exit $rc
bash tools/kmer_timing.sh > gpurun_out/kmer_timing.txt 2>&1; echo "timing rc=$?"; tail -10 gpurun_out/kmer_timing.txt
