#!/bin/bash
# GPU box: H3 tests, then C2 A/B: look-back scans (k_scan_rt, k_roots_scan_lb) + one
# 8-position local CC launch (new default) vs the round-3 resolve (ROGTK_FUSED_SCAN=0
# ROGTK_LOCAL8_SINGLE=0), interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_gpu_dist_sharded.py tests/test_gpu_bench.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ab4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab4.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export ROGTK_FUSED_SCAN=0 ROGTK_LOCAL8_SINGLE=0; else unset ROGTK_FUSED_SCAN ROGTK_LOCAL8_SINGLE; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
