#!/bin/bash
# GPU box: H3 tests with the single-pass look-back scan (k_scan_rt), then C2 A/B against
# the three-kernel scan (ROGTK_FUSED_SCAN=0), interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_gpu_dist_sharded.py tests/test_gpu_bench.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ab3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab3.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for fs in 1 0; do
    ROGTK_FUSED_SCAN=$fs timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 > gpurun_out/c.log 2>&1 || { echo "failed: $fs"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[FUSED_SCAN=$fs]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
