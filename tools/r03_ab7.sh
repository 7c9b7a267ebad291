#!/bin/bash
# GPU box: H3 tests with single-exception word labels, then C2 A/B vs ROGTK_WORD_EXC1=0, interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_gpu_dist_sharded.py tests/test_gpu_bench.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ab7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab7.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in 1 0; do
    ROGTK_WORD_EXC1=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[WORD_EXC1=$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
