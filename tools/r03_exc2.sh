#!/bin/bash
# GPU box: H3 tests with two-exception word labels, then C2 A/B: new (one- and two-exception
# forms) vs base (one-exception form only, HEAD), interleaved (library builds in tools/kt).
set -u
mkdir -p gpurun_out
cp tools/kt/new.so rogtk_amd/librogtk_hip.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_gpu_dist_sharded.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_exc2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exc2.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in new base; do
    cp tools/kt/$v.so rogtk_amd/librogtk_hip.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
cp tools/kt/new.so rogtk_amd/librogtk_hip.so
