#!/bin/bash
# GPU box: dense-space local tilings vs the oracle, knob test; emulated ranks with and
# without the 16384-code 8-position instance.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -v -m gpu -k "dense or LOCAL8 or sharded_resolve" --timeout 300 --timeout-method thread > gpurun_out/pytest_z.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_z.log; [ $rc -eq 0 ] || exit $rc
for w in 2 4 8; do
  for v in "X=1" "ROGTK_LOCAL8_BIG=0"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 --emulate-ranks $w > gpurun_out/em.log 2>&1 || { echo "emulate $w $v failed"; tail -5 gpurun_out/em.log; exit 1; }
    echo "EMU[$w $v]: $(python tools/ab_line.py gpurun_out/em.log)"
  done
done
