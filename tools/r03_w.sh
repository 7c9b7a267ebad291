#!/bin/bash
# GPU box: knob tests for the slice chunk default; interleaved A/B of the assign grid.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -x -v -m gpu -k "SLICE or BUCKET" --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_w.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "X=1" "ROGTK_ASSIGN_BLOCKS=0" "ROGTK_ASSIGN_BLOCKS=1024" "ROGTK_ASSIGN_GROUPS=4" "ROGTK_ASSIGN_BLOCKS=1024 ROGTK_ASSIGN_GROUPS=1"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), k.get('cluster_mark'), k.get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
