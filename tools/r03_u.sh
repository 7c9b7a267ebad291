#!/bin/bash
# GPU box: slice-chunk knob tests; interleaved A/B of the slice chunk count.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -x -v -m gpu -k "SLICE_CHUNKS" --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_u.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "" "ROGTK_SLICE_CHUNKS=1" "ROGTK_SLICE_CHUNKS=2" "ROGTK_SLICE_CHUNKS=8"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), k.get('cluster_mark'), k.get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 2; do
rm -rf /tmp/ptl && ROGTK_SLICE_CHUNKS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --settle-seconds 0 > gpurun_out/prof_tl.log 2>&1
echo "stats $v rc=$?"; cp /tmp/ptl/run_kernel_stats.csv gpurun_out/c2_chunks${v}_kernel_stats.csv
done
