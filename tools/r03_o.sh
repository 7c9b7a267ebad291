#!/bin/bash
# GPU box: fused score + assign parity, pipeline tests; A/B of the fused schedule.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fused or pipeline" --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_o.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "" "--fused-assign --depth 2" "--fused-assign --depth 3" "--fused-assign --depth 3 --resolve-streams 2" "--fused-assign --depth 4 --resolve-streams 2"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), (r.get('isolated') or {}).get('avg_us'), k.get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/ptl && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --fused-assign --depth 3 > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"
python tools/trace_timeline.py /tmp/ptl/run_kernel_trace.csv 120 > gpurun_out/c2fused_timeline.txt
