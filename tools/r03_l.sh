#!/bin/bash
# GPU box: pipeline tests; interleaved A/B of the mark stream and resolve concurrency.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "pipeline" --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "" "--mark-stream" "--mark-stream --depth 3" "--mark-stream --depth 3 --resolve-streams 2"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), r.get('event_avg_us'), l['kernels_us'].get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/ptl && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --mark-stream > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"
python tools/trace_timeline.py /tmp/ptl/run_kernel_trace.csv 140 > gpurun_out/c2ms_timeline.txt
