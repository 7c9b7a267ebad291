#!/bin/bash
# GPU box: new knob / pipeline tests; interleaved A/B of the assign stream (separate vs
# main) and of the settle phase; a kernel timeline of --assign-on main.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_parity.py -x -q -m gpu -k "pipeline" --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_i.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in "--torch-events" "--assign-on main --torch-events" "" "--assign-on main" "--assign-on main --no-profile"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 --settle-seconds 1 $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), r.get('event_avg_us'), l['kernels_us'].get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/ptl && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --assign-on main --settle-seconds 1 > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"; cp /tmp/ptl/run_kernel_stats.csv gpurun_out/c2mainev_kernel_stats.csv
python tools/trace_timeline.py /tmp/ptl/run_kernel_trace.csv 140 > gpurun_out/c2mainev_timeline.txt
python tools/trace_split.py /tmp/ptl/run_kernel_trace.csv k_score_packed 3 20 561250000 gpurun_out/c2mainev_score_trace.json > /dev/null
grep '^{' gpurun_out/prof_tl.log > gpurun_out/c2mainev_prof_bench_line.json || true
