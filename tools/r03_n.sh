#!/bin/bash
# GPU box: does the assign gain from running beside the score kernel? (separate stream,
# no score-alone gate) vs the default (assign on main behind the score kernel)
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in "" "--assign-on separate --overlap-score" "--assign-on separate"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), k.get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/ptl && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --assign-on separate --overlap-score > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"
python tools/trace_timeline.py /tmp/ptl/run_kernel_trace.csv 100 > gpurun_out/c2ov_timeline.txt
