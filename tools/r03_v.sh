#!/bin/bash
# GPU box: mark stream with more hardware queues; slice chunks 8 vs 16.
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in "X=1|" "X=1|--mark-stream" "GPU_MAX_HW_QUEUES=8|--mark-stream" "GPU_MAX_HW_QUEUES=8|" "ROGTK_SLICE_CHUNKS=8|"; do
    e="${v%%|*}"; a="${v#*|}"
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $a > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), k.get('cluster_mark'), k.get('cluster_assign'), l['sustained']['ms_per_step'])")"
  done
done
