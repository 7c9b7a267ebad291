#!/bin/bash
# GPU box: interleaved A/B of the H3 global phase with and without the mark stream.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for v in "" "--mark-stream" "--mark-stream --global-mode uf" "--mark-stream --global-mode rounds1f" "--global-mode rounds1f" "--global-mode uf"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "
import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=l['roofline'] or {}; k=l['kernels_us']
print(l['ms_per_step'], round(l['value']/1e9,2), r.get('frac'), r.get('avg_us'), k.get('cluster_assign'), k.get('cluster_union'), k.get('cluster_flatten'), l['sustained']['ms_per_step'])")"
  done
done
