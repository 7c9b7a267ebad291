#!/bin/bash
# GPU box: C2 A/B of k_assign launch shapes now that most flagged words need no mask load; interleaved.
set -u
mkdir -p gpurun_out
for pass in 1 2; do
  for v in "ROGTK_ASSIGN_GROUPS=2" "ROGTK_ASSIGN_GROUPS=4" "ROGTK_ASSIGN_BLOCKS=768" "ROGTK_ASSIGN_BLOCKS=0"; do
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
