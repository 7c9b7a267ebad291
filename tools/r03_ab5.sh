#!/bin/bash
# GPU box: C2 A/B of the resolve-chain variants, interleaved (env knobs).
set -u
mkdir -p gpurun_out
for pass in 1 2 3; do
  for v in "ROGTK_FUSED_SCAN=1 ROGTK_ROOTS_LB=0 ROGTK_LOCAL8_SINGLE=0" "ROGTK_FUSED_SCAN=1 ROGTK_ROOTS_LB=1 ROGTK_LOCAL8_SINGLE=0" "ROGTK_FUSED_SCAN=1 ROGTK_ROOTS_LB=0 ROGTK_LOCAL8_SINGLE=1" "ROGTK_FUSED_SCAN=0 ROGTK_LOCAL8_SINGLE=0"; do
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
