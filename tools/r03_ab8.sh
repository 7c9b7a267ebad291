#!/bin/bash
# GPU box: C2 A/B of ROGTK_WLAB2=1 (second word label) vs off, with single-exception labels on; interleaved.
set -u
mkdir -p gpurun_out
for pass in 1 2 3; do
  for v in 1 0; do
    ROGTK_WLAB2=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 > gpurun_out/c.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[WLAB2=$v]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
