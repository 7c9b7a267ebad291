#!/bin/bash
# GPU box: C2 A/B of --mark-parts (partials ORed by the single-pass scan k_scan_rt) vs default, interleaved.
set -u
mkdir -p gpurun_out
for pass in 1 2 3; do
  for a in "--mark-parts" ""; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 3 $a > gpurun_out/c.log 2>&1 || { echo "failed: $a"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$a]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
