#!/bin/bash
# GPU box: is the resolve chain or the main stream critical? Longer resolve (more
# speculative rounds) vs default, resolve stream at high priority; interleaved, 2 passes.
set -u
mkdir -p gpurun_out
for pass in 1 2; do
  for a in "" "--spec-rounds 5" "--spec-rounds 6" "--prio 0,-1,0" "--spec-rounds 3"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $a > gpurun_out/c.log 2>&1 || { echo "failed: $a"; tail -5 gpurun_out/c.log; exit 1; }
    echo "[$a]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
