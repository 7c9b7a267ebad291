#!/bin/bash
# GPU box: per-rank step at N = 1, 2, 4, 8 emulated on one GPU (other shards' bitmaps
# prebuilt, the all-gather replaced by a device copy). Columns: tools/ab_line.py.
set -u
mkdir -p gpurun_out
for w in 1 2 4 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 --emulate-ranks $w > gpurun_out/em.log 2>&1 || { echo "emulate $w failed"; tail -5 gpurun_out/em.log; exit 1; }
  echo "EMU[$w]: $(python tools/ab_line.py gpurun_out/em.log)"
done
