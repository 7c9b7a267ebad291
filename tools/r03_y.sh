#!/bin/bash
# GPU box: kernel timeline + stats of the emulated 4-rank step (resolve over the union of
# 4 shards' bitmaps).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pem && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pem -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 --settle-seconds 0 --emulate-ranks 4 > gpurun_out/prof_em.log 2>&1
echo "prof rc=$?"; cp /tmp/pem/run_kernel_stats.csv gpurun_out/em4_kernel_stats.csv
python tools/trace_timeline.py /tmp/pem/run_kernel_trace.csv 200 > gpurun_out/em4_timeline.txt
