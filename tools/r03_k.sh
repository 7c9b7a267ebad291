#!/bin/bash
# GPU box: host launch vs GPU start (kernel + HIP runtime trace) of the default bench.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/plag && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/plag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 > gpurun_out/prof_lag.log 2>&1
echo "lag rc=$?"; ls /tmp/plag
python tools/launch_lag.py /tmp/plag/run_kernel_trace.csv /tmp/plag/run_hip_api_trace.csv 160 > gpurun_out/launch_lag.txt
tail -1 gpurun_out/launch_lag.txt
grep '^{' gpurun_out/prof_lag.log | cut -c1-200
