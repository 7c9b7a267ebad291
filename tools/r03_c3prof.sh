#!/bin/bash
# GPU box: C3 at 100M reads under a kernel + memory-copy trace (where do the copies come from)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/c3prof -o run -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/c3prof.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/c3prof.log | cut -c1-300; exit $rc
