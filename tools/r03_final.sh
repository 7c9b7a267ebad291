#!/bin/bash
# GPU box, end-of-round evidence at HEAD: smoke -> every GPU test -> the default bench
# line -> rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the bench
# -> the C3 front end at 100M reads. Stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
bash tools/gpu_check.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 1" bash tools/profile_bench.sh || exit 1
timeout -k 10 400 python tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 > gpurun_out/kmer100m.log 2>&1; echo "kmer rc=$?"; tail -1 gpurun_out/kmer100m.log | cut -c1-400
