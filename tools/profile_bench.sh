#!/bin/bash
# GPU box: rocprofv3 kernel-trace/stats of bench.py plus separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (they do not fit one pass on gfx950). Stops at the
# first failing step.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_bench
rm -rf $OUT && mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT/bench_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS --no-profile > $OUT/bench_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo profile-ok
