#!/bin/bash
# GPU box: kernel trace + HIP runtime API trace of a short bench.py run, to line up when
# the host enqueued each kernel with when it ran (no counters in this run).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_api
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} > $OUT/log 2>&1 || { echo "rc=$?"; tail -5 $OUT/log; exit 1; }
ls $OUT
