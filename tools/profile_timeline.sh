#!/bin/bash
# GPU box: kernel trace of a short bench.py run; prints the timeline of the last dispatches.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_tl
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} > $OUT/log 2>&1 || { echo "rc=$?"; tail -5 $OUT/log; exit 1; }
tail -1 $OUT/log | cut -c1-200
f=$(find $OUT -name '*kernel_trace.csv' | head -1)
head -1 $f
python3 tools/trace_timeline.py $f ${LAST:-120} > $OUT/timeline.txt
cat $OUT/timeline.txt
