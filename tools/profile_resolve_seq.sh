#!/bin/bash
# GPU box: per-dispatch kernel trace of tools/resolve_bench.py (one n, max_distance 1).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_seq
rm -rf $OUT && mkdir -p $OUT
NS=${NS:-10000000} MDS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 tools/resolve_bench.py > $OUT/log 2>&1 || { echo "rc=$?"; tail -5 $OUT/log; exit 1; }
cat $OUT/log
f=$(find $OUT -name '*kernel_trace.csv' | head -1)
python3 tools/trace_seq.py $f ${LAST:-40} | tee $OUT/seq.txt
