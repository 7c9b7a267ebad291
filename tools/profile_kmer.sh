#!/bin/bash
# GPU box: rocprofv3 kernel trace/stats of the C3 k-mer bench (tools/bench_kmer.py).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_kmer
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/bench_kmer.py ${KARGS:---steps 3} > $OUT/bench.log 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -1 $OUT/bench.log
echo profile-ok
