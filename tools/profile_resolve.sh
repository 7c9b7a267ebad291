#!/bin/bash
# GPU box: rocprofv3 kernel stats of tools/resolve_bench.py (10M or 80M via NS).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_resolve_${NS:-10000000}
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/resolve_bench.py > $OUT/log 2>&1 || { echo "rc=$?"; exit 1; }
echo ok
