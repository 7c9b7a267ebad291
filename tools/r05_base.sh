#!/bin/bash
# GPU box: a C2 baseline of the tree as it stands: the default bench line, a kernel trace of
# the pipelined steps reduced to the stream timeline (tools/trace_chain.py, with per-launch
# offsets), and a kernel trace of the resolve alone (tools/resolve_bench.py, 10M reads).
# Results under gpurun_out/base/; stops at the first failing step.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/base
rm -rf $O && mkdir -p $O
if [ "${SKIP_BENCH:-0}" != 1 ]; then
    timeout -k 10 300 python3 bench.py ${BENCH_FULL_ARGS:-} > $O/bench.log 2>&1
    rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.log; exit $rc; }
    grep '^{' $O/bench.log | tail -1 > $O/bench.json
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c3 --no-end-to-end --sustain-seconds 0.3 --settle-seconds 0.5 --iso-launches 0 ${TRACE_ARGS:-} > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.log; exit $rc; }
python3 tools/trace_chain.py $(find $O/trace -name '*kernel_trace.csv' | head -1) $O/c2_timeline.json > /dev/null
echo "timeline rc=$?"
cp $(find $O/trace -name '*kernel_stats.csv' | head -1) $O/c2_kernel_stats.csv
find $O/trace -name '*kernel_trace.csv' -delete
NS=10000000 MDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rtrace -o run --output-format csv -- python3 tools/resolve_bench.py > $O/resolve.log 2>&1
rc=$?; echo "resolve trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/resolve.log; exit $rc; }
cp $(find $O/rtrace -name '*kernel_stats.csv' | head -1) $O/resolve_kernel_stats.csv
find $O/rtrace -name '*kernel_trace.csv' -delete
echo base-ok
