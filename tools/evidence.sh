#!/bin/bash
# GPU box: a round's closing evidence, in two parts (one gpurun call each).
#   PART=1: smoke(), the GPU tests, the default bench.py line
#   PART=2: the C2 kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile_bench.sh),
#           the C2 stream timeline, a C3 kernel trace, C4 rank-of-8 emulated, C5
# Results under gpurun_out/evidence/; stops at the first failing step. Here afterwards:
#   PART=2 writes the kernel stats + PMC digest (tools/summarize_profiles.py, TAG=<tag>) to
#   gpurun_out/evidence/profiles/; copy what is cited into profiles/
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/evidence
mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
    timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
    rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/smoke.txt; exit $rc; }
    timeout -k 10 600 python3 -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
    rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.log; exit $rc; }
    grep '^{' $O/bench.log | tail -1 > $O/bench.json
else
    # only summaries come back (gpurun_out/ is capped at 64 MiB): the traces are reduced here
    BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-c3 --no-h5 --no-end-to-end" bash tools/profile_bench.sh || exit 1
    python3 tools/trace_chain.py $(find gpurun_out/prof_bench/trace -name '*kernel_trace.csv' | head -1) $O/c2_timeline.json > /dev/null
    echo "timeline rc=$?"
    PROFILES_OUT=$O/profiles python3 tools/summarize_profiles.py ${TAG:-rXX} > $O/summarize.log 2>&1; echo "summarize rc=$?"
    rm -rf gpurun_out/prof_bench
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3trace -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > $O/c3_trace.log 2>&1
    rc=$?; echo "c3 trace rc=$rc"; find $O/c3trace -name '*kernel_trace.csv' -delete; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3k16trace -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --k 15 --min-coverage 5 --steps 2 --warmup 1 > $O/c3k16_trace.log 2>&1
    rc=$?; echo "c3 k16 trace rc=$rc"; find $O/c3k16trace -name '*kernel_trace.csv' -delete; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 240 python3 tools/bench_kmer.py --reads 100000000 --steps 3 --warmup 1 > $O/c3.log 2>&1
    rc=$?; echo "c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python3 tools/bench_kmer.py --reads 100000000 --k 15 --min-coverage 5 --steps 3 --warmup 1 > $O/c3_k16.log 2>&1
    rc=$?; echo "c3 k16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 240 python3 bench.py --workload C4 --emulate-ranks 8 --steps 20 --warmup 3 --no-cpu-baseline --no-h5 > $O/c4_emul8.log 2>&1
    rc=$?; echo "c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 240 python3 bench.py --emulate-ranks 8 --steps 20 --warmup 5 --no-cpu-baseline --no-h5 --no-end-to-end > $O/c2_emul8.log 2>&1
    rc=$?; echo "c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python3 tools/bench_bam.py > $O/c5.log 2>&1
    rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/c5.log; exit $rc; }
fi
echo evidence-ok
