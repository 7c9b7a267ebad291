#!/bin/bash
# GPU box: GPU tests; C2 A/B of the second word label (ROGTK_WLAB2); the bench line; C3
# kernel split; a C2 kernel timeline summary; the k_assign counter passes. Raw traces are
# summarised here and deleted (gpurun_out must stay under 64 MiB to come back).
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
for i in 1 2; do
  for v in "" "ROGTK_WLAB2=0"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 0 > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "import json,sys; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(l['ms_per_step'], l['value'], l['roofline']['frac'], l['roofline']['avg_us'], l['roofline']['step']['frac'], l['kernels_us'].get('cluster_assign'))")"
  done
done
timeout -k 10 400 python bench.py > gpurun_out/bench_line.json 2>gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_line.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pc3 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pc3 -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1
echo "prof c3 rc=$?"; cp /tmp/pc3/run_kernel_stats.csv gpurun_out/c3_kernel_stats.csv
rm -rf /tmp/ptl && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ptl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end --sustain-seconds 0 > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"; cp /tmp/ptl/run_kernel_stats.csv gpurun_out/c2_kernel_stats.csv
python tools/trace_split.py /tmp/ptl/run_kernel_trace.csv k_score_packed 3 20 561250000 gpurun_out/c2_score_trace.json > /dev/null
python tools/trace_timeline.py /tmp/ptl/run_kernel_trace.csv 140 > gpurun_out/c2_timeline.txt
tail -1 gpurun_out/prof_tl.log | cut -c1-200 > gpurun_out/c2_prof_bench_line.txt
bash tools/r03_pmc.sh
python tools/pmc_digest.py /tmp/pmcraw gpurun_out/pmc_digest.json
