#!/bin/bash
# GPU box: k-mer (C3) tests, then the C3 bench with block staging vs ASCII staging at 10M
# and 100M reads, then a kernel trace of the 100M block-staged run.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_kmer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for args in "--reads 10000000" "--reads 10000000 --ascii" "--reads 100000000 --steps 3" "--reads 100000000 --steps 3 --ascii"; do
  timeout -k 10 300 python tools/bench_kmer.py $args > gpurun_out/kb.log 2>&1 || { echo "bench_kmer $args failed"; tail -5 gpurun_out/kb.log; exit 1; }
  echo "$args: $(tail -1 gpurun_out/kb.log | cut -c1-600)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_c3 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1
echo "prof rc=$?"
timeout -k 10 200 python tools/host_submit_time.py separate > gpurun_out/host_submit.log 2>&1; echo "host_submit rc=$?"; tail -15 gpurun_out/host_submit.log
rm -rf gpurun_out/prof_tl && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_tl -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-profile --no-cpu-baseline --no-end-to-end > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"
