#!/bin/bash
# GPU box: pipeline tests, then interleaved C2 bench A/B of the pipeline orders, C3 bench
# with block staging, and a clean kernel timeline of the best order.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -x -q -m gpu -k "pipeline or packed or c3_path" --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in "" "--mark-first" "--mark-first --overlap-score" "--late-assign"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end $v > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "import json,sys; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(l['ms_per_step'], l['value'], l['roofline']['frac'], l['roofline']['avg_us'], l['roofline']['event_avg_us'])")"
  done
done
for args in "--reads 10000000" "--reads 100000000 --steps 3"; do
  timeout -k 10 300 python tools/bench_kmer.py $args > gpurun_out/kb.log 2>&1 || { echo "bench_kmer $args failed"; tail -5 gpurun_out/kb.log; exit 1; }
  echo "KMER $args: $(tail -1 gpurun_out/kb.log | cut -c1-300) ... $(tail -1 gpurun_out/kb.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['phases_ms'])")"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_tl2 && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_tl2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-profile --no-cpu-baseline --no-end-to-end --mark-first > gpurun_out/prof_tl2.log 2>&1
echo "timeline rc=$?"
rm -rf gpurun_out/prof_c3 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1
echo "prof c3 rc=$?"
