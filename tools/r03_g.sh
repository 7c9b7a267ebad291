#!/bin/bash
# GPU box: all GPU tests, C3 bench + kernel split (block staging), C2 bench (mark-first
# default) + its kernel timeline, then the k_assign counter passes (tools/r03_pmc.sh).
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=12 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -18 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
for args in "--reads 10000000" "--reads 100000000 --steps 3"; do
  timeout -k 10 300 python tools/bench_kmer.py $args > gpurun_out/kb.log 2>&1 || { echo "bench_kmer $args failed"; tail -5 gpurun_out/kb.log; exit 1; }
  echo "KMER $args: $(tail -1 gpurun_out/kb.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['ms_per_step'], l['phases_ms'], l['config']['staging'])")"
done
for i in 1 2; do
  for v in "" "ROGTK_LCC_LOOP=0" "--score-first"; do
    if [ "$v" = "ROGTK_LCC_LOOP=0" ]; then e="ROGTK_LCC_LOOP=0"; a=""; else e=""; a="$v"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 0 $a > gpurun_out/ab.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "AB[$v]: $(python -c "import json,sys; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(l['ms_per_step'], l['value'], l['roofline']['frac'], l['roofline']['avg_us'], l['roofline']['step']['frac'])")"
  done
done
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_c3 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 tools/bench_kmer.py --reads 100000000 --steps 2 --warmup 1 > gpurun_out/prof_c3.log 2>&1
echo "prof c3 rc=$?"
rm -rf gpurun_out/prof_tl && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tl -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/prof_tl.log 2>&1
echo "timeline rc=$?"
bash tools/r03_pmc.sh
