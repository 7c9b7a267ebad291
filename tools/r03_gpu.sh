#!/bin/bash
# GPU box, round 3: smoke -> GPU tests -> bench C2 -> bench C4 (N=1) -> rocprof trace + PMC of
# bench C2. Stops at the first crash / abort / timeout (test failures, rc 1, do not stop it).
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
if [ -n "${C4:-1}" ]; then
timeout -k 10 400 python bench.py --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "bench C4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROF:-1}" ]; then
bash tools/profile_bench.sh; rc=$?; echo "profile rc=$rc"
fi
exit $rc
