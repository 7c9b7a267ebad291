#!/bin/bash
# Runs on the GPU box: smoke -> gpu tests -> short bench. Stops at the first crash,
# abort or timeout (exit codes other than 0/1); test failures (1) do not stop the bench.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${SMOKE_T:-400} python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 ${TEST_T:-900} python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
