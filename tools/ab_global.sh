set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --global-mode rounds > gpurun_out/bench_rounds.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --global-mode uf > gpurun_out/bench_uf.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rounds.log; tail -1 gpurun_out/bench_uf.log
