# Isolated resolve, both H3 global modes, with rocprofv3 kernel stats per mode.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in ${MODES:-2 1}; do
  MODE=$m NS=${NS:-10000000,80000000} MDS=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mode$m -o run -- python3 tools/resolve_bench.py > gpurun_out/resolve_mode$m.log 2>&1 || exit $?
  echo "### mode $m"; grep "n=\|assign" gpurun_out/resolve_mode$m.log
  python3 tools/rocpd_stats.py gpurun_out/prof_mode$m/run_results.db
done
