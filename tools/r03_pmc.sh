#!/bin/bash
# GPU box: counter evidence for k_assign's memory-side traffic.
#  1. the available counters;
#  2. FETCH_SIZE calibration on a known pattern: tools/gather_rate (10M random 4-B gathers
#     from tables of 4 MB .. 1 GB, indices streamed with 16-B loads);
#  3. bench (C2, pipeline) under TCC_HIT/TCC_MISS, TCC_EA0_RDREQ (+ DRAM-side where the
#     counter exists) passes, one counter group per run.
set -u
mkdir -p gpurun_out/pmc /tmp/pmcraw
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1; echo "avail rc=$?"
run() {  # name, counters..., -- cmd
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  rm -rf /tmp/pmcraw/$name
  timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --kernel-trace -d /tmp/pmcraw/$name -o run --output-format csv -- "$@" > gpurun_out/pmc/$name.log 2>&1
  echo "$name rc=$?"
}
run gr_fetch FETCH_SIZE -- ./tools/gather_rate
run gr_hit TCC_HIT_sum TCC_MISS_sum -- ./tools/gather_rate
run gr_req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- ./tools/gather_rate
B="python3 bench.py --steps 6 --warmup 2 --no-profile --no-cpu-baseline --no-end-to-end --sustain-seconds 0"
run b_hit TCC_HIT_sum TCC_MISS_sum -- $B
run b_req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- $B
if grep -q "TCC_EA0_RDREQ_DRAM" gpurun_out/pmc/avail.txt; then
  run b_dram TCC_EA0_RDREQ_DRAM_sum -- $B
  run gr_dram TCC_EA0_RDREQ_DRAM_sum -- ./tools/gather_rate
fi
echo pmc-done
