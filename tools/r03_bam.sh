#!/bin/bash
# GPU box: BAM tests, then C5 with and without the BGZF read-ahead thread (interleaved).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bam.py tests/test_gpu_dist_sharded.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bam_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bam_tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for ra in 1 0; do
    ROGTK_BAM_READAHEAD=$ra timeout -k 10 300 python tools/bench_bam.py --no-cpu-baseline > gpurun_out/bam_$ra.json 2> gpurun_out/bam_err.log || { tail -5 gpurun_out/bam_err.log; exit 1; }
    python -c "import json,sys; j=json.load(open(sys.argv[1])); print('READAHEAD=$ra', 'decode', round(j['decode']['records_per_s']/1e6,2), 'M/s', j['decode']['kernels']['host_stages_s'], 'convert', round(j['convert_ipc']['records_per_s']/1e6,2), 'c5', round(j['c5_umi_cluster']['records_per_s']/1e6,2))" gpurun_out/bam_$ra.json
  done
done
