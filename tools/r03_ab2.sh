#!/bin/bash
# GPU box: tests of the mark partials / BAM read-ahead / flattened k-mer insert, then
# C2 A/B (mark partials ORed by the resolve's scan vs a merge pass) and the C3 k-mer A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py tests/test_bam.py tests/test_gpu_kmer.py tests/test_gpu_c3.py -x -q -m gpu --timeout 200 --timeout-method thread -k "mark_parts or knob or bam or bgzf or kmer or c3 or spectr or streaming or deferred" > gpurun_out/pytest_ab2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab2.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for a in "" "--no-mark-parts"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --sustain-seconds 2 $a > gpurun_out/c.log 2>&1 || { echo "failed: $a"; tail -5 gpurun_out/c.log; exit 1; }
    echo "C2[$a]: $(python tools/ab_line.py gpurun_out/c.log)"
  done
done
cp rogtk_amd/librogtk_hip.so tools/kt/cur.so
AB_ORDER="base flat1 flat2 base flat1 flat2" KARGS="--reads 100000000 --steps 3 --warmup 1" bash tools/ab_kmer.sh; rc=$?
cp tools/kt/cur.so rogtk_amd/librogtk_hip.so
exit $rc
