#!/bin/bash
# GPU box: interleaved A/B of the C3 k-mer front end between two builds of the library
# (tools/kt/base.so, tools/kt/new.so; box copy only). Prints one bench line per run.
set -u
cd "$GRAFT_REPO_ROOT"
for v in ${AB_ORDER:-base new base new}; do
    cp tools/kt/$v.so rogtk_amd/librogtk_hip.so
    timeout -k 10 120 python3 tools/bench_kmer.py ${KARGS:---steps 3 --warmup 1} > gpurun_out/ab_kmer_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value']/1e6, 'M reads/s', j['phases_ms'])" gpurun_out/ab_kmer_$v.log $v
done
