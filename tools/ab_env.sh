#!/bin/bash
# A/B of bench.py under environment settings: each argument is "VAR=VAL ..." (or "" for none).
set -u
for a in "$@"; do env $a timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }; python -c "import json,sys; j=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(sys.argv[1:], j['ms_per_step'], (j.get('roofline') or {}).get('frac'), j['kernels_us'].get('cluster_assign'), j['kernels_us'].get('cluster_label'))" "$a"; done
