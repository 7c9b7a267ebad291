#!/bin/bash
# GPU box: one SQ-counter pass over the C3 k-mer bench (wave-cycle breakdown of the LDS kernels).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_kmer
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $OUT -o run --output-format csv -- python3 tools/bench_kmer.py --steps 1 --warmup 0 > $OUT/log 2>&1 || { echo "rc=$?"; tail -5 $OUT/log; exit 1; }
f=$(find $OUT -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_kmer_lds" not in n:
        continue
    key = n.split("(")[0].split("::")[-1]
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k, {c: round(x / 1e6, 3) for c, x in sorted(v.items())})
PY
rm -rf $OUT/*.csv
