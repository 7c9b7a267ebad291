#!/bin/bash
# GPU box: kernel trace/stats of the C3 k-mer bench for each library build named in
# AB_PROF (tools/kt/<name>.so, box copy only); prints the k-mer kernels' average times.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${AB_PROF:-base}; do
    cp tools/kt/$v.so rogtk_amd/librogtk_hip.so
    OUT=gpurun_out/abk/$v
    rm -rf $OUT && mkdir -p $OUT
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/bench_kmer.py --steps 3 --warmup 1 > $OUT/bench.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 - $OUT/run_kernel_stats.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
out = []
for r in rows:
    n = r["Name"].replace("rogtk::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if n.startswith(("k_kmer_lds", "k_row_stage", "k_group_classify", "k_class_lists", "k_row_meta")):
        out.append(f"{n}={float(r['AverageNs'])/1000:.0f}us")
print(sys.argv[2], " ".join(out))
PY
done
