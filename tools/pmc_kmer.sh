#!/bin/bash
# GPU box: PMC passes (one counter group each) over the C3 k-mer bench, k_kmer_lds only.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_kmer
rm -rf $OUT && mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT" "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" "VALUBusy" "SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "k_kmer_lds<1>" -d $OUT/p$i -o run --output-format csv -- python3 tools/bench_kmer.py --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc-ok
