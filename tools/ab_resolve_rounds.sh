# Isolated resolve (tools/resolve_bench.py) under rocprofv3 for abtmp/old.so vs abtmp/new.so;
# prints the per-round median of k_hook_g / k_jump (tools only).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in old new; do
  cp abtmp/$v.so rogtk_amd/librogtk_hip.so
  OUT=gpurun_out/abr_$v; rm -rf $OUT; mkdir -p $OUT
  NS=${NS:-10000000,80000000} timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 tools/resolve_bench.py > $OUT/log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "== $v"; grep -v "^$" $OUT/log | grep -v amdgpu.ids
done
