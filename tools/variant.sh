#!/bin/bash
# CPU side: an experiment build of librogtk_hip.so as tools/ab/<name>.so (for tools/ab.sh).
#   tools/variant.sh <name> <source.hip[,source2.hip...]> [-DMACRO=value ...]
# Recompiles the listed sources (under rogtk_amd/csrc/) with the extra flags, links them with
# the tree's other objects (make first), and leaves the tree's own library untouched.
set -eu
name=$1; src=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/rogtk_amd/csrc
make -s -j8 -C "$C" >/dev/null
T=$(mktemp -d)
for one in ${src//,/ }; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall \
        -Wno-unused-result -Wno-unused-value "$@" -c "$C/$one" -o "$T/${one%.hip}.o"
done
objs=""
for o in capi umi_kernels cluster_kernels irregular kmer_kernels assembly fastq polars_plugin bam route long_cluster strings dist_cluster; do
    if [ -f "$T/$o.o" ]; then objs="$objs $T/$o.o"; else objs="$objs $C/$o.o"; fi
done
mkdir -p "$ROOT/tools/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/ab/$name.so" $objs -lz -lpthread
rm -rf "$T"
echo "tools/ab/$name.so"
